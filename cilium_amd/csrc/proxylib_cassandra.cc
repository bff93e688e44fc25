// proxylib_cassandra.cc — see proxylib_cassandra.h.
//
// Go slice semantics carry over: a frame is data[0:9+len] of the joined
// input, and a slice expression past the frame's length but within the
// joined input (its capacity) is legal in Go, so a query length reaching into
// the next frame reads that frame's bytes; past the joined input, or an index
// past the frame, is a runtime panic — CassPanic here, PARSER_ERROR in the op
// loop (connection.go:119-135).  Queries are lowered and split as Go does it
// (strings.ToLower / strings.Fields over decoded runes, go_text.h).
#include "proxylib_cassandra.h"

#include <algorithm>
#include <cstring>

#include "go_text.h"

namespace cg {

namespace {

struct CassPanic {};

constexpr int64_t kNop = 256;         // proxylib OpType NOP (types.go:34)
constexpr uint32_t kHdr = 9;          // cassHdrLen
constexpr uint32_t kMaxLen = 1u << 28;  // cassMaxLen, 256 MB

struct Op {
  int64_t op, n;
};

// runtime.roundupsize for a byte slice (Go 1.10 size classes; above 32 KiB
// whole 8 KiB pages)
size_t go_roundupsize(size_t n) {
  static const uint32_t cls[] = {8,    16,   32,    48,    64,    80,    96,    112,   128,   144,   160,   176,
                                 192,  208,  224,   240,   256,   288,   320,   352,   384,   416,   448,   480,
                                 512,  576,  640,   704,   768,   896,   1024,  1152,  1280,  1408,  1536,  1792,
                                 2048, 2304, 2688,  3072,  3200,  3456,  4096,  4864,  5376,  6144,  6528,  6784,
                                 6912, 8192, 9472,  9728,  10240, 10880, 12288, 13568, 14336, 16384, 18432, 19072,
                                 20480, 21760, 24576, 27264, 28672, 32768};
  if (n == 0) return 0;
  for (uint32_t c : cls)
    if (n <= c) return c;
  return (n + 8191) / 8192 * 8192;
}

size_t inject(GoSlice* buf, const void* p, size_t n) {  // connection.go:190-202
  if (!buf || !buf->data) return 0;
  const size_t off = (size_t)buf->len, room = (size_t)(buf->cap - buf->len);
  const size_t k = n < room ? n : room;
  memcpy((char*)buf->data + off, p, k);
  buf->len += (int64_t)k;
  return k;
}

// The joined input (bytes.Join, :174) and the current frame's length: slice
// expressions are bounded by the joined length (the frame's capacity), index
// expressions by the frame's.  bytes.Join of a single slice is an append
// to nil (Go 1.10), whose capacity is rounded up to a malloc size class and
// zeroed: `cap` covers that slack, which reads as zero bytes.
struct Frame {
  const std::string& in;
  size_t len, cap;
  std::string sl(size_t lo, size_t hi) const {
    if (lo > hi || hi > cap) throw CassPanic{};
    std::string s = lo < in.size() ? in.substr(lo, std::min(hi, in.size()) - lo) : std::string();
    s.resize(hi - lo, '\0');
    return s;
  }
  uint8_t at(size_t i) const {
    if (i >= len) throw CassPanic{};
    return (uint8_t)in[i];
  }
  uint32_t be32(size_t lo) const {
    const std::string s = sl(lo, lo + 4);
    return (uint32_t)(uint8_t)s[0] << 24 | (uint32_t)(uint8_t)s[1] << 16 | (uint32_t)(uint8_t)s[2] << 8 |
           (uint8_t)s[3];
  }
  uint16_t be16(size_t lo) const {
    const std::string s = sl(lo, lo + 2);
    return (uint16_t)((uint8_t)s[0] << 8 | (uint8_t)s[1]);
  }
};

const char* opcode_name(uint8_t op) {  // opcodeMap (:285-302)
  switch (op) {
    case 0x00: return "error";
    case 0x01: return "startup";
    case 0x02: return "ready";
    case 0x03: return "authenticate";
    case 0x05: return "options";
    case 0x06: return "supported";
    case 0x07: return "query";
    case 0x08: return "result";
    case 0x09: return "prepare";
    case 0x0A: return "execute";
    case 0x0B: return "register";
    case 0x0C: return "event";
    case 0x0D: return "batch";
    case 0x0E: return "auth_challenge";
    case 0x0F: return "auth_response";
    case 0x10: return "auth_success";
    default: return "";
  }
}

std::string trim_chars(const std::string& s, const char* cut) {  // strings.Trim
  size_t b = 0, e = s.size();
  while (b < e && strchr(cut, s[b])) ++b;
  while (e > b && strchr(cut, s[e - 1])) --e;
  return s.substr(b, e - b);
}

// parseQuery (:344-455): {action, table}, action "" = unparseable.
std::pair<std::string, std::string> parse_query(CassState& st, std::string query) {
  while (!query.empty() && query.back() == ';') query.pop_back();  // TrimRight(query, ";")
  const std::vector<std::string> f = go::fields(go::to_lower(query));  // :373
  for (const std::string& x : f)
    if (x.size() >= 2 && (x.compare(0, 2, "--") == 0 || x.compare(0, 2, "/*") == 0 || x.compare(0, 2, "//") == 0))
      return {"", ""};
  if (f.size() < 2) return {"", ""};
  std::string action = f[0], table;
  if (action == "select" || action == "delete") {
    for (size_t i = 1; i < f.size(); ++i)
      if (f[i] == "from") {
        if (i + 1 >= f.size()) throw CassPanic{};  // fields[i+1]
        table = go::to_lower(f[i + 1]);  // :402
      }
    if (table.empty()) return {"", ""};
  } else if (action == "insert") {
    if (f.size() < 3) return {"", ""};
    table = go::to_lower(f[2]);  // :414
  } else if (action == "update") {
    table = go::to_lower(f[1]);  // :417
  } else if (action == "use") {
    st.keyspace = trim_chars(f[1], "\"\\'");
    table = st.keyspace;
  } else if (action == "alter" || action == "create" || action == "drop" || action == "truncate" ||
             action == "list") {
    action += "-" + f[1];
    if (f[1] == "table" || f[1] == "keyspace") {
      if (f.size() < 3) return {"", ""};
      table = f[2];
      if (table == "if") {
        if (action == "create-table") {
          if (f.size() < 6) return {"", ""};
          table = f[5];  // IF NOT EXISTS
        } else if (action == "drop-table" || action == "drop-keyspace") {
          if (f.size() < 5) return {"", ""};
          table = f[4];  // IF EXISTS
        }
      }
    }
    // (:430-433 compares the already-joined action with "truncate": never true)
    if (f[1] == "materialized") action += "-view";
    else if (f[1] == "custom") action = "create-index";
  } else {
    return {"", ""};
  }
  if (!table.empty() && table.find('.') == std::string::npos && action != "use") table = st.keyspace + "." + table;
  return {action, table};
}

const uint8_t kUnauth[] = {0, 0, 0, 0, 0, 0, 0, 0, 0x1a, 0, 0, 0x21, 0, 0, 0x14, 'R', 'e', 'q', 'u', 'e', 's',
                           't', ' ', 'U', 'n', 'a', 'u', 't', 'h', 'o', 'r', 'i', 'z', 'e', 'd'};
const uint8_t kUnprepared[] = {0, 0, 0, 0, 0, 0, 0, 0, 0x1a, 0, 0, 0x25, 0};

// sendUnpreparedMsg (:580-598)
void send_unprepared(const Frame& d, GoSlice* reply_buf, uint8_t version, const std::string& stream,
                     const std::string& id_short_bytes) {
  uint8_t m[sizeof kUnprepared];
  memcpy(m, kUnprepared, sizeof m);
  m[0] = (uint8_t)(0x80 | (version & 0x07));
  m[2] = (uint8_t)stream[0];
  m[3] = (uint8_t)stream[1];
  inject(reply_buf, m, sizeof m);
  inject(reply_buf, id_short_bytes.data(), id_short_bytes.size());
  (void)d;
}

// cassandraParseRequest (:457-578): error code (0 = ok) and the paths.
int64_t parse_request(CassState& st, const Frame& d, GoSlice* reply_buf, std::vector<std::string>* paths) {
  if (d.at(0) & 0x80) return FILTEROP_ERROR_INVALID_FRAME_TYPE;  // a reply frame
  if (d.at(1) & 0x01) return FILTEROP_ERROR_INVALID_FRAME_TYPE;  // compressed
  const uint8_t opcode = d.at(4);
  std::string path = opcode_name(opcode);
  if (opcode == 0x07 || opcode == 0x09) {  // query, prepare
    const uint64_t qlen = d.be32(9);
    const std::string query = d.sl(13, (size_t)((13 + qlen) & 0xFFFFFFFFull));  // uint32 end index
    auto [action, table] = parse_query(st, query);
    if (action.empty()) return FILTEROP_ERROR_INVALID_FRAME_TYPE;
    path = "/" + path + "/" + action + "/" + table;
    if (opcode == 0x09) {
      // strings.Replace(path, "prepare", "execute", 1)
      std::string ex = path;
      const size_t k = ex.find("prepare");
      if (k != std::string::npos) ex.replace(k, 7, "execute");
      st.by_stream[d.be16(2)] = ex;
    }
    paths->push_back(path);
    return 0;
  }
  if (opcode == 0x0d) {
    // binary.BigEndian.Uint16(data[10:11]) reads index 1 of a one-byte slice
    (void)d.sl(10, 11);
    throw CassPanic{};
  }
  if (opcode == 0x0a) {  // execute
    const size_t idlen = d.be16(9);
    const std::string id = d.sl(11, 11 + idlen);
    auto it = st.by_id.find(id);
    if (it == st.by_id.end() || it->second.empty()) {
      send_unprepared(d, reply_buf, d.at(0), d.sl(2, 4), d.sl(9, 11 + idlen));
      return FILTEROP_ERROR_INVALID_FRAME_TYPE;
    }
    paths->push_back(it->second);
    return 0;
  }
  paths->push_back("/" + path);
  return 0;
}

// cassandraParseReply (:600-642)
void parse_reply(CassState& st, const Frame& d) {
  if ((d.at(0) & 0x80) != 0x80) return;
  if (d.at(1) & 0x01) return;
  const uint16_t stream = d.be16(2);
  if (d.at(4) != 0x08) return;
  if (d.be32(9) != 0x0004) return;  // RESULT kind "prepared"
  const size_t idlen = d.be16(13);
  const std::string id = d.sl(15, 15 + idlen);
  auto it = st.by_stream.find(stream);
  if (it != st.by_stream.end() && !it->second.empty()) st.by_id[id] = it->second;
}

// CassandraParser.OnData (:171-256)
Op on_data(CassState& st, bool reply, const std::string& in, size_t cap, GoSlice* reply_buf,
           const CassMatch& match) {
  if (in.size() < kHdr) return {FILTEROP_MORE, (int64_t)(kHdr - in.size())};
  const uint32_t rlen = (uint32_t)(uint8_t)in[5] << 24 | (uint32_t)(uint8_t)in[6] << 16 |
                        (uint32_t)(uint8_t)in[7] << 8 | (uint8_t)in[8];
  if (rlen > kMaxLen) return {FILTEROP_ERROR, FILTEROP_ERROR_INVALID_FRAME_LENGTH};
  const int64_t total = (int64_t)kHdr + rlen;
  if (total > (int64_t)in.size()) return {FILTEROP_MORE, total - (int64_t)in.size()};
  const Frame d{in, (size_t)total, cap};
  if (reply) {
    parse_reply(st, d);
    return {FILTEROP_PASS, total};
  }
  std::vector<std::string> paths;
  const int64_t err = parse_request(st, d, reply_buf, &paths);
  if (err) return {FILTEROP_ERROR, err};
  bool ok = true;
  for (const std::string& p : paths)  // every path is matched (no short cut)
    if (!match(p)) ok = false;
  if (!ok) {
    uint8_t m[sizeof kUnauth];
    memcpy(m, kUnauth, sizeof m);
    m[0] = (uint8_t)(0x80 | (d.at(0) & 0x07));
    m[2] = d.at(2);
    m[3] = d.at(3);
    inject(reply_buf, m, sizeof m);
    return {FILTEROP_DROP, total};
  }
  return {FILTEROP_PASS, total};
}

}  // namespace

CassFields cassandra_path_fields(const std::string& path) {
  // strings.Split(path, "/") as CassandraRule.Matches splits it (:73-89)
  std::vector<std::string> parts;
  size_t a = 0;
  while (true) {
    const size_t b = path.find('/', a);
    parts.push_back(path.substr(a, b == std::string::npos ? std::string::npos : b - a));
    if (b == std::string::npos) break;
    a = b + 1;
  }
  if (parts.size() <= 2) return {'S', "", ""};
  if (parts.size() < 4) return {'X', "", ""};
  return {'L', parts[2], parts[3]};
}

FilterResult cassandra_on_data(CassState& st, bool reply, bool end_stream, const GoSlice* data, GoSlice* ops,
                               GoSlice* reply_buf, const CassMatch& match) {
  (void)end_stream;
  std::string in;
  const GoSlice* parts = data ? static_cast<const GoSlice*>(data->data) : nullptr;
  for (int64_t i = 0; data && i < data->len; ++i) in.append(static_cast<const char*>(parts[i].data), (size_t)parts[i].len);
  FilterOp* out = static_cast<FilterOp*>(ops->data);
  // the input slices left after advanceInput (connection.go:103-116): their
  // count decides bytes.Join's capacity
  std::vector<size_t> lens;
  for (int64_t i = 0; data && i < data->len; ++i) lens.push_back((size_t)parts[i].len);
  size_t pos = 0;
  try {
    while (ops->len < ops->cap) {
      const std::string rest = in.substr(pos);
      const size_t cap = lens.size() == 1 ? go_roundupsize(rest.size()) : rest.size();
      const Op r = on_data(st, reply, rest, cap, reply_buf, match);
      if (r.op == kNop) break;
      if (r.n == 0) return FILTER_PARSER_ERROR;
      out[ops->len++] = FilterOp{(uint64_t)r.op, r.n};
      if (r.op == FILTEROP_MORE) break;
      if (r.op == FILTEROP_PASS || r.op == FILTEROP_DROP) {
        size_t b = (size_t)r.n;
        pos = std::min(in.size(), pos + b);
        while (b > 0 && !lens.empty()) {
          if (b < lens[0]) {
            lens[0] -= b;
            b = 0;
          } else {
            b -= lens[0];
            lens.erase(lens.begin());
          }
        }
      }
    }
  } catch (const CassPanic&) {
    return FILTER_PARSER_ERROR;
  }
  return FILTER_OK;
}

}  // namespace cg
