// proxylib_memcache.cc — see proxylib_memcache.h.  Go's runtime panics in
// these parsers (an index past a slice, e.g. a request line with too few
// tokens) are the McPanic exception, turned into PARSER_ERROR by the op loop
// as connection.go:124-136 recovers them.
#include "proxylib_memcache.h"

#include <cstring>
#include <string_view>

#include "go_text.h"

namespace cg {

const char kMcTextDenied[] = "CLIENT_ERROR access denied\r\n";
const uint8_t kMcBinaryDenied[37] = {0x81, 0, 0, 0, 0, 0, 0, 8, 0, 0, 0, 0x0d, 0, 0, 0, 0, 0, 0, 0,
                                     0,    0, 0, 0, 0, 'a', 'c', 'c', 'e', 's', 's', ' ', 'd', 'e', 'n', 'i', 'e', 'd'};

namespace {

struct McPanic {};

constexpr int64_t kNop = 256;  // proxylib OpType NOP (types.go:34)

using Input = std::vector<std::string_view>;

struct Op {
  int64_t op, n;
};

// connection.Inject: append what fits (connection.go:190-202)
size_t inject(GoSlice* buf, const void* p, size_t n) {
  if (!buf || !buf->data) return 0;
  const size_t off = (size_t)buf->len, room = (size_t)(buf->cap - buf->len);
  const size_t k = n < room ? n : room;
  memcpy((char*)buf->data + off, p, k);
  buf->len += (int64_t)k;
  return k;
}
bool inject_full(const GoSlice* buf) { return !buf || buf->len == buf->cap; }

std::string join(const Input& in) {
  std::string s;
  for (auto v : in) s.append(v.data(), v.size());
  return s;
}

using go::fields;  // bytes.Fields over decoded runes (go_text.h)

bool has_prefix(const std::string& s, const char* p) { return s.compare(0, strlen(p), p) == 0; }

// strconv.Atoi (64-bit int): optional sign, decimal digits, in range
bool atoi_go(const std::string& s, int64_t* v) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i >= s.size()) return false;
  uint64_t x = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    const uint64_t d = (uint64_t)(s[i] - '0');
    if (x > (UINT64_MAX - d) / 10) return false;
    x = x * 10 + d;
  }
  if (neg ? x > (uint64_t)INT64_MAX + 1 : x > (uint64_t)INT64_MAX) return false;
  *v = neg ? (int64_t)(0 - x) : (int64_t)x;
  return true;
}

template <class T>
const T& at(const std::vector<T>& v, size_t i) {
  if (i >= v.size()) throw McPanic{};
  return v[i];
}

// ---- text protocol (text/parser.go)
bool is_retrieval(const std::string& c) { return has_prefix(c, "get") || has_prefix(c, "gat"); }
bool is_storage(const std::string& c) {
  return c == "set" || c == "add" || c == "replace" || c == "append" || c == "prepend" || c == "cas";
}
bool is_incr_decr(const std::string& c) { return c == "incr" || c == "decr"; }
bool is_error_reply(const std::string& t) { return t == "ERROR" || t == "CLIENT_ERROR" || t == "SERVER_ERROR"; }

Op text_until_end(const std::string& data) {
  const size_t e = data.find("\r\nEND\r\n");
  if (e != std::string::npos && e > 0) return {FILTEROP_PASS, (int64_t)e + 7};
  return {FILTEROP_MORE, 1};
}

int64_t text_inject_from_queue(McState& st, GoSlice* reply_buf) {
  int64_t injected = 0;
  while (!st.text_queue.empty() && st.text_queue.front().second) {
    inject(reply_buf, kMcTextDenied, sizeof(kMcTextDenied) - 1);
    st.text_queue.pop_front();
    ++injected;
  }
  return injected * (int64_t)(sizeof(kMcTextDenied) - 1);
}

Op text_on_data(McState& st, bool reply, const Input& in, GoSlice* reply_buf, const McMatch& match) {
  if (reply) {
    const int64_t injected = text_inject_from_queue(st, reply_buf);
    if (injected > 0) return {FILTEROP_INJECT, injected};
    if (in.empty()) return {kNop, 0};
  }
  const std::string data = join(in);
  const size_t lf = data.find("\r\n");
  if (lf == std::string::npos) return {FILTEROP_MORE, !data.empty() && data.back() == '\r' ? 1 : 2};
  const std::vector<std::string> tokens = fields(std::string_view(data).substr(0, lf));
  if (!reply) {
    McMeta meta;
    const std::string& command = at(tokens, 0);
    meta.command = command;
    int64_t frame = (int64_t)lf + 2;
    bool noreply = false;
    auto keys_from = [&](size_t lo, size_t hi) {  // tokens[lo:hi] (Go slice bounds: lo <= hi <= len)
      if (lo > hi || hi > tokens.size()) throw McPanic{};
      meta.keys.assign(tokens.begin() + (long)lo, tokens.begin() + (long)hi);
    };
    if (is_retrieval(command)) {
      if (has_prefix(command, "get")) keys_from(1, tokens.size());
      else keys_from(2, tokens.size());
    } else if (is_storage(command)) {
      keys_from(1, 2);
      int64_t nbytes = 0;
      if (!atoi_go(at(tokens, 4), &nbytes)) return {FILTEROP_ERROR, 0};
      frame = (int64_t)((uint64_t)frame + (uint64_t)nbytes + 2u);  // Go int arithmetic wraps
      noreply = tokens.size() == (command[0] == 'c' ? 7u : 6u);
    } else if (command == "delete") {
      keys_from(1, 2);
      noreply = tokens.size() == 3;
    } else if (is_incr_decr(command)) {
      keys_from(1, 2);
      noreply = tokens.size() == 4;
    } else if (command == "touch") {
      keys_from(1, 2);
      noreply = tokens.size() == 4;
    } else if (command == "slabs" || command == "lru" || command == "lru_crawler" || command == "stats" ||
               command == "version" || command == "misbehave") {
    } else if (command == "flush_all" || command == "cache_memlimit") {
      noreply = tokens.back() == "noreply";
    } else if (command == "quit") {
      noreply = true;
    } else if (command == "watch") {
      st.watching = true;
    } else {
      return {FILTEROP_ERROR, 0};
    }
    if (match(meta)) {
      if (!noreply) st.text_queue.push_back({command, false});
      return {FILTEROP_PASS, frame};
    }
    if (!noreply) {
      if (st.text_queue.empty()) inject(reply_buf, kMcTextDenied, sizeof(kMcTextDenied) - 1);
      else st.text_queue.push_back({command, true});
    }
    return {FILTEROP_DROP, frame};
  }
  // reply
  if (st.text_queue.empty()) throw McPanic{};
  const std::string intent = st.text_queue.front().first;
  if (st.watching) return {FILTEROP_PASS, (int64_t)lf + 2};
  if (is_error_reply(at(tokens, 0)) || is_storage(intent) || intent == "delete" || is_incr_decr(intent) ||
      intent == "touch" || intent == "slabs" || intent == "lru" || intent == "flush_all" ||
      intent == "cache_memlimit" || intent == "version" || intent == "misbehave") {
    st.text_queue.pop_front();
    return {FILTEROP_PASS, (int64_t)lf + 2};
  }
  if (is_retrieval(intent) || intent == "stats") {
    const Op r = text_until_end(data);
    if (r.op == FILTEROP_PASS) st.text_queue.pop_front();
    return r;
  }
  if (intent == "lru_crawler") {
    if (tokens[0] == "OK" || tokens[0] == "BUSY" || tokens[0] == "BADCLASS") {
      st.text_queue.pop_front();
      return {FILTEROP_PASS, (int64_t)lf + 2};
    }
    const Op r = text_until_end(data);
    if (r.op == FILTEROP_PASS) st.text_queue.pop_front();
    return r;
  }
  return {FILTEROP_ERROR, 0};
}

// ---- binary protocol (binary/parser.go)
void bin_inject_denied(McState& st, uint8_t magic, GoSlice* reply_buf) {
  uint8_t msg[sizeof(kMcBinaryDenied)];
  memcpy(msg, kMcBinaryDenied, sizeof msg);
  msg[0] = magic;
  inject(reply_buf, msg, sizeof msg);
  ++st.replies;
}

Op bin_on_data(McState& st, bool reply, const Input& in, GoSlice* reply_buf, const McMatch& match) {
  if (reply) {
    if (!st.bin_queue.empty() && st.bin_queue.front().second == st.replies + 1) {
      bin_inject_denied(st, st.bin_queue.front().first, reply_buf);
      st.bin_queue.pop_front();
      return {FILTEROP_INJECT, (int64_t)sizeof(kMcBinaryDenied)};
    }
    if (in.empty()) return {kNop, 0};
  }
  const std::string data = join(in);
  const uint8_t* d = (const uint8_t*)data.data();
  if (data.size() < 24) return {FILTEROP_MORE, (int64_t)(24 - data.size())};
  const uint32_t body = (uint32_t)d[8] << 24 | (uint32_t)d[9] << 16 | (uint32_t)d[10] << 8 | d[11];
  const uint32_t keylen = (uint32_t)d[2] << 8 | d[3];
  const uint32_t extras = d[4];
  if (keylen > 0) {
    const size_t need = 24 + keylen + extras;
    if (need > data.size()) return {FILTEROP_MORE, (int64_t)(need - data.size())};
  }
  if ((d[0] & 0x80) != 0x80) return {FILTEROP_ERROR, FILTEROP_ERROR_INVALID_FRAME_TYPE};
  const uint8_t opcode = d[1];
  const int64_t frame = (int64_t)(uint32_t)(body + 24u);  // int(bodyLength + headerSize): uint32 sum
  if (reply) {
    ++st.replies;
    return {FILTEROP_PASS, frame};
  }
  ++st.requests;
  McMeta meta;
  meta.opcode = opcode;
  meta.keys.push_back(keylen ? data.substr(24 + extras, keylen) : std::string());
  if (match(meta)) return {FILTEROP_PASS, frame};
  const uint8_t magic = 0x81 | d[0];
  if (st.requests == st.replies + 1) bin_inject_denied(st, magic, reply_buf);
  else st.bin_queue.push_back({magic, st.requests});
  st.bin_queue.push_back({magic, st.requests});  // queued in both cases, as the reference does
  return {FILTEROP_DROP, frame};
}

// memcached/parser.go:176-199
Op mc_on_data(McState& st, bool reply, const Input& in, GoSlice* reply_buf, const McMatch& match) {
  if (st.mode == 0) {
    if (in.empty() || in[0].empty()) return {kNop, 0};
    st.mode = (uint8_t)in[0][0] >= 128 ? 2 : 1;
  }
  return st.mode == 2 ? bin_on_data(st, reply, in, reply_buf, match) : text_on_data(st, reply, in, reply_buf, match);
}

}  // namespace

FilterResult memcache_on_data(McState& st, bool reply, bool end_stream, const GoSlice* data, GoSlice* ops,
                              GoSlice* reply_buf, const McMatch& match) {
  (void)end_stream;
  Input in;
  const GoSlice* parts = data ? static_cast<const GoSlice*>(data->data) : nullptr;
  for (int64_t i = 0; data && i < data->len; ++i)
    in.emplace_back(static_cast<const char*>(parts[i].data), (size_t)parts[i].len);
  FilterOp* out = static_cast<FilterOp*>(ops->data);
  try {
    while (ops->len < ops->cap) {
      const Op r = mc_on_data(st, reply, in, reply_buf, match);
      if (r.op == kNop) break;
      if (r.n == 0) return FILTER_PARSER_ERROR;
      out[ops->len++] = FilterOp{(uint64_t)r.op, r.n};
      if (r.op == FILTEROP_MORE) break;
      if (r.op == FILTEROP_PASS || r.op == FILTEROP_DROP) {
        // advanceInput (connection.go:103-116)
        int64_t b = r.n;
        while (b > 0 && !in.empty()) {
          const int64_t rem = (int64_t)in[0].size();
          if (b < rem) {
            in[0] = in[0].substr((size_t)b);
            b = 0;
          } else {
            b -= rem;
            in.erase(in.begin());
          }
        }
      }
      if (r.op == FILTEROP_INJECT && inject_full(reply ? reply_buf : nullptr)) break;
    }
  } catch (const McPanic&) {
    return FILTER_PARSER_ERROR;
  }
  return FILTER_OK;
}

}  // namespace cg
