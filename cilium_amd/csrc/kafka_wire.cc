// kafka_wire.cc — the host Kafka request decoder (kafka_wire.h) and the
// cg_kafka_decode_host / cg_kafka_verdicts_raw_host entry points.
//
// The host finishes what the GPU decoder cannot: gzip and snappy message
// payloads (compress/gzip multistream members, golang/snappy blocks and the
// xerial framing of proto/snappy.go:23-50), whose inner message sets it
// parses with the same kw_message_set.
#include "kafka_wire.h"

#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "engine.h"
#include "kafka.h"

namespace cg {

namespace {

// CRC-32 (IEEE) of a message: zlib's, the same polynomial as hash/crc32
struct HostCrc {
  uint32_t operator()(const uint8_t* p, uint32_t n) const { return (uint32_t)crc32(0, p, n); }
};

// compress/gzip Reader + ioutil.ReadAll (Go 1.10): members back to back; a
// clean end of input before a header ends the stream.
bool gunzip_go(const uint8_t* b, size_t n, std::vector<uint8_t>* out) {
  size_t pos = 0;
  bool first = true;
  for (;;) {
    if (pos == n && !first) return true;
    if (n - pos < 10) return false;
    const uint8_t* h = b + pos;
    if (h[0] != 0x1F || h[1] != 0x8B || h[2] != 8) return false;
    const uint8_t flg = h[3];
    size_t q = pos + 10;
    if (flg & 4) {  // FEXTRA
      if (q + 2 > n) return false;
      q += 2 + (size_t)(b[q] | b[q + 1] << 8);
      if (q > n) return false;
    }
    for (uint8_t bit : {8, 16}) {  // FNAME, FCOMMENT: NUL-terminated within 512 bytes
      if (!(flg & bit)) continue;
      const size_t lim = std::min(n, q + 512);
      size_t z = q;
      while (z < lim && b[z] != 0) ++z;
      if (z >= lim) return false;
      q = z + 1;
    }
    if (flg & 2) {  // FHCRC
      if (q + 2 > n) return false;
      if ((crc32(0, b + pos, (uInt)(q - pos)) & 0xFFFF) != (uint32_t)(b[q] | b[q + 1] << 8)) return false;
      q += 2;
    }
    z_stream zs{};
    if (inflateInit2(&zs, -15) != Z_OK) return false;
    zs.next_in = const_cast<Bytef*>(b + q);
    zs.avail_in = (uInt)(n - q);
    const size_t start = out->size();
    int rc = Z_OK;
    while (rc == Z_OK) {
      // readMessageSet rejects a decoded set above maxParseBufSize: stop there
      if (out->size() > (size_t)kKafkaMaxParseBuf) {
        inflateEnd(&zs);
        return false;
      }
      const size_t at = out->size();
      out->resize(at + 65536);
      zs.next_out = out->data() + at;
      zs.avail_out = 65536;
      rc = inflate(&zs, Z_NO_FLUSH);
      out->resize(at + 65536 - zs.avail_out);
      if (rc == Z_BUF_ERROR && zs.avail_in == 0) break;  // input ended inside the stream
      if (rc == Z_BUF_ERROR) rc = Z_OK;
    }
    const size_t used = (n - q) - zs.avail_in;
    inflateEnd(&zs);
    if (rc != Z_STREAM_END) return false;
    q += used;
    if (q + 8 > n) return false;
    const uint32_t crc = (uint32_t)(b[q] | b[q + 1] << 8 | b[q + 2] << 16 | (uint32_t)b[q + 3] << 24);
    const uint32_t isize = (uint32_t)(b[q + 4] | b[q + 5] << 8 | b[q + 6] << 16 | (uint32_t)b[q + 7] << 24);
    const uint32_t got = (uint32_t)crc32(0, out->data() + start, (uInt)(out->size() - start));
    if (crc != got || isize != (uint32_t)(out->size() - start)) return false;
    pos = q + 8;
    first = false;
  }
}

// golang/snappy Decode (decode.go, decode_other.go): one block.
bool snappy_block(const uint8_t* src, size_t n, std::vector<uint8_t>* out) {
  uint64_t v = 0;
  size_t s = 0;
  for (int shift = 0;; shift += 7, ++s) {  // binary.Uvarint
    if (s >= n || s == 10) return false;
    const uint8_t c = src[s];
    if (c < 0x80) {
      if (s == 9 && c > 1) return false;
      v |= (uint64_t)c << shift;
      ++s;
      break;
    }
    v |= (uint64_t)(c & 0x7F) << shift;
  }
  if (v > 0xFFFFFFFFull) return false;
  // readMessageSet rejects a decoded set above maxParseBufSize, so a longer
  // block is an error whatever its content
  if (out->size() + v > (size_t)kKafkaMaxParseBuf) return false;
  const size_t base = out->size();
  out->resize(base + v);
  uint8_t* dst = out->data() + base;
  size_t d = 0;
  while (s < n) {
    size_t length, offset;
    switch (src[s] & 3) {
      case 0: {
        uint32_t x = src[s] >> 2;
        if (x < 60) {
          s += 1;
        } else {
          const size_t k = x - 59;
          s += 1 + k;
          if (s > n) return false;
          x = 0;
          for (size_t i = 0; i < k; ++i) x |= (uint32_t)src[s - k + i] << (8 * i);
        }
        length = (size_t)x + 1;
        if (length > v - d || length > n - s) return false;
        memcpy(dst + d, src + s, length);
        d += length;
        s += length;
        continue;
      }
      case 1:
        s += 2;
        if (s > n) return false;
        length = 4 + ((src[s - 2] >> 2) & 7);
        offset = (size_t)((src[s - 2] & 0xE0) << 3 | src[s - 1]);
        break;
      case 2:
        s += 3;
        if (s > n) return false;
        length = 1 + (src[s - 3] >> 2);
        offset = (size_t)(src[s - 2] | src[s - 1] << 8);
        break;
      default:
        s += 5;
        if (s > n) return false;
        length = 1 + (src[s - 5] >> 2);
        offset = (size_t)src[s - 4] | (size_t)src[s - 3] << 8 | (size_t)src[s - 2] << 16 | (size_t)src[s - 1] << 24;
    }
    if (offset == 0 || d < offset || length > v - d) return false;
    for (size_t end = d + length; d != end; ++d) dst[d] = dst[d - offset];
  }
  return d == v;
}

const uint8_t kSnappyJavaMagic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};

bool snappy_go(const uint8_t* b, size_t n, std::vector<uint8_t>* out) {
  if (n < 8 || memcmp(b, kSnappyJavaMagic, 8) != 0) return snappy_block(b, n, out);
  // xerial framing (a truncated frame panics in Go; an error here)
  if (n < 16) return false;
  if ((uint32_t)(b[8] << 24 | b[9] << 16 | b[10] << 8 | b[11]) != 1) return false;
  for (size_t i = 16; i < n;) {
    if (i + 4 > n) return false;
    const size_t k = (size_t)b[i] << 24 | (size_t)b[i + 1] << 16 | (size_t)b[i + 2] << 8 | b[i + 3];
    i += 4;
    if (i + k > n) return false;
    if (!snappy_block(b + i, k, out)) return false;
    i += k;
  }
  return true;
}

// The host's Inflate for kw_message_set: decompress, then parse the inner set.
// Intended deviations from readMessageSet (messages.go:363-500), which
// recurses without a depth limit: at most kMaxDepth nested compressed sets,
// and at most kBudget decoded bytes alive across the nesting levels of one
// request (each level keeps its buffer while the inner set parses; Go bounds
// only each level, at maxParseBufSize).  Past either bound the request is a
// decode error (the connection closes) where Go would keep parsing.  KAT:
// tests/test_kafka_wire.py test_nested_compression_bounds.
struct HostInflate {
  static constexpr int kMaxDepth = 64;
  static constexpr size_t kBudget = (size_t)64 << 20;
  int depth = 0;
  size_t* left = nullptr;  // decoded-byte budget shared by the levels
  uint8_t operator()(uint32_t codec, const uint8_t* p, uint32_t n, int16_t version) {
    if (depth >= kMaxDepth) return kKwError;  // stack guard
    size_t own = kBudget;
    size_t* budget = left ? left : &own;
    std::vector<uint8_t> dec;
    if (!(codec == 1 ? gunzip_go(p, n, &dec) : snappy_go(p, n, &dec))) return kKwError;
    if (dec.size() > *budget) return kKwError;
    *budget -= dec.size();
    KwStream inner{dec.data(), (uint32_t)dec.size(), 0};
    HostInflate next{depth + 1, budget};
    const uint8_t rc = kw_message_set(&inner, (int32_t)dec.size(), version, HostCrc{}, next);
    *budget += dec.size();  // this level's buffer goes with the return
    return rc;
  }
};

uint32_t intern(const std::unordered_map<std::string, uint32_t>& m, const uint8_t* p, uint32_t n) {
  auto it = m.find(std::string((const char*)p, n));
  return it == m.end() ? CG_KAFKA_UNKNOWN_STR : it->second;
}

}  // namespace

// One request decoded on the host into its record (topics beyond
// CG_KAFKA_MAX_TOPICS appended to `spill`); returns the status.
uint8_t kafka_decode_host_one(const KafkaSnapshot& s, const uint8_t* raw, uint64_t len, uint16_t redirect,
                              uint32_t remote, cg_kafka_request* q, std::vector<uint32_t>* spill) {
  memset(q, 0, sizeof(*q));
  q->policy = redirect;
  q->remote = remote;
  KwRequest r;
  std::vector<uint32_t> topics;
  HostInflate inflate;
  const uint32_t l32 = len > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len;
  struct Sink {
    const KafkaSnapshot& s;
    const uint8_t* raw;
    std::vector<uint32_t>& topics;
    void begin(int32_t) {}
    void topic(uint32_t off, uint32_t n) { topics.push_back(intern(s.topic_ids, raw + off, n)); }
  } sink{s, raw, topics};
  const uint8_t st = kw_decode(raw, l32, HostCrc{}, &r, sink, inflate);
  if (st != kKwOk) {
    // ReadRequest failed: the connection closes; the record can only be denied
    q->policy = 0xFFFF;
    q->kind = CG_KAFKA_K_NIL;
    return kKwError;
  }
  q->api_key = r.api_key;
  q->api_version = r.version;
  q->kind = r.cls;
  q->client_id = intern(s.client_ids, raw + r.client_off, r.client_len);
  q->n_topics = (uint8_t)std::min<size_t>(topics.size(), CG_KAFKA_TOPICS_IN_ARENA);
  if (topics.size() <= CG_KAFKA_MAX_TOPICS) {
    for (size_t i = 0; i < topics.size(); ++i) q->topic_ids[i] = topics[i];
  } else {
    q->topic_ids[0] = (uint32_t)spill->size();
    if (topics.size() >= CG_KAFKA_TOPICS_IN_ARENA) q->topic_ids[1] = (uint32_t)topics.size();
    spill->insert(spill->end(), topics.begin(), topics.end());
  }
  return kKwOk;
}

}  // namespace cg
