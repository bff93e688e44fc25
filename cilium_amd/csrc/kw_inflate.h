// kw_inflate.h — the compressed Kafka message payloads, decoded where the
// request is decoded: one lane per request on the GPU (kernels_kafka.hip), or
// the host (tests/test_kw_inflate.py drives the same code on the CPU).
//
// A message whose attributes name codec 1 or 2 carries a compressed inner
// message set (optiopay proto/messages.go:460-480): gzip through Go's
// compress/gzip (RFC 1952 members of RFC 1951 DEFLATE data) or snappy through
// golang/snappy (a raw block, or the xerial framing of proto/snappy.go:23-50).
// The host decoder (kafka_wire.cc) restates those with zlib's inflate and a
// snappy restatement; this header decodes the same formats into a bounded
// caller buffer with the same outcomes:
//   gzip   one member: header (FEXTRA / FNAME / FCOMMENT / FHCRC), DEFLATE
//          (stored, fixed and dynamic blocks; the code checks zlib applies —
//          over-subscribed or incomplete codes, a missing end-of-block code,
//          lengths 286/287 and distances 30/31, distances past the output),
//          trailer CRC-32 and ISIZE.  A second member (input left after the
//          first) returns kKwzMore: the caller hands the request to the host.
//   snappy the varint length, literals and copies as golang/snappy's decode
//          (decode_other.go), and the xerial chunks.
// The DEFLATE decoder reads codes bit by bit over canonical code counts
// (RFC 1951 3.2.2): small per-lane state (two tables of 16 counts and <= 288
// symbols), no lookup tables to build in LDS — compressed message sets are a
// small share of a batch's requests.
#pragma once

#include <cstdint>

#include "dev_types.h"

namespace cg {
namespace kwz {

constexpr int kKwzOk = 0;
constexpr int kKwzError = 1;
// the host decodes it: gzip input continues past the first member, or the
// output passes the caller's buffer (sized from ISIZE / the snappy lengths,
// which the data may contradict: the host then reports the error)
constexpr int kKwzMore = 2;

struct Bits {
  const uint8_t* p;
  uint32_t n, pos, buf, cnt;
  bool err;
  CG_HD uint32_t get(uint32_t need) {  // need <= 16
    while (cnt < need) {
      if (pos >= n) {
        err = true;
        return 0;
      }
      buf |= (uint32_t)p[pos++] << cnt;
      cnt += 8;
    }
    const uint32_t v = buf & ((1u << need) - 1u);
    buf >>= need;
    cnt -= need;
    return v;
  }
  // the next `need` (<= 16) bits without consuming them; bits past the input
  // read as 0 (drop() then fails if a code needs them)
  CG_HD uint32_t peek(uint32_t need) {
    while (cnt < need && pos < n) {
      buf |= (uint32_t)p[pos++] << cnt;
      cnt += 8;
    }
    return buf & ((1u << need) - 1u);
  }
  CG_HD void drop(uint32_t k) {
    if (k > cnt) {
      err = true;
      return;
    }
    buf >>= k;
    cnt -= k;
  }
};

// A canonical code: count[l] codes of length l, symbols in code order.
struct Huff {
  uint16_t count[16];
  uint16_t sym[288];
  uint16_t maxlen;
};

// Build from code lengths len[0, n); returns the unused code space: 0 for a
// complete code, > 0 incomplete, < 0 over-subscribed.
CG_HD inline int huff_build(Huff& h, const uint8_t* len, int n) {
  for (int l = 0; l < 16; ++l) h.count[l] = 0;
  for (int s = 0; s < n; ++s) h.count[len[s]]++;
  h.maxlen = 0;
  for (int l = 15; l >= 1; --l)
    if (h.count[l]) {
      h.maxlen = (uint16_t)l;
      break;
    }
  int left = 1;
  for (int l = 1; l < 16; ++l) {
    left <<= 1;
    left -= h.count[l];
    if (left < 0) return left;
  }
  uint16_t offs[16];
  offs[1] = 0;
  for (int l = 1; l < 15; ++l) offs[l + 1] = (uint16_t)(offs[l] + h.count[l]);
  for (int s = 0; s < n; ++s)
    if (len[s]) h.sym[offs[len[s]]++] = (uint16_t)s;
  return left;
}

// The next symbol, or -1 (input ended, or a code the table does not hold).
CG_HD inline int huff_decode(Bits& b, const Huff& h) {
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16; ++l) {
    code |= (int)b.get(1);
    if (b.err) return -1;
    const int c = h.count[l];
    if (code - c < first) return h.sym[index + (code - first)];
    index += c;
    first += c;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

// zlib's acceptance of a built code (inflate_table): over-subscribed never;
// incomplete only when its longest code has length 1 (one symbol) — or, for
// distances, no codes at all (any distance then fails to decode).
CG_HD inline bool code_ok(const Huff& h, int left, bool dist) {
  if (left < 0) return false;
  if (left == 0) return true;
  if (dist && h.maxlen == 0) return true;
  return h.maxlen == 1;
}

constexpr uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
constexpr uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                    193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
constexpr uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

// Literal/length and distance codes of one block until end-of-block.
CG_HD inline int codes(Bits& b, const Huff& lit, const Huff& dist, uint8_t* dst, uint32_t cap, uint32_t& d) {
  for (;;) {
    const int s = huff_decode(b, lit);
    if (s < 0) return kKwzError;
    if (s < 256) {
      if (d >= cap) return kKwzMore;
      dst[d++] = (uint8_t)s;
      continue;
    }
    if (s == 256) return kKwzOk;
    const int li = s - 257;
    if (li >= 29) return kKwzError;  // 286, 287
    const uint32_t len = kLenBase[li] + b.get(kLenExtra[li]);
    const int ds = huff_decode(b, dist);
    if (ds < 0 || ds >= 30 || b.err) return kKwzError;
    const uint32_t off = kDistBase[ds] + b.get(kDistExtra[ds]);
    if (b.err || off > d) return kKwzError;  // distance too far back
    if (len > cap - d) return kKwzMore;
    for (uint32_t k = 0; k < len; ++k, ++d) dst[d] = dst[d - off];
  }
}

// A fixed-code block (RFC 1951 3.2.6) decoded arithmetically: the codes are
// canonical over four ranges, so the next 9 bits, bit-reversed into code
// order, name the symbol and its length with no table (small payloads —
// Kafka's message sets — are compressed as fixed blocks: zlib picks them
// below a few hundred bytes).  Same results as codes() over the built
// fixed tables, errors included (literal/length 286-287, distance 30-31).
CG_HD inline int codes_fixed(Bits& b, uint8_t* dst, uint32_t cap, uint32_t& d) {
  for (;;) {
    const uint32_t c9 = __builtin_bitreverse32(b.peek(9)) >> 23;
    int s;
    uint32_t l;
    if ((c9 >> 2) <= 23) {  // 0000000-0010111: 256-279
      s = 256 + (int)(c9 >> 2);
      l = 7;
    } else if ((c9 >> 1) <= 0xBF) {  // 00110000-10111111: 0-143
      s = (int)(c9 >> 1) - 0x30;
      l = 8;
    } else if ((c9 >> 1) <= 0xC7) {  // 11000000-11000111: 280-287
      s = 280 + (int)(c9 >> 1) - 0xC0;
      l = 8;
    } else {  // 110010000-111111111: 144-255
      s = 144 + (int)c9 - 0x190;
      l = 9;
    }
    b.drop(l);
    if (b.err) return kKwzError;
    if (s < 256) {
      if (d >= cap) return kKwzMore;
      dst[d++] = (uint8_t)s;
      continue;
    }
    if (s == 256) return kKwzOk;
    const int li = s - 257;
    if (li >= 29) return kKwzError;  // 286, 287
    const uint32_t len = kLenBase[li] + b.get(kLenExtra[li]);
    const int ds = (int)(__builtin_bitreverse32(b.get(5)) >> 27);
    if (ds >= 30 || b.err) return kKwzError;
    const uint32_t off = kDistBase[ds] + b.get(kDistExtra[ds]);
    if (b.err || off > d) return kKwzError;  // distance too far back
    if (len > cap - d) return kKwzMore;
    for (uint32_t k = 0; k < len; ++k, ++d) dst[d] = dst[d - off];
  }
}

// RFC 1951 DEFLATE data at src[0, n) into dst[0, cap): *out = bytes
// written, *used = input bytes consumed (through the byte holding the last
// block's end).
CG_HD inline int inflate_raw(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, uint32_t* used,
                             uint32_t* out) {
  Bits b{src, n, 0, 0, 0, false};
  uint32_t d = 0;
  Huff lit, dist;
  uint8_t len[320];
  for (;;) {
    const uint32_t last = b.get(1), type = b.get(2);
    if (b.err) return kKwzError;
    if (type == 0) {  // stored: to the byte boundary, LEN, NLEN, the bytes
      b.pos -= b.cnt / 8;  // (whole bytes a fixed block's peek loaded ahead)
      b.buf = 0;
      b.cnt = 0;
      if (b.pos + 4 > n) return kKwzError;
      const uint32_t l = src[b.pos] | (uint32_t)src[b.pos + 1] << 8;
      const uint32_t nl = src[b.pos + 2] | (uint32_t)src[b.pos + 3] << 8;
      b.pos += 4;
      if (l != (~nl & 0xFFFFu)) return kKwzError;
      if (l > n - b.pos) return kKwzError;
      if (l > cap - d) return kKwzMore;
      for (uint32_t k = 0; k < l; ++k) dst[d++] = src[b.pos + k];
      b.pos += l;
    } else if (type == 1) {  // fixed codes (RFC 1951 3.2.6)
      const int r = codes_fixed(b, dst, cap, d);
      if (r != kKwzOk) return r;
    } else if (type == 2) {  // dynamic codes (RFC 1951 3.2.7)
      const uint32_t nlen = b.get(5) + 257, ndist = b.get(5) + 1, ncode = b.get(4) + 4;
      if (b.err || nlen > 286 || ndist > 30) return kKwzError;
      const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
      for (int k = 0; k < 19; ++k) len[order[k]] = (uint8_t)(k < (int)ncode ? b.get(3) : 0);
      if (b.err) return kKwzError;
      Huff cl;
      if (huff_build(cl, len, 19) != 0) return kKwzError;  // the code-length code must be complete
      uint32_t k = 0;
      while (k < nlen + ndist) {
        const int s = huff_decode(b, cl);
        if (s < 0) return kKwzError;
        if (s < 16) {
          len[k++] = (uint8_t)s;
          continue;
        }
        uint32_t rep;
        uint8_t v = 0;
        if (s == 16) {
          if (k == 0) return kKwzError;  // no previous length
          v = len[k - 1];
          rep = 3 + b.get(2);
        } else if (s == 17) {
          rep = 3 + b.get(3);
        } else {
          rep = 11 + b.get(7);
        }
        if (b.err || k + rep > nlen + ndist) return kKwzError;
        while (rep--) len[k++] = v;
      }
      if (len[256] == 0) return kKwzError;  // no end-of-block code
      if (!code_ok(lit, huff_build(lit, len, (int)nlen), false)) return kKwzError;
      if (!code_ok(dist, huff_build(dist, len + nlen, (int)ndist), true)) return kKwzError;
      const int r = codes(b, lit, dist, dst, cap, d);
      if (r != kKwzOk) return r;
    } else {
      return kKwzError;  // reserved block type
    }
    if (last) break;
  }
  *used = b.pos - b.cnt / 8;
  *out = d;
  return kKwzOk;
}

// One gzip member at src[0, n) (compress/gzip Reader.readHeader + the
// trailer): *out = decoded bytes.  crc(p, len) is CRC-32 (IEEE).
template <class Crc>
CG_HD int gunzip_one(const uint8_t* b, uint32_t n, uint8_t* dst, uint32_t cap, uint32_t* out, Crc&& crc) {
  if (n < 10) return kKwzError;
  if (b[0] != 0x1F || b[1] != 0x8B || b[2] != 8) return kKwzError;
  const uint8_t flg = b[3];
  uint32_t q = 10;
  if (flg & 4) {  // FEXTRA
    if (q + 2 > n) return kKwzError;
    q += 2 + (uint32_t)(b[q] | b[q + 1] << 8);
    if (q > n) return kKwzError;
  }
  for (int f = 0; f < 2; ++f) {  // FNAME, FCOMMENT: NUL-terminated within 512 bytes
    if (!(flg & (f ? 16 : 8))) continue;
    const uint32_t lim = n < q + 512 ? n : q + 512;
    uint32_t z = q;
    while (z < lim && b[z] != 0) ++z;
    if (z >= lim) return kKwzError;
    q = z + 1;
  }
  if (flg & 2) {  // FHCRC
    if (q + 2 > n) return kKwzError;
    if ((crc(b, q) & 0xFFFFu) != (uint32_t)(b[q] | b[q + 1] << 8)) return kKwzError;
    q += 2;
  }
  uint32_t used = 0, d = 0;
  const int r = inflate_raw(b + q, n - q, dst, cap, &used, &d);
  if (r != kKwzOk) return r;
  q += used;
  if (q + 8 > n) return kKwzError;
  const uint32_t c = b[q] | (uint32_t)b[q + 1] << 8 | (uint32_t)b[q + 2] << 16 | (uint32_t)b[q + 3] << 24;
  const uint32_t isize = b[q + 4] | (uint32_t)b[q + 5] << 8 | (uint32_t)b[q + 6] << 16 | (uint32_t)b[q + 7] << 24;
  if (c != crc(dst, d) || isize != d) return kKwzError;
  if (q + 8 != n) return kKwzMore;
  *out = d;
  return kKwzOk;
}

// golang/snappy Decode of one block into dst[0, cap): the varint length must
// fit cap (the caller sized cap from it).
CG_HD inline int snappy_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, uint32_t* out) {
  uint64_t v = 0;
  uint32_t s = 0;
  for (int shift = 0;; shift += 7, ++s) {  // binary.Uvarint
    if (s >= n || s == 10) return kKwzError;
    const uint8_t c = src[s];
    if (c < 0x80) {
      if (s == 9 && c > 1) return kKwzError;
      v |= (uint64_t)c << shift;
      ++s;
      break;
    }
    v |= (uint64_t)(c & 0x7F) << shift;
  }
  if (v > cap) return kKwzMore;
  uint32_t d = 0;
  while (s < n) {
    uint32_t length, offset;
    const uint32_t tag = src[s] & 3;
    if (tag == 0) {
      uint32_t x = src[s] >> 2;
      if (x < 60) {
        s += 1;
      } else {
        const uint32_t k = x - 59;
        s += 1 + k;
        if (s > n) return kKwzError;
        x = 0;
        for (uint32_t i = 0; i < k; ++i) x |= (uint32_t)src[s - k + i] << (8 * i);
      }
      const uint64_t len64 = (uint64_t)x + 1;
      if (len64 > v - d || len64 > n - s) return kKwzError;
      for (uint32_t i = 0; i < (uint32_t)len64; ++i) dst[d + i] = src[s + i];
      d += (uint32_t)len64;
      s += (uint32_t)len64;
      continue;
    }
    if (tag == 1) {
      s += 2;
      if (s > n) return kKwzError;
      length = 4 + ((src[s - 2] >> 2) & 7);
      offset = (uint32_t)((src[s - 2] & 0xE0) << 3 | src[s - 1]);
    } else if (tag == 2) {
      s += 3;
      if (s > n) return kKwzError;
      length = 1 + (src[s - 3] >> 2);
      offset = (uint32_t)(src[s - 2] | src[s - 1] << 8);
    } else {
      s += 5;
      if (s > n) return kKwzError;
      length = 1 + (src[s - 5] >> 2);
      offset = (uint32_t)src[s - 4] | (uint32_t)src[s - 3] << 8 | (uint32_t)src[s - 2] << 16 |
               (uint32_t)src[s - 1] << 24;
    }
    if (offset == 0 || d < offset || length > v - d) return kKwzError;
    for (uint32_t end = d + length; d != end; ++d) dst[d] = dst[d - offset];
  }
  if (d != v) return kKwzError;
  *out = d;
  return kKwzOk;
}

// The decoded size of a snappy payload (a block, or xerial chunks), for the
// caller's reservation; false = not sized here (the host decides).
CG_HD inline bool snappy_size(const uint8_t* b, uint32_t n, uint64_t* size) {
  auto varint = [](const uint8_t* p, uint32_t m, uint64_t* v) {
    *v = 0;
    for (uint32_t s = 0, shift = 0; s < m && s < 10; ++s, shift += 7) {
      *v |= (uint64_t)(p[s] & 0x7F) << shift;
      if (p[s] < 0x80) return true;
    }
    return false;
  };
  const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
  bool xerial = n >= 8;
  for (int i = 0; xerial && i < 8; ++i) xerial = b[i] == magic[i];
  if (!xerial) return varint(b, n, size);
  if (n < 16) return false;
  uint64_t tot = 0;
  for (uint32_t i = 16; i < n;) {
    if (i + 4 > n) return false;
    const uint32_t k = (uint32_t)b[i] << 24 | (uint32_t)b[i + 1] << 16 | (uint32_t)b[i + 2] << 8 | b[i + 3];
    i += 4;
    if (k > n - i) return false;
    uint64_t v;
    if (!varint(b + i, k, &v)) return false;
    tot += v;
    i += k;
  }
  *size = tot;
  return true;
}

// The xerial framing (proto/snappy.go:23-50) or one block, into dst[0, cap).
CG_HD inline int snappy_go(const uint8_t* b, uint32_t n, uint8_t* dst, uint32_t cap, uint32_t* out) {
  const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
  bool xerial = n >= 8;
  for (int i = 0; xerial && i < 8; ++i) xerial = b[i] == magic[i];
  if (!xerial) return snappy_block(b, n, dst, cap, out);
  if (n < 16) return kKwzError;
  if (((uint32_t)b[8] << 24 | (uint32_t)b[9] << 16 | (uint32_t)b[10] << 8 | b[11]) != 1) return kKwzError;
  uint32_t d = 0;
  for (uint32_t i = 16; i < n;) {
    if (i + 4 > n) return kKwzError;
    const uint32_t k = (uint32_t)b[i] << 24 | (uint32_t)b[i + 1] << 16 | (uint32_t)b[i + 2] << 8 | b[i + 3];
    i += 4;
    if (k > n - i) return kKwzError;
    uint32_t got = 0;
    const int r = snappy_block(b + i, k, dst + d, cap - d, &got);
    if (r != kKwzOk) return r;
    d += got;
    i += k;
  }
  *out = d;
  return kKwzOk;
}

}  // namespace kwz
}  // namespace cg
