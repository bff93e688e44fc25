// kafka_wire.h — Kafka request decoding, shared by the host decoder
// (kafka_wire.cc) and the GPU decode kernel (kernels_kafka.hip).
//
// What the Kafka proxy does with the bytes of one request, restated from
// pkg/kafka/request.go:186-229 (ReadRequest) and the vendored optiopay/kafka
// proto package (cilium fork @01ce283b, Gopkg.toml:58-60):
//   ReadReq                    messages.go:124-166   size, apiKey, allocParseBuf
//   Read{Produce,Fetch,Offset,Metadata,ConsumerMetadata,OffsetCommit,
//        OffsetFetch}Req        messages.go:1591,767,1810,504,1033,1173,1389
//   readMessageSet             messages.go:352-494   (CRC32 per message; the
//                              proxy parses message sets in full,
//                              pkg/proxy/kafka.go:449-451)
//   decoder                    serialization.go:32-190 (sticky first error)
//   allocParseBuf              utils.go:9,18-24 (maxParseBufSize = 100 * 65535)
//
// The decoder reads one request from the start of its slice of the
// connection's bytes: 4 + size bytes.  Its outcome is what the verdict
// needs: ReadRequest's error (the proxy closes the connection), or apiKey,
// version, the request class (the six topic-carrying kinds / consumer
// metadata / any other key, request == nil), the clientID and the topic
// names (GetTopics, request.go:88-108).
//
// The stream positions follow Go's exactly: every decoder of one request
// reads the same bytes.Buffer, and readMessageSet's early returns (short
// set, bad CRC, empty message) leave the rest of a message set unread for
// the next partition's decoder.  Compressed messages (gzip, snappy) are
// decompressed and their inner set parsed through `Inflate`: zlib and a
// snappy restatement on the host (kafka_wire.cc), kw_inflate.h on the device
// (kernels_kafka.hip), which hands what it cannot finish to the host as
// kKwDefer.
#pragma once

#include <cstddef>
#include <cstdint>

#include "dev_types.h"

namespace cg {

constexpr uint32_t kKafkaMaxParseBuf = 100u * 65535u;  // utils.go:9
// Device bytes per decode call for compressed payloads decoded on the GPU
// (kernels_kafka.hip DevInflate); a payload past it is decoded by the host.
constexpr size_t kKafkaInflateArena = (size_t)64 << 20;

// Decoder outcomes (also the cg_kafka_decode status values).
constexpr uint8_t kKwOk = CG_KAFKA_DECODE_OK;
constexpr uint8_t kKwError = CG_KAFKA_DECODE_ERROR;
constexpr uint8_t kKwDefer = 2;  // a compressed message the device decoder hands to the host

// io.ReadFull over a shared bytes.Buffer, optionally through io.LimitReader.
// err: 0 none, 1 EOF / ErrUnexpectedEOF, 2 another error (sticky).
struct KwStream {
  const uint8_t* p;
  uint32_t len, pos;
};

struct KwDec {
  KwStream* s;
  uint32_t* limit;  // LimitReader budget, or nullptr
  uint32_t err = 0;

  CG_HD bool take(uint32_t n, const uint8_t** out) {
    if (err) return false;
    uint32_t avail = s->len - s->pos;
    if (limit && *limit < avail) avail = *limit;
    if (n > avail) {  // ReadFull consumes what there is, then EOF
      s->pos += avail;
      if (limit) *limit -= avail;
      err = 1;
      return false;
    }
    *out = s->p + s->pos;
    s->pos += n;
    if (limit) *limit -= n;
    return true;
  }
  CG_HD uint64_t be(uint32_t n) {
    const uint8_t* b;
    if (!take(n, &b)) return 0;
    uint64_t x = 0;
    for (uint32_t i = 0; i < n; ++i) x = x << 8 | b[i];
    return x;
  }
  CG_HD int8_t i8() { return (int8_t)be(1); }
  CG_HD int16_t i16() { return (int16_t)be(2); }
  CG_HD int32_t i32() { return (int32_t)be(4); }
  CG_HD uint32_t u32() { return (uint32_t)be(4); }
  CG_HD int64_t i64() { return (int64_t)be(8); }
  // DecodeString: int16 length, < 1 = "" (nothing more read)
  CG_HD bool str(uint32_t* off, uint32_t* n) {
    *off = s->pos;
    *n = 0;
    if (err) return false;
    const int16_t l = i16();
    if (err || l < 1) return !err;
    const uint8_t* b;
    if (!take((uint32_t)l, &b)) return false;
    *off = (uint32_t)(b - s->p);
    *n = (uint32_t)l;
    return true;
  }
  // DecodeBytes: int32 length, < 1 = nil, > maxParseBufSize = error
  CG_HD bool bytes(uint32_t* off, uint32_t* n) {
    *n = 0;
    if (err) return false;
    const int32_t l = i32();
    if (err || l < 1) return !err;
    if ((uint32_t)l > kKafkaMaxParseBuf) {
      err = 2;
      return false;
    }
    const uint8_t* b;
    if (!take((uint32_t)l, &b)) return false;
    *off = (uint32_t)(b - s->p);
    *n = (uint32_t)l;
    return true;
  }
  // DecodeArrayLen: returns false on ErrInvalidArrayLen (the callers return
  // it); a pending error reads 0
  CG_HD bool array_len(bool nullable, int32_t* out) {
    const int32_t l = i32();
    *out = l;
    if (l < 0) return nullable;
    return (uint32_t)l <= kKafkaMaxParseBuf;
  }
};

// readMessageSet over stream s (messages.go:352-494).  Returns kKwOk,
// kKwError or kKwDefer.  crc(p, n) is CRC-32 (IEEE); inflate(codec, data, n,
// version) decodes a compressed message's value and parses its inner set
// (host), or returns kKwDefer (device).
template <class Crc, class Inflate>
CG_HD uint8_t kw_message_set(KwStream* s, int32_t size, int16_t version, Crc&& crc, Inflate&& inflate) {
  if (size < 0) return kKwOk;  // null RECORDS
  if ((uint32_t)size > kKafkaMaxParseBuf) return kKwError;
  uint32_t lim = (uint32_t)size;
  KwDec dec{s, &lim};
  for (;;) {
    dec.i64();  // offset
    if (dec.err) return dec.err == 1 ? kKwOk : kKwError;
    const int32_t msize = dec.i32();
    if (dec.err) return dec.err == 1 ? kKwOk : kKwError;
    if (msize <= 0) return kKwOk;
    if ((uint32_t)msize > kKafkaMaxParseBuf) return kKwError;
    const uint8_t* msg;
    if (!dec.take((uint32_t)msize, &msg)) return kKwOk;  // a message cut short: the set so far
    // the message, decoded from its own buffer
    KwStream ms{msg, (uint32_t)msize, 0};
    KwDec md{&ms, nullptr};
    const uint32_t crc_field = md.u32();
    if (msize <= 4) return kKwOk;
    if (crc_field != crc(msg + 4, (uint32_t)msize - 4)) return kKwOk;  // stop, keep the set
    md.i8();  // magic
    const int8_t attributes = md.i8();
    if (version >= 1) md.i64();  // timestamp
    const uint32_t codec = (uint32_t)attributes & 3;
    uint32_t koff = 0, kn = 0, voff = 0, vn = 0;
    if (codec == 0) {
      md.bytes(&koff, &kn);
      md.bytes(&voff, &vn);
      if (md.err) return kKwError;
    } else if (codec == 1 || codec == 2) {
      md.bytes(&koff, &kn);
      md.bytes(&voff, &vn);
      if (md.err) return kKwError;
      const uint8_t r = inflate(codec, msg + voff, vn, version);
      if (r != kKwOk) return r;
    } else {
      return kKwOk;  // `return nil, err` with err == nil: the set ends
    }
  }
}

// The decoded request, as MatchesRule needs it.
struct KwRequest {
  int16_t api_key = 0, version = 0;
  uint8_t cls = CG_KAFKA_K_NIL;
  uint32_t client_off = 0, client_len = 0;
};

// ReadRequest on raw[0, len): the outcome, r, and the topic names (GetTopics)
// through the sink: sink.begin(count) once the topics array length is read
// (count >= 0), then sink.topic(off, len) per name in request order.  On a
// kKwOk outcome exactly `count` names follow begin.
template <class Crc, class Sink, class Inflate>
CG_HD uint8_t kw_decode(const uint8_t* raw, uint32_t len, Crc&& crc, KwRequest* r, Sink&& sink, Inflate&& inflate) {
  // ---- ReadReq (messages.go:124-166) on the connection's bytes
  KwStream conn{raw, len, 0};
  KwDec d{&conn, nullptr};
  const int32_t size = d.i32();
  if (d.err) return kKwError;
  if (size <= 0) return kKwError;
  const int16_t kind = d.i16();
  if (d.err) return kKwError;
  if ((uint64_t)(uint32_t)size + 4 > kKafkaMaxParseBuf) return kKwError;
  const uint32_t total = (uint32_t)size + 4;
  if (total > 6 && len < total) return kKwError;  // io.ReadFull of the rest
  // ReadRequest: length < 12 is an error; the version is at [6:8]
  if (total < 12) return kKwError;
  r->api_key = kind;
  r->version = (int16_t)((uint16_t)raw[6] << 8 | raw[7]);
  const bool typed = kind == 0 || kind == 1 || kind == 2 || kind == 3 || kind == 8 || kind == 9;
  if (!typed && kind != 10) {
    r->cls = CG_KAFKA_K_NIL;  // unknown key: request == nil, nothing more parsed
    return kKwOk;
  }
  // ---- the kind's decoder on rawMsg (with apiKey written back at [4:6])
  KwStream s{raw, total, 0};
  KwDec dec{&s, nullptr};
  dec.i32();
  dec.i16();
  const int16_t ver = dec.i16();
  dec.i32();  // correlation id
  dec.str(&r->client_off, &r->client_len);
  if (kind == 10) {  // ConsumerMetadata
    uint32_t o, n;
    dec.str(&o, &n);
    if (ver >= 1) dec.i8();
    r->cls = CG_KAFKA_K_CONSUMER_METADATA;
    return dec.err ? kKwError : kKwOk;
  }
  r->cls = CG_KAFKA_K_TYPED;
  int32_t nt = 0;
  uint32_t o, n;
  if (kind == 3) {  // Metadata: nullable topics, then the v4 flag
    if (!dec.array_len(true, &nt)) return kKwError;
    if (dec.err) return kKwError;
    if (nt > 0) sink.begin(nt);
    for (int32_t i = 0; i < nt && !dec.err; ++i) {
      dec.str(&o, &n);
      if (!dec.err) sink.topic(o, n);
    }
    if (ver >= 4) dec.i8();
    return dec.err ? kKwError : kKwOk;
  }
  if (kind == 0) {  // Produce
    if (ver >= 3) dec.str(&o, &n);  // transactional id
    dec.i16();
    dec.i32();
  } else if (kind == 1) {  // Fetch
    dec.i32();
    dec.i32();
    dec.i32();
    if (ver >= 3) dec.i32();
    if (ver >= 4) dec.i8();
  } else if (kind == 2) {  // Offset
    dec.i32();
    if (ver >= 2) dec.i8();
  } else if (kind == 8) {  // OffsetCommit
    dec.str(&o, &n);
    if (ver >= 1) {
      dec.i32();
      dec.str(&o, &n);
    }
    if (ver >= 2) dec.i64();
  } else {  // 9: OffsetFetch
    dec.str(&o, &n);
  }
  if (!dec.array_len(kind == 9, &nt)) return kKwError;
  if (dec.err) return kKwError;
  if (nt > 0) sink.begin(nt);
  // a pending error makes the remaining decodes no-ops that read 0: the loop
  // ends at the first array length it cannot read, with the same outcome
  for (int32_t t = 0; t < nt && !dec.err; ++t) {
    dec.str(&o, &n);
    if (!dec.err) sink.topic(o, n);
    int32_t np = 0;
    if (!dec.array_len(false, &np)) return kKwError;
    for (int32_t p = 0; p < np && !dec.err; ++p) {
      if (kind == 0) {
        dec.i32();
        if (dec.err) return kKwError;
        const int32_t mss = dec.i32();
        if (dec.err) return kKwError;
        const uint8_t m = kw_message_set(&s, mss, ver, crc, inflate);
        if (m != kKwOk) return m;
      } else if (kind == 1) {
        dec.i32();
        dec.i64();
        if (ver >= 5) dec.i64();
        dec.i32();
      } else if (kind == 2) {
        dec.i32();
        dec.i64();
        if (ver == 0) dec.i32();
      } else if (kind == 8) {
        dec.i32();
        dec.i64();
        if (ver == 1) dec.i64();
        dec.str(&o, &n);
      } else {
        dec.i32();
      }
    }
  }
  return dec.err ? kKwError : kKwOk;
}

}  // namespace cg
