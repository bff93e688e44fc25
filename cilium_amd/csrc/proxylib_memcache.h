// proxylib_memcache.h — the memcached proxylib parser (text and binary
// protocols) and the connection op loop it runs under, for the proxylib C ABI
// shim (proxylib_shim.cc).
//
//   memcached/parser.go:176-199        protocol choice on the first byte
//   memcached/text/parser.go:70-330    text framing, reply tracking, denial
//   memcached/binary/parser.go:62-205  binary framing, in-order denials
//   proxylib/connection.go:118-174     the op loop (NOP / MORE / PASS / DROP /
//                                      INJECT, parser panics → PARSER_ERROR)
//
// Policy matching (memcached/parser.go:46-97, Rule.Matches) is not done here:
// `match` is called once per request frame in order, and the shim answers it
// with verdicts computed on the GPU for all the frames of an OnData call.
#pragma once

#include <cstdint>
#include <deque>
#include <functional>
#include <string>
#include <vector>

#include "../../include/cilium_proxylib.h"

namespace cg {

// What Rule.Matches sees (memcached/meta/meta.go): a text command, or a
// binary opcode (command empty), and the request's keys.
struct McMeta {
  std::string command;
  uint8_t opcode = 0;
  std::vector<std::string> keys;
  bool binary() const { return command.empty(); }
};

struct McState {
  int mode = 0;  // 0 undecided, 1 text, 2 binary (the first request byte)
  // text
  std::deque<std::pair<std::string, bool>> text_queue;  // (command, denied)
  bool watching = false;
  // binary
  uint32_t requests = 0, replies = 0;
  std::deque<std::pair<uint8_t, uint32_t>> bin_queue;  // (magic, request id)
};

using McMatch = std::function<bool(const McMeta&)>;

// One OnData call of a memcache connection: parser calls until the ops
// slice is full, the parser asks for MORE or returns NOP.  Denial messages
// go into reply_buf.  Returns the FilterResult.
FilterResult memcache_on_data(McState& st, bool reply, bool end_stream, const GoSlice* data, GoSlice* ops,
                              GoSlice* reply_buf, const McMatch& match);

// The text denial and the binary denial template (text/parser.go:326,
// binary/parser.go:195-205).
extern const char kMcTextDenied[];
extern const uint8_t kMcBinaryDenied[37];

}  // namespace cg
