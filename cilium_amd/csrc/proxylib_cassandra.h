// proxylib_cassandra.h — the Cassandra v3/v4 proxylib parser (request and
// reply framing, query → "/opcode/action/table" paths, prepared-statement
// tracking) and the connection op loop it runs under, for the proxylib C ABI
// shim (proxylib_shim.cc).
//
//   cassandra/cassandraparser.go:171-256   OnData (framing, verdict, inject)
//   cassandra/cassandraparser.go:344-455   parseQuery
//   cassandra/cassandraparser.go:457-578   cassandraParseRequest
//   cassandra/cassandraparser.go:580-642   unprepared reply, reply parsing
//   proxylib/connection.go:118-174         the op loop (ERROR does not advance
//                                          the input; parser panics →
//                                          PARSER_ERROR)
//
// Policy matching (CassandraRule.Matches, :57-94) is not done here: `match`
// is called once per path, in order, and the shim answers it with verdicts
// computed on the GPU for all the paths of an OnData call.
#pragma once

#include <cstdint>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "../../include/cilium_proxylib.h"

namespace cg {

struct CassState {
  std::string keyspace;                          // from the last "use"
  std::map<uint16_t, std::string> by_stream;     // prepare path by stream id
  std::map<std::string, std::string> by_id;      // execute path by prepared id
};

using CassMatch = std::function<bool(const std::string& path)>;

// One OnData call of a cassandra connection.  Denials go into reply_buf.
FilterResult cassandra_on_data(CassState& st, bool reply, bool end_stream, const GoSlice* data, GoSlice* ops,
                               GoSlice* reply_buf, const CassMatch& match);

// The request fields a path is matched on (see proxylib_shim.cc
// cassandra_rules): cshape S (≤ 2 parts: allowed by every rule), X (3 parts:
// matched by none), L (action = part 2, table = part 3).
struct CassFields {
  char shape;
  std::string action, table;
};
CassFields cassandra_path_fields(const std::string& path);

}  // namespace cg
