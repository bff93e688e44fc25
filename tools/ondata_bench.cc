// ondata_bench.cc — proxylib OnData through the C ABI Envoy calls
// (include/cilium_proxylib.h = proxylib/libcilium.h:77-115), timed per call.
//
// For each parser (r2d2, memcache text, cassandra) and each thread count,
// every thread owns one connection and makes `calls` OnData calls of
// `frames` request frames (16 = Envoy's ops buffer, cilium_proxylib.cc:199),
// half of them denied by the policy (memcache: all allowed — a denial
// waits for the replies before it in the reference's in-order reply
// tracking).  Each call's ops are checked against the expected PASS / DROP
// sequence.  One JSON line per (parser, threads): calls/s, frames/s, p50 /
// p99 call latency and the GPU batches that decided them
// (cg_proxylib_stats: concurrent calls share one batch).
//
// Build (in-tree, CPU): g++ -O2 -std=c++17 -I include tools/ondata_bench.cc
//   -L cilium_amd -lciliumgpu -lpthread -Wl,-rpath,'$ORIGIN/../cilium_amd' -o tools/ondata_bench
// Run (GPU box): CILIUM_GPU_DEVICE=0 tools/ondata_bench [calls] [frames]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "cilium_gpu.h"
#include "cilium_proxylib.h"

namespace {

GoString gs(const std::string& s) { return GoString{s.data(), (ptrdiff_t)s.size()}; }

const char* kPolicy =
    "[{\"name\":\"bench\",\"ingress_per_port_policies\":["
    "{\"port\":80,\"rules\":[{\"remote_policies\":[1],\"l7_proto\":\"r2d2\",\"l7_rules\":{\"l7_rules\":["
    "{\"rule\":{\"cmd\":\"READ\",\"file\":\"^/public/[a-z0-9]+$\"}},{\"rule\":{\"cmd\":\"HALT\"}}]}}]},"
    "{\"port\":11211,\"rules\":[{\"remote_policies\":[1],\"l7_proto\":\"memcache\",\"l7_rules\":{\"l7_rules\":["
    "{\"rule\":{\"command\":\"get\",\"keyPrefix\":\"user:\"}}]}}]},"
    "{\"port\":9042,\"rules\":[{\"remote_policies\":[1],\"l7_proto\":\"cassandra\",\"l7_rules\":{\"l7_rules\":["
    "{\"rule\":{\"query_action\":\"select\",\"query_table\":\"^ks\\\\.\"}}]}}]}]}]";

struct Work {
  std::string proto;
  uint16_t port;
  std::vector<std::string> frames;  // request frames of one call
  std::vector<uint64_t> want_op;    // FILTEROP_PASS / FILTEROP_DROP per frame
};

std::string be32(uint32_t v) {
  return std::string{(char)(v >> 24), (char)(v >> 16), (char)(v >> 8), (char)v};
}

// A CQL v4 QUERY frame (cassandraparser.go:171-236): 9-byte header, long
// string query, consistency ONE, no flags.
std::string cql_query(uint16_t stream, const std::string& q) {
  std::string body = be32((uint32_t)q.size()) + q + std::string("\x00\x01\x00", 3);
  return std::string{'\x04', '\x00', (char)(stream >> 8), (char)stream, '\x07'} + be32((uint32_t)body.size()) + body;
}

Work make_work(const std::string& proto, int frames, int seed) {
  Work w;
  w.proto = proto;
  for (int i = 0; i < frames; ++i) {
    const bool allow = proto == "memcache" || ((i + seed) % 2 == 0);
    const std::string id = std::to_string(seed * 1000 + i);
    if (proto == "r2d2") {
      w.port = 80;
      w.frames.push_back(allow ? "READ /public/f" + id + "\r\n" : "READ /private/f" + id + "\r\n");
    } else if (proto == "memcache") {
      w.port = 11211;
      w.frames.push_back("get user:" + id + "\r\n");
    } else {
      w.port = 9042;
      w.frames.push_back(cql_query((uint16_t)(i + 1), allow ? "SELECT a FROM ks.t" + id : "SELECT a FROM other.t" + id));
    }
    w.want_op.push_back(allow ? FILTEROP_PASS : FILTEROP_DROP);
  }
  return w;
}

struct Result {
  std::vector<double> lat_us;
  uint64_t bad = 0;
};

void run_conn(uint64_t inst, uint64_t conn_id, const Work& w, int calls, Result* res) {
  std::vector<char> orig(1 << 16), reply(1 << 20);
  GoSlice ob{orig.data(), 0, (int64_t)orig.size()}, rb{reply.data(), 0, (int64_t)reply.size()};
  const std::string src = "1.1.1.1:40000", dst = "2.2.2.2:" + std::to_string(w.port), pol = "bench";
  if (OnNewConnection(inst, gs(w.proto), conn_id, 1, 1, 2, gs(src), gs(dst), gs(pol), &ob, &rb) != FILTER_OK) {
    res->bad += (uint64_t)calls;
    return;
  }
  std::string data;
  for (const auto& f : w.frames) data += f;
  std::vector<FilterOp> ops(w.frames.size() + 2);
  res->lat_us.reserve((size_t)calls);
  for (int k = 0; k < calls; ++k) {
    GoSlice chunk{(void*)data.data(), (int64_t)data.size(), (int64_t)data.size()};
    GoSlice dv{&chunk, 1, 1};
    GoSlice ov{ops.data(), 0, (int64_t)w.frames.size()};
    const auto t0 = std::chrono::steady_clock::now();
    const FilterResult rc = OnData(conn_id, 0, 0, &dv, &ov);
    const auto t1 = std::chrono::steady_clock::now();
    res->lat_us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    bool ok = rc == FILTER_OK && ov.len == (int64_t)w.frames.size();
    for (int64_t i = 0; ok && i < ov.len; ++i)
      ok = ops[i].op == w.want_op[i] && ops[i].n_bytes == (int64_t)w.frames[i].size();
    res->bad += !ok;
    rb.len = 0;  // Envoy drains the injected replies between calls
    ob.len = 0;
  }
  Close(conn_id);
}

double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1)))];
}

}  // namespace

int main(int argc, char** argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 2000;
  const int frames = argc > 2 ? atoi(argv[2]) : 16;
  const std::string node = "ondata-bench";
  std::vector<GoString> kv{gs("node-id"), gs(node)};
  GoSlice params{kv.data(), 1, 1};
  const uint64_t inst = OpenModule(params, 0);
  if (!inst) {
    fprintf(stderr, "OpenModule failed: %s\n", cg_last_error());
    return 2;
  }
  if (cg_proxylib_policy_update(inst, kPolicy, strlen(kPolicy)) != CG_OK) {
    fprintf(stderr, "policy update failed: %s\n", cg_last_error());
    return 2;
  }
  uint64_t next_conn = 1;
  int rc = 0;
  for (const char* proto : {"r2d2", "memcache", "cassandra"}) {
    for (int threads : {1, 16}) {
      std::vector<Work> work;
      for (int t = 0; t < threads; ++t) work.push_back(make_work(proto, frames, t));
      std::vector<Result> res(threads);
      // warm-up call per connection outside the clock
      {
        Result warm;
        run_conn(inst, next_conn++, work[0], 20, &warm);
      }
      uint64_t b0 = 0, c0 = 0, b1 = 0, c1 = 0;
      cg_proxylib_stats(inst, &b0, &c0);
      std::vector<std::thread> th;
      const auto t0 = std::chrono::steady_clock::now();
      for (int t = 0; t < threads; ++t)
        th.emplace_back(run_conn, inst, next_conn++, std::cref(work[t]), calls, &res[t]);
      for (auto& x : th) x.join();
      const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      cg_proxylib_stats(inst, &b1, &c1);
      std::vector<double> lat;
      uint64_t bad = 0;
      for (auto& r : res) {
        lat.insert(lat.end(), r.lat_us.begin(), r.lat_us.end());
        bad += r.bad;
      }
      const double ncalls = (double)calls * threads;
      printf("{\"metric\": \"proxylib OnData calls/s through the C ABI (%s)\", \"parser\": \"%s\", "
             "\"threads\": %d, \"connections\": %d, \"frames_per_call\": %d, \"calls\": %.0f, "
             "\"calls_per_s\": %.1f, \"frames_per_s\": %.1f, \"p50_us\": %.1f, \"p99_us\": %.1f, "
             "\"gpu_batches\": %llu, \"calls_per_batch\": %.2f, \"bad_calls\": %llu}\n",
             proto, proto, threads, threads, frames, ncalls, ncalls / sec, ncalls * frames / sec, pct(lat, 0.5),
             pct(lat, 0.99), (unsigned long long)(b1 - b0), (b1 > b0) ? (double)(c1 - c0) / (double)(b1 - b0) : 0.0,
             (unsigned long long)bad);
      fflush(stdout);
      if (bad) rc = 1;
    }
  }
  CloseModule(inst);
  return rc;
}
