// http_latency.cc — Envoy-shaped HTTP verdict calls through the C ABI, timed
// per call at the batch sizes an Envoy worker would submit.
//
// The reference decides one request per AccessFilter::decodeHeaders
// (envoy/cilium_l7policy.cc:127-182 → NetworkPolicyMap::Allowed,
// cilium_network_policy.h:223-237).  A drop-in hands the engine the header
// lists it has (cg_http_pack's name\0value\0 input) in batches of B requests.
// Three host entries are timed, each for B in {1, 16, 256, 4096, 65536} and 1
// and 16 submitting threads (the ring also 4 and 8):
//   ring    cg_http_ring_verdicts: the persistent verdict ring (a resident
//           kernel polls request slots the host writes into device memory: no launch, no
//           copies, no stream synchronization per call; B <= 256)
//   fields  cg_http_verdicts_fields_host: calls of <= 1024 lists packed on
//           the calling thread (one copy in, one launch, one copy out),
//           larger ones: lists → pinned staging → H2D → grouping/packing on
//           the GPU → http_kernel → D2H
//   pack    cg_http_pack on the calling thread (CPU packer) +
//           cg_http_verdicts_host (staging → H2D → http_kernel → D2H)
// Each call's verdicts are checked against the pool's expected verdicts
// (want.bin: the engine's verdicts for the whole pool in one batch, checked
// against the oracle by tools/http_latency.py before this runs).
//
// Inputs (a directory written by tools/http_latency.py): policy.json,
// blob.bin, off.bin (u64, n + 1), pol.bin (u32), ing.bin (u8), port.bin
// (u16), rem.bin (u32), want.bin (u8).
//
// Build (in-tree, CPU): g++ -O2 -std=c++17 -I include tools/http_latency.cc
//   -L cilium_amd -lciliumgpu -lpthread -Wl,-rpath,'$ORIGIN/../cilium_amd' -o tools/http_latency
// Run (GPU box): tools/http_latency <dir> [seconds per point] [entries: ring,fields,pack]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <thread>
#include <vector>

#include "cilium_gpu.h"

namespace {

template <class T>
std::vector<T> load(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  std::vector<T> v(b.size() / sizeof(T));
  if (!v.empty()) memcpy(v.data(), b.data(), v.size() * sizeof(T));
  return v;
}

struct Pool {
  std::vector<uint8_t> blob, ing, want;
  std::vector<uint64_t> off;
  std::vector<uint32_t> pol, rem;
  std::vector<uint16_t> port;
  size_t n = 0;
};

struct Result {
  std::vector<double> lat_us;
  uint64_t calls = 0, bad = 0, requests = 0;
};

// One submitting thread: batches of B consecutive pool requests, starting at
// a per-thread offset, until the deadline.
void submit(uint64_t h, const Pool& p, int mode, size_t B, size_t start, double seconds, Result* r) {
  const bool pack = mode == 2;
  std::vector<uint8_t> out(B);
  std::vector<uint8_t> batch;
  std::vector<uint32_t> order;
  std::vector<uint8_t> arena(16u << 20);
  if (pack) {
    batch.resize(cg_http_batch_bytes(h, B));
    order.resize(cg_http_batch_slots(h, B) + 1);
  }
  const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double>(seconds);
  size_t a = start % (p.n - B + 1);
  r->lat_us.reserve(1 << 16);
  while (std::chrono::steady_clock::now() < end) {
    const auto t0 = std::chrono::steady_clock::now();
    int rc;
    if (pack) {
      size_t nslots = 0, used = 0;
      rc = cg_http_pack(h, B, &p.pol[a], &p.ing[a], &p.port[a], &p.rem[a], p.blob.data(), &p.off[a], batch.data(),
                        batch.size(), order.data(), &nslots, arena.data(), arena.size(), &used);
      if (rc == CG_OK)
        rc = cg_http_verdicts_host(h, batch.data(), nslots, order.data(), B, arena.data(), used, out.data());
    } else if (mode == 1) {
      rc = cg_http_ring_verdicts(h, p.blob.data(), &p.off[a], B, &p.pol[a], &p.ing[a], &p.port[a], &p.rem[a],
                                 out.data());
    } else {
      rc = cg_http_verdicts_fields_host(h, p.blob.data(), &p.off[a], B, &p.pol[a], &p.ing[a], &p.port[a], &p.rem[a],
                                        out.data());
    }
    const auto t1 = std::chrono::steady_clock::now();
    r->lat_us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    r->calls += 1;
    r->requests += B;
    r->bad += rc != CG_OK || memcmp(out.data(), &p.want[a], B) != 0;
    a += B;
    if (a + B > p.n) a = 0;
  }
}

double pct(std::vector<double>& v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1)))];
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: http_latency <dir> [seconds per point]\n");
    return 2;
  }
  const std::string d = argv[1];
  const double seconds = argc > 2 ? atof(argv[2]) : 1.0;
  const std::string entries = argc > 3 ? argv[3] : "ring,fields,pack";
  Pool p;
  p.blob = load<uint8_t>(d + "/blob.bin");
  p.off = load<uint64_t>(d + "/off.bin");
  p.pol = load<uint32_t>(d + "/pol.bin");
  p.ing = load<uint8_t>(d + "/ing.bin");
  p.port = load<uint16_t>(d + "/port.bin");
  p.rem = load<uint32_t>(d + "/rem.bin");
  p.want = load<uint8_t>(d + "/want.bin");
  p.n = p.pol.size();
  if (p.n == 0 || p.off.size() != p.n + 1 || p.ing.size() != p.n || p.port.size() != p.n || p.rem.size() != p.n ||
      p.want.size() != p.n) {
    fprintf(stderr, "bad pool in %s\n", d.c_str());
    return 2;
  }
  std::ifstream pf(d + "/policy.json", std::ios::binary);
  const std::string pol((std::istreambuf_iterator<char>(pf)), std::istreambuf_iterator<char>());
  const char* dev = getenv("CILIUM_GPU_DEVICE");
  cg_kv kv{"device", dev ? dev : "0"};
  const uint64_t h = cg_open(&kv, 1, 0);
  if (!h) {
    fprintf(stderr, "cg_open: %s\n", cg_last_error());
    return 2;
  }
  if (cg_http_policy_update(h, pol.data(), pol.size()) != CG_OK) {
    fprintf(stderr, "policy: %s\n", cg_last_error());
    return 2;
  }
  int rc = 0;
  const char* wg = getenv("CILIUM_RING_WORKGROUPS");
  const char* sl = getenv("CILIUM_RING_SLOTS");
  const uint32_t ring_wg = wg ? (uint32_t)atoi(wg) : 16, ring_slots = sl ? (uint32_t)atoi(sl) : 32;
  // modes: 1 cg_http_ring_verdicts, 0 cg_http_verdicts_fields_host, 2 pack + host
  for (const int mode : {1, 0, 2}) {
    const char* name = mode == 1 ? "ring" : mode == 0 ? "fields" : "pack";
    if (entries.find(name) == std::string::npos) continue;
    const bool pack = mode == 2;
    if (mode == 1 && cg_http_ring_open(h, ring_wg, ring_slots) != CG_OK) {
      fprintf(stderr, "cg_http_ring_open: %s\n", cg_last_error());
      return 2;
    }
    // CILIUM_LAT_ONLY="B:T" times one point (e.g. a phase trace of 1:1 alone)
    const char* only = getenv("CILIUM_LAT_ONLY");
    size_t only_b = 0;
    int only_t = 0;
    if (only) sscanf(only, "%zu:%d", &only_b, &only_t);
    for (const size_t B : {(size_t)1, (size_t)16, (size_t)256, (size_t)4096, (size_t)65536}) {
      if (B > p.n || (mode == 1 && B > 256)) continue;
      if (only && B != only_b) continue;
      for (const int threads : {1, 4, 8, 16}) {
        if (mode != 1 && (threads == 4 || threads == 8)) continue;  // (the ring's scaling only)
        if (only && threads != only_t) continue;
        {  // warm-up (pinned buffers, workers, launch caches) outside the clock
          Result w;
          submit(h, p, mode, B, 0, 0.05, &w);
        }
        std::vector<Result> res(threads);
        std::vector<std::thread> th;
        const auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < threads; ++t)
          th.emplace_back(submit, h, std::cref(p), mode, B, (size_t)t * 7919 * B, seconds, &res[t]);
        for (auto& x : th) x.join();
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::vector<double> lat;
        uint64_t calls = 0, bad = 0, reqs = 0;
        for (auto& r : res) {
          lat.insert(lat.end(), r.lat_us.begin(), r.lat_us.end());
          calls += r.calls;
          bad += r.bad;
          reqs += r.requests;
        }
        printf("{\"metric\": \"HTTP verdicts through the host C ABI at Envoy batch sizes\", \"entry\": \"%s\", "
               "\"batch\": %zu, \"threads\": %d, \"calls\": %llu, \"requests_per_s\": %.1f, \"calls_per_s\": %.1f, "
               "\"p50_us\": %.1f, \"p99_us\": %.1f, \"bad_calls\": %llu}\n",
               pack ? "cg_http_pack+cg_http_verdicts_host" : mode == 1 ? "cg_http_ring_verdicts"
                                                            : "cg_http_verdicts_fields_host", B, threads,
               (unsigned long long)calls, (double)reqs / sec, (double)calls / sec, pct(lat, 0.5), pct(lat, 0.99),
               (unsigned long long)bad);
        fflush(stdout);
        if (bad) rc = 1;
      }
    }
    if (mode == 1) {
      uint64_t served = 0, launches = 0;
      cg_http_ring_stats(h, &served, &launches);
      printf("{\"ring\": {\"workgroups\": %u, \"slots\": %u, \"served\": %llu, \"launches\": %llu}}\n", ring_wg,
             ring_slots, (unsigned long long)served, (unsigned long long)launches);
      cg_http_ring_close(h);
    }
  }
  cg_close(h);
  return rc;
}
