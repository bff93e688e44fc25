// ring_probe.hip — transport experiment for the verdict ring:
// one call's round trip host → device → host with the doorbell and the
// call's data in (a) pinned host memory, polled by the device across the bus
// (the ring's way), or (b) fine-grained device memory written by the host
// through its mapping, polled by the device locally.  The reply goes to
// pinned host memory in both.  Not product code.
//
//   hipcc --offload-arch=gfx950 -O2 tools/ring_probe.hip -o tools/_exp/ring_probe
//   tools/_exp/ring_probe [calls] [payload bytes]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

// One wave: lane 0 polls the doorbell word (relaxed system scope), the wave
// loads the payload after an acquire fence, folds it, writes {sum, seq} to
// the reply with a release fence.  Leaves on seq == 0xFFFFFFFF or after
// `limit` wall-clock ticks without a call.
__global__ void probe_kernel(uint32_t* door, const uint4* payload, uint32_t nvec, uint32_t* reply,
                             unsigned long long limit) {
  const uint32_t lane = threadIdx.x;
  uint32_t last = 0;
  unsigned long long t0 = wall_clock64();
  for (;;) {
    uint32_t s = 0;
    if (lane == 0) s = __hip_atomic_load(door, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s = (uint32_t)__shfl((int)s, 0, 64);
    if (s == 0xFFFFFFFFu) break;
    if (s == last) {
      if (wall_clock64() - t0 > limit) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    uint32_t acc = 0;
    for (uint32_t v = lane; v < nvec; v += 64) {
      const uint4 x = payload[v];
      acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
    for (int o = 32; o > 0; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o, 64);
    if (lane == 0) reply[1] = acc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (lane == 0) __hip_atomic_store(reply, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    last = s;
    t0 = wall_clock64();
  }
}

static double pct(std::vector<double>& v, double p) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * v.size()))];
}

// door / payload: host-writable pointers of the region the device polls
static void run(const char* name, uint8_t* region_host, uint8_t* region_dev, int calls, uint32_t bytes) {
  uint32_t* reply;
  CK(hipHostMalloc((void**)&reply, 64, hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(reply, 0, 64);
  uint32_t* reply_dev;
  CK(hipHostGetDevicePointer((void**)&reply_dev, reply, 0));
  volatile uint32_t* door_h = (volatile uint32_t*)region_host;
  *door_h = 0;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  const uint32_t nvec = (bytes + 15) / 16;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, st, (uint32_t*)region_dev, (const uint4*)(region_dev + 256),
                     nvec, reply_dev, 100ull * 1000 * 1000 * 5);  // 5 s idle at 100 MHz
  std::vector<uint8_t> src(bytes);
  std::vector<double> us;
  us.reserve(calls);
  uint32_t bad = 0;
  for (int i = 1; i <= calls + 1000; ++i) {
    for (uint32_t k = 0; k < bytes; ++k) src[k] = (uint8_t)(i * 131 + k);
    uint32_t want = 0;
    for (uint32_t k = 0; k + 4 <= bytes; k += 4) want ^= *(uint32_t*)&src[k];
    const auto t0 = std::chrono::steady_clock::now();
    std::memcpy(region_host + 256, src.data(), bytes);
    std::atomic_thread_fence(std::memory_order_seq_cst);  // (sfence: the data before the doorbell)
    *door_h = (uint32_t)i;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const auto spin0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(&reply[0], __ATOMIC_ACQUIRE) != (uint32_t)i) {
      if (std::chrono::steady_clock::now() - spin0 > std::chrono::seconds(2)) {
        std::fprintf(stderr, "%s: call %d timed out\n", name, i);
        std::exit(2);
      }
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (reply[1] != want) ++bad;
    if (i > 1000) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  *door_h = 0xFFFFFFFFu;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  CK(hipStreamSynchronize(st));
  std::printf("{\"mode\": \"%s\", \"calls\": %d, \"payload\": %u, \"bad\": %u, \"p50_us\": %.2f, \"p90_us\": %.2f, "
              "\"p99_us\": %.2f}\n",
              name, calls, bytes, bad, pct(us, 0.5), pct(us, 0.9), pct(us, 0.99));
  std::fflush(stdout);
  CK(hipStreamDestroy(st));
  CK(hipHostFree(reply));
}

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 20000;
  const uint32_t bytes = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 256;
  CK(hipSetDevice(0));
  // (a) pinned host memory, the ring's slots
  uint8_t* h;
  CK(hipHostMalloc((void**)&h, 64 * 1024, hipHostMallocCoherent | hipHostMallocMapped));
  uint8_t* hd;
  CK(hipHostGetDevicePointer((void**)&hd, h, 0));
  run("host_pinned", h, hd, calls, bytes);
  // (b) fine-grained / uncached device memory, if the host can reach it
  const unsigned flags[2] = {hipDeviceMallocFinegrained, hipDeviceMallocUncached};
  const char* names[2] = {"device_finegrained", "device_uncached"};
  for (int f = 0; f < 2; ++f) {
    uint8_t* d = nullptr;
    if (hipExtMallocWithFlags((void**)&d, 64 * 1024, flags[f]) != hipSuccess) {
      std::printf("{\"mode\": \"%s\", \"error\": \"alloc\"}\n", names[f]);
      continue;
    }
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, d);
    std::printf("{\"mode\": \"%s\", \"attr_err\": %d, \"type\": %d, \"host\": \"%p\", \"dev\": \"%p\"}\n", names[f],
                (int)e, (int)a.type, a.hostPointer, a.devicePointer);
    std::fflush(stdout);
    uint8_t* hp = (uint8_t*)a.hostPointer;
    if (!hp) {
      // the same virtual address from the CPU, once the CPU agent may access it
      hsa_agent_t cpu{};
      (void)hsa_iterate_agents(
          [](hsa_agent_t ag, void* out) {
            hsa_device_type_t t;
            hsa_agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &t);
            if (t == HSA_DEVICE_TYPE_CPU) {
              *(hsa_agent_t*)out = ag;
              return HSA_STATUS_INFO_BREAK;
            }
            return HSA_STATUS_SUCCESS;
          },
          &cpu);
      const hsa_status_t s = hsa_amd_agents_allow_access(1, &cpu, nullptr, d);
      hsa_amd_pointer_info_t pi{};
      pi.size = sizeof(pi);
      (void)hsa_amd_pointer_info(d, &pi, nullptr, nullptr, nullptr);
      std::printf("{\"mode\": \"%s\", \"allow_access\": %d, \"host_base\": \"%p\", \"agent_base\": \"%p\"}\n",
                  names[f], (int)s, pi.hostBaseAddress, pi.agentBaseAddress);
      std::fflush(stdout);
      if (s == HSA_STATUS_SUCCESS) hp = pi.hostBaseAddress ? (uint8_t*)pi.hostBaseAddress : d;
    }
    if (hp) {
      // a CPU write and read back before any kernel runs on it
      volatile uint32_t* w = (volatile uint32_t*)(hp + 128);
      *w = 0x12345678u;
      std::atomic_thread_fence(std::memory_order_seq_cst);
      std::printf("{\"mode\": \"%s\", \"cpu_rw\": %d}\n", names[f], (int)(*w == 0x12345678u));
      std::fflush(stdout);
      run(names[f], hp, d, calls, bytes);
    }
    CK(hipFree(d));
  }
  CK(hipHostFree(h));
  return 0;
}
