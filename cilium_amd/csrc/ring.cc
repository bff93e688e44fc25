// ring.cc — the persistent verdict ring (include/cilium_gpu.h cg_http_ring_*).
//
// Envoy decides one request per AccessFilter::decodeHeaders
// (envoy/cilium_l7policy.cc:127-182), from many worker threads.  Through
// cg_http_verdicts_fields_host such a call pays a staged copy in, a launch, a
// copy out and a stream synchronization (~30 us).  The ring removes all four:
// a resident kernel (kernels_http_raw.hip http_ring_kernel) polls request
// slots; a call claims a slot, writes its header lists and inputs there,
// stores the slot's doorbell and spins on the completion word the kernel
// stores after the verdicts.  The request slots are fine-grained device
// memory the host writes through its mapping (posted writes; the kernel
// polls and reads them without crossing the bus), the replies pinned host
// memory the host polls (dev_types.h kRingReplyBytes).
//
// Lifetime: the kernel runs with the tables of one HTTP snapshot (held here,
// so they outlive it).  A call first makes sure a launch with the handle's
// current snapshot is running — a policy update stops the old launch (stop
// word, stream synchronize) and starts a new one — so a call that begins
// after an update returns is decided by the new tables.  A launch also ends
// by itself after kIdleMs without a call or kLifeMs in all; a caller whose
// doorbell it missed sees the stream idle while it waits and relaunches.
// cg_http_ring_close and cg_close stop it.  Calls that do not fit a slot
// (more than kRingReqs lists, more than kRingBlob bytes) or a snapshot the
// device list parser does not take (more than 32 header fields) are decided
// by cg_http_verdicts_fields_host instead.
#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "engine.h"
#include "http.h"
#include "kernels.h"
#include "ring.h"

namespace cg {

namespace {

constexpr uint32_t kIdleMs = 50, kLifeMs = 2000;

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

inline void cpu_relax() { __builtin_ia32_pause(); }

// Fine-grained device memory the host can store to (the same virtual address
// on both sides), or nullptr: hipExtMallocWithFlags(hipDeviceMallocFinegrained)
// and the CPU agents let in (hsa_amd_agents_allow_access), checked with one
// store and load from the host.
uint8_t* device_slots_for_host(size_t bytes) {
  uint8_t* d = nullptr;
  if (hipExtMallocWithFlags((void**)&d, bytes, hipDeviceMallocFinegrained) != hipSuccess) return nullptr;
  std::vector<hsa_agent_t> cpus;
  (void)hsa_iterate_agents(
      [](hsa_agent_t ag, void* out) {
        hsa_device_type_t t;
        if (hsa_agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU)
          static_cast<std::vector<hsa_agent_t>*>(out)->push_back(ag);
        return HSA_STATUS_SUCCESS;
      },
      &cpus);
  hsa_amd_pointer_info_t pi{};
  pi.size = sizeof(pi);
  if (cpus.empty() || hsa_amd_agents_allow_access((uint32_t)cpus.size(), cpus.data(), nullptr, d) != HSA_STATUS_SUCCESS ||
      hsa_amd_pointer_info(d, &pi, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS || pi.hostBaseAddress != d) {
    (void)hipFree(d);
    return nullptr;
  }
  volatile uint32_t* w = reinterpret_cast<volatile uint32_t*>(d);
  *w = 0x5A5A5A5Au;
  __builtin_ia32_mfence();
  if (*w != 0x5A5A5A5Au) {
    (void)hipFree(d);
    return nullptr;
  }
  return d;
}

}  // namespace

HttpRing::~HttpRing() {
  stop_locked_noexcept();
  if (state_) (void)hipFree(state_);
  if (host_) (void)hipHostFree(host_);
  if (req_in_device_ && req_) (void)hipFree(req_);
  if (stream_) (void)hipStreamDestroy((hipStream_t)stream_);
}

void HttpRing::open(Engine& e, uint32_t workgroups, uint32_t slots) {
  if (workgroups < 1 || workgroups > 256) fail(CG_INVALID_ARGUMENT, "ring workgroups must be 1..256");
  if (slots < 1 || slots > 64 * workgroups) fail(CG_INVALID_ARGUMENT, "ring slots must be 1..64 * workgroups");
  e.set_device();
  device_ = e.device;
  nwg_ = workgroups;
  nslots_ = slots;
  hip_check(hipStreamCreateWithFlags((hipStream_t*)&stream_, hipStreamNonBlocking), "hipStreamCreate");
  {
    const char* w = getenv("CILIUM_GPU_RING_SLOTS");
    if (!(w && !strcmp(w, "host"))) req_ = device_slots_for_host((size_t)slots * kRingSlotBytes);
    req_in_device_ = req_ != nullptr;
  }
  rep_stride_ = req_in_device_ ? kRingReplyBytes : kRingSlotBytes;
  const size_t bytes = kRingCtlBytes + (size_t)slots * rep_stride_;
  hip_check(hipHostMalloc((void**)&host_, bytes, hipHostMallocCoherent | hipHostMallocMapped), "hipHostMalloc");
  memset(host_, 0, bytes);
  hip_check(hipHostGetDevicePointer((void**)&dev_view_, host_, 0), "hipHostGetDevicePointer");
  rep_ = host_ + kRingCtlBytes;
  rep_dev_ = dev_view_ + kRingCtlBytes;
  if (req_in_device_) {
    hip_check(hipMemset(req_, 0, (size_t)slots * kRingSlotBytes), "hipMemset");
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    req_dev_ = req_;
  } else {
    req_ = rep_;
    req_dev_ = rep_dev_;
  }
  hip_check(hipMalloc(&state_, http_ring_state_bytes()), "hipMalloc");
  // the rate of the kernel's wall_clock64(), measured (two reads 20 ms apart)
  // rather than taken from hipDeviceAttributeWallClockRate
  {
    auto* d = static_cast<unsigned long long*>(state_);
    unsigned long long c[2] = {0, 0};
    uint64_t t[2] = {0, 0};
    for (int k = 0; k < 2; ++k) {
      if (k) std::this_thread::sleep_for(std::chrono::milliseconds(20));
      hip_check(ring_clock(d, stream_), "ring clock");
      hip_check(hipStreamSynchronize((hipStream_t)stream_), "ring clock");
      t[k] = now_ns();
      hip_check(hipMemcpy(&c[k], d, 8, hipMemcpyDeviceToHost), "D2H");
    }
    const double khz = (double)(c[1] - c[0]) / ((double)(t[1] - t[0]) * 1e-6);
    clock_khz_ = khz > 1000.0 ? (uint64_t)khz : 100000;
    if (e.debug || getenv("CILIUM_GPU_DEBUG"))
      fprintf(stderr, "[cilium-gpu] ring: device wall clock %.0f kHz (attribute %d kHz)\n", khz,
              [&] {
                int a = 0;
                (void)hipDeviceGetAttribute(&a, hipDeviceAttributeWallClockRate, device_);
                return a;
              }());
  }
  slot_st_.reset(new SlotState[slots]);
  busy_.reset(new Busy[workgroups]);
  trace_ = getenv("CILIUM_GPU_RING_TRACE") != nullptr;
  if (e.debug || getenv("CILIUM_GPU_DEBUG"))
    fprintf(stderr, "[cilium-gpu] ring: %u workgroups, %u slots, request slots in %s memory\n", nwg_, nslots_,
            req_in_device_ ? "device" : "host");
}

bool HttpRing::stream_idle() const { return hipStreamQuery((hipStream_t)stream_) == hipSuccess; }

// Stop the running launch (if any) and wait for it; mu_ held.
void HttpRing::stop_locked() {
  if (!launched_) return;
  __atomic_store_n(reinterpret_cast<uint32_t*>(host_) + kRingStop, 1u, __ATOMIC_SEQ_CST);
  hip_check(hipStreamSynchronize((hipStream_t)stream_), "ring stop");
  __atomic_store_n(reinterpret_cast<uint32_t*>(host_) + kRingStop, 0u, __ATOMIC_SEQ_CST);
  launched_ = false;
  snap_.reset();
}

void HttpRing::stop_locked_noexcept() {
  std::lock_guard<std::mutex> lk(mu_);
  try {
    if (host_ && stream_) stop_locked();
  } catch (...) {
  }
}

void HttpRing::launch_locked(const std::shared_ptr<HttpSnapshot>& s) {
  // the previous launch has ended (stop_locked, or it left by itself)
  hip_check(hipStreamSynchronize((hipStream_t)stream_), "ring launch");
  if (launches_) {  // keep its served count
    unsigned long long st[3] = {0, 0, 0};
    hip_check(hipMemcpy(st, state_, sizeof(st), hipMemcpyDeviceToHost), "D2H");
    served_before_ += st[2];
  }
  hip_check(hipMemsetAsync(state_, 0, http_ring_state_bytes(), (hipStream_t)stream_), "hipMemsetAsync");
  HttpRingDev G{};
  G.slots = req_dev_;
  G.reply = rep_dev_;
  G.reply_stride = (uint32_t)rep_stride_;
  G.ctl = reinterpret_cast<uint32_t*>(dev_view_);
  G.nslots = nslots_;
  G.nwg = nwg_;
  G.idle_ticks = clock_khz_ * kIdleMs;
  G.life_ticks = clock_khz_ * kLifeMs;
  // the largest walked, rebased program that fits beside the slot and spans
  uint32_t maxc = 0;
  for (const auto& pg : s->progs)
    if (!(pg.flags & kProgAllowAll) && (pg.flags & kProgRebased)) maxc = std::max(maxc, pg.cell_count);
  // the list parser's lookup tables (program lookup, name keys) go to LDS too
  // when the largest program still fits beside them (a single-request call
  // then reads no table from global memory), or when they are small anyway
  G.lds_tabs = ring_tables_small(s->raw) || ring_lds_bytes(s->raw, maxc, true) <= 160 * 1024;
  const size_t base = ring_lds_bytes(s->raw, 0, G.lds_tabs != 0);
  const uint32_t room = base < 160 * 1024 ? (uint32_t)((160 * 1024 - base) / 4) : 0u;
  G.lds_cells = std::min(maxc, room);
  if (getenv("CILIUM_GPU_DEBUG"))
    fprintf(stderr, "[cilium-gpu] ring launch: tables %s LDS, largest program %u cells, %u staged cells at most\n",
            G.lds_tabs ? "in" : "not in", maxc, G.lds_cells);
  G.trace = trace_;
  {
    const char* ec = getenv("CILIUM_GPU_RING_ECHO");  // (measuring only: no verdicts are decided)
    G.echo = ec ? (uint32_t)atoi(ec) : 0u;
  }
  check_launch_rc(launch_http_ring(s->dev, s->raw, G, state_, stream_));
  s->fence.record(stream_);
  snap_ = s;
  snap_ptr_.store(s.get(), std::memory_order_release);
  launched_.store(true, std::memory_order_release);
  launch_ns_.store(now_ns(), std::memory_order_relaxed);
  ++launches_;
}

void HttpRing::check_launch_rc(int rc) { hip_check(rc, "ring kernel launch"); }

// A launch with snapshot s is running (or about to) when this returns.
void HttpRing::ensure(const std::shared_ptr<HttpSnapshot>& s) {
  const uint64_t t = now_ns();
  // fast path: the same tables, served a call recently enough that the
  // launch cannot have idled out, and young enough not to have hit its life
  if (launched_.load(std::memory_order_acquire) && snap_ptr_.load(std::memory_order_acquire) == s.get() &&
      t - last_ns_.load(std::memory_order_relaxed) < (uint64_t)kIdleMs * 500000ull &&
      t - launch_ns_.load(std::memory_order_relaxed) < (uint64_t)kLifeMs * 500000ull)
    return;
  std::lock_guard<std::mutex> lk(mu_);
  if (snap_ != s) {
    stop_locked();
    launch_locked(s);
  } else if (!launched_ || stream_idle()) {
    launched_ = false;
    launch_locked(s);
  }
  snap_ptr_.store(s.get(), std::memory_order_release);
}

void HttpRing::verdicts(Engine& e, const std::shared_ptr<HttpSnapshot>& s, const uint8_t* blob, const uint64_t* off,
                        size_t n, const uint32_t* pol, const uint8_t* ing, const uint16_t* port, const uint32_t* rem,
                        uint8_t* out) {
  (void)e;
  ensure(s);
  // a free slot (callers never hold more than one), preferably one of the
  // home workgroup of the first request's program (its index modulo the
  // workgroups): slot s is served by workgroup s % nwg, which keeps the last
  // program it staged in LDS, so calls of one listener find theirs there
  const uint32_t prog = n ? s->lookup_prog(pol[0], ing[0] != 0, port[0]) : 0u;
  const uint32_t home = (prog < s->progs.size() ? prog : prog * 0x9E3779B1u >> 7) % nwg_;
  // a rotating start per calling thread (no counter shared by the callers)
  thread_local uint32_t next = 0;
  const uint32_t r = next++;
  uint32_t i = nslots_;
  auto try_wg = [&](uint32_t wg) {  // a free slot of workgroup wg (slots wg, wg + nwg, ...)
    const uint32_t mine = wg < nslots_ ? (nslots_ - wg + nwg_ - 1) / nwg_ : 0u;
    for (uint32_t k = 0; k < mine && i == nslots_; ++k) {
      const uint32_t c = wg + ((r + k) % mine) * nwg_;
      uint32_t z = 0;
      if (slot_st_[c].claimed.compare_exchange_strong(z, 1u, std::memory_order_acquire)) i = c;
    }
  };
  // the home workgroup when no call is in it, else the nearest idle one (a
  // workgroup serves its slots one after another: a hot program spreads over
  // the neighbours, which then hold it too), else home, else any slot
  if (!busy_[home].n.load(std::memory_order_relaxed)) try_wg(home);
  for (uint32_t d = 1; d < nwg_ && i == nslots_; ++d)
    if (!busy_[(home + d) % nwg_].n.load(std::memory_order_relaxed)) try_wg((home + d) % nwg_);
  if (i == nslots_) try_wg(home);
  for (uint32_t k = 1; i == nslots_; ++k) {
    const uint32_t c = (r + k) % nslots_;
    uint32_t z = 0;
    if (slot_st_[c].claimed.compare_exchange_strong(z, 1u, std::memory_order_acquire)) i = c;
    if (k % nslots_ == 0) std::this_thread::yield();
  }
  busy_[i % nwg_].n.fetch_add(1, std::memory_order_relaxed);
  uint8_t* sl = req_slot(i);
  uint8_t* rp = rep_slot(i);
  uint8_t* d = sl + kRingData;
  const RingLayout L = ring_layout((uint32_t)n);
  const uint64_t a0 = off[0];
  const uint32_t bytes = (uint32_t)(off[n] - a0);
  memcpy(d, pol, n * 4);
  memcpy(d + L.rem, rem, n * 4);
  memcpy(d + L.port, port, n * 2);
  memcpy(d + L.ing, ing, n);
  uint32_t* o = reinterpret_cast<uint32_t*>(d + L.off);
  for (size_t k = 0; k <= n; ++k) o[k] = (uint32_t)(off[k] - a0);
  if (bytes) memcpy(d + L.blob, blob + a0, bytes);
  uint32_t* w = reinterpret_cast<uint32_t*>(sl);   // request header
  uint32_t* rw = reinterpret_cast<uint32_t*>(rp);  // reply header: done, stamps
  w[2] = (uint32_t)n;
  w[3] = bytes;
  uint32_t& sq = slot_st_[i].seq;
  const uint32_t seq = ++sq ? sq : ++sq;  // never 0 (the slot's initial done)
  // the doorbell after the slot's bytes: stores to device memory through the
  // mapping may be write-combined, which a release store does not order —
  // fence them, store, and fence again so the doorbell leaves at once
  __builtin_ia32_sfence();
  __atomic_store_n(&w[0], seq, __ATOMIC_RELEASE);
  __builtin_ia32_sfence();
  const uint64_t t0 = now_ns();
  uint64_t checked = t0;
  while (__atomic_load_n(&rw[1], __ATOMIC_ACQUIRE) != seq) {
    cpu_relax();
    const uint64_t t = now_ns();
    // past the device's usual time, spin yielding the core: callers on every
    // core (Envoy's workers) must not keep one another's turn waiting
    if (t - t0 > 6000) std::this_thread::yield();
    if (t - checked < 20000) continue;
    checked = t;
    // not served within 20 us: the launch may have left (idle or life)
    // between ensure() and the doorbell — relaunch, the slot is still ready
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (__atomic_load_n(&rw[1], __ATOMIC_ACQUIRE) == seq) break;
      if (stream_idle()) {
        launched_ = false;
        launch_locked(snap_ ? snap_ : s);
      }
    }
    if (t - t0 > 5ull * 1000 * 1000 * 1000) {
      busy_[i % nwg_].n.fetch_sub(1, std::memory_order_relaxed);
      slot_st_[i].claimed.store(0, std::memory_order_release);
      fail(CG_UNKNOWN_ERROR, "ring: a call was not served within 5 s");
    }
  }
  memcpy(out, rp + kRingOut, n);
  const uint64_t t_done = now_ns();
  // (written at most once a millisecond: every caller reads it)
  if (t_done - last_ns_.load(std::memory_order_relaxed) > 1000000) last_ns_.store(t_done, std::memory_order_relaxed);
  if (trace_) {  // device phases (10 ns ticks at 100 MHz) and the whole call
    uint32_t st[kRingStamps + 1];
    for (uint32_t j = 0; j <= kRingStamps; ++j) st[j] = __atomic_load_n(&rw[kRingStampAt + j], __ATOMIC_ACQUIRE);
    std::lock_guard<std::mutex> lk(trace_mu_);
    const double ns_per_tick = 1e6 / (double)clock_khz_;
    const int c = n == 1 ? 0 : n <= 16 ? 1 : 2;
    for (uint32_t j = 1; j < kRingStamps; ++j)
      trace_sum_[c][j - 1] += (double)(uint32_t)(st[j] - st[j - 1]) * ns_per_tick;
    trace_sum_[c][kRingStamps - 1] += (double)(t_done - t0);
    trace_sum_[c][kRingStamps] += (double)st[kRingStamps];
    ++trace_n_[c];
  }
  busy_[i % nwg_].n.fetch_sub(1, std::memory_order_relaxed);
  slot_st_[i].claimed.store(0, std::memory_order_release);
}

void HttpRing::stats(uint64_t* served, uint64_t* launches) {
  std::lock_guard<std::mutex> lk(mu_);
  if (launches) *launches = launches_;
  if (served) {
    // the running launch's count (its state is reset per launch) plus the
    // finished ones'
    unsigned long long st[3] = {0, 0, 0};
    hip_check(hipMemcpy(st, state_, sizeof(st), hipMemcpyDeviceToHost), "D2H");
    *served = served_before_ + st[2];
  }
}

void HttpRing::close() {
  std::lock_guard<std::mutex> lk(mu_);
  stop_locked();
  static const char* const kClass[3] = {"1", "2-16", "17-256"};
  for (int c = 0; c < 3 && trace_; ++c) {
    if (!trace_n_[c]) continue;
    const double k = 1e-3 / (double)trace_n_[c];
    const double* t = trace_sum_[c];
    fprintf(stderr,
            "[cilium-gpu] ring trace, calls of %s requests (%llu), mean us: copy-in+masks %.2f, lookup+stage %.2f, "
            "parse (request 0) %.2f, walk and the rest %.2f, release %.2f, whole call (host) %.2f; shader clock "
            "%.0f MHz\n",
            kClass[c], (unsigned long long)trace_n_[c], t[0] * k, t[1] * k, t[2] * k, t[3] * k + t[4] * k, t[5] * k,
            t[6] * k, t[kRingStamps] * 1e3 / (t[0] + t[1] + t[2] + t[3] + t[4] + t[5]));
  }
}

}  // namespace cg
