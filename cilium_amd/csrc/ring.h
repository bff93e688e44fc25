// ring.h — the persistent verdict ring of a handle (ring.cc).
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <vector>

#include "engine.h"

namespace cg {

struct HttpSnapshot;

class HttpRing {
 public:
  HttpRing() = default;
  HttpRing(const HttpRing&) = delete;
  HttpRing& operator=(const HttpRing&) = delete;
  ~HttpRing();
  void open(Engine& e, uint32_t workgroups, uint32_t slots);
  // n <= kRingReqs lists of at most kRingBlob bytes in all, on a snapshot
  // with lists_ok (the caller checks)
  void verdicts(Engine& e, const std::shared_ptr<HttpSnapshot>& s, const uint8_t* blob, const uint64_t* off, size_t n,
                const uint32_t* pol, const uint8_t* ing, const uint16_t* port, const uint32_t* rem, uint8_t* out);
  void stats(uint64_t* served, uint64_t* launches);
  void close();

 private:
  void ensure(const std::shared_ptr<HttpSnapshot>& s);
  void launch_locked(const std::shared_ptr<HttpSnapshot>& s);
  void stop_locked();
  void stop_locked_noexcept();
  bool stream_idle() const;
  uint8_t* req_slot(uint32_t i) const { return req_ + (size_t)i * kRingSlotBytes; }
  uint8_t* rep_slot(uint32_t i) const { return rep_ + (size_t)i * rep_stride_; }
  static void check_launch_rc(int rc);

  int device_ = 0;
  uint32_t nwg_ = 0, nslots_ = 0;
  uint8_t* host_ = nullptr;      // control words + reply slots (hipHostMalloc, coherent, mapped)
  uint8_t* dev_view_ = nullptr;  // the same memory as the device addresses it
  uint8_t* req_ = nullptr;       // request slots: fine-grained device memory the host writes through its mapping
                                 // (one address for both), or inside host_ (CILIUM_GPU_RING_SLOTS=host)
  uint8_t* req_dev_ = nullptr;   // the request slots as the device addresses them
  uint8_t* rep_ = nullptr;       // reply slots (host_), rep_stride_ apart
  uint8_t* rep_dev_ = nullptr;
  size_t rep_stride_ = 0;
  bool req_in_device_ = false;
  void* state_ = nullptr;        // the launch's RingState (device memory)
  void* stream_ = nullptr;       // hipStream_t of the launches
  uint64_t clock_khz_ = 100000;  // wall clock of the device (hipDeviceAttributeWallClockRate)
  std::mutex mu_;                // launches, stops, stats
  std::shared_ptr<HttpSnapshot> snap_;  // the running launch's tables
  std::atomic<const HttpSnapshot*> snap_ptr_{nullptr};
  std::atomic<bool> launched_{false};
  std::atomic<uint64_t> launch_ns_{0}, last_ns_{0};
  uint64_t launches_ = 0, served_before_ = 0;
  // per slot, a cache line of its own (callers on many cores claim slots
  // side by side): the claim and the slot's last doorbell value
  struct alignas(64) SlotState {
    std::atomic<uint32_t> claimed{0};  // a call owns the slot
    uint32_t seq = 0;                  // under the claim
  };
  std::unique_ptr<SlotState[]> slot_st_;
  // per workgroup: calls in its slots, a cache line each (callers on many
  // cores add and drop theirs on every call; a scan for an idle neighbour
  // reads only as far as the first idle one)
  struct alignas(64) Busy {
    std::atomic<uint32_t> n{0};
  };
  std::unique_ptr<Busy[]> busy_;
  // CILIUM_GPU_RING_TRACE: per-phase device stamps summed over calls
  bool trace_ = false;
  std::mutex trace_mu_;
  // per call-size class (1, 2..16, 17..256 requests): phase sums, calls
  double trace_sum_[3][kRingStamps + 1] = {};  // + shader clock cycles
  uint64_t trace_n_[3] = {0, 0, 0};
};

}  // namespace cg
