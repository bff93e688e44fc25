// kernels.h — host-callable launchers of the gfx950 kernels (kernels.hip).
#pragma once

#include <cstddef>
#include <cstdint>

#include "dev_types.h"

namespace cg {

// All launchers enqueue on `stream` (hipStream_t) and return the hipError_t
// of the launch.  n == 0 launches nothing.
// mode: CG_L4_CAN_ACCESS / CG_L4_INGRESS / CG_L4_EGRESS [| CG_L4_IGNORE_DROP].
int launch_l4(const L4Dev& t, const void* tuples, size_t n, int32_t* out, uint32_t mode, void* stream, int cus);
// launch_l4 with each tuple's identity taken from the ipcache resolution of
// addrs[i] (remote address, network order: u32 for family 4, 16 bytes for 6).
int launch_l4_ipcache(const L4Dev& t, const IpcacheDev& ipc, int family, const void* addrs, const void* tuples,
                      size_t n, int32_t* out, uint32_t mode, void* stream, int cus);
int launch_lpm(const LpmDev& t, bool v4_filter, bool v6_filter, const uint32_t* v4, size_t n4,
               uint8_t* out4, const uint8_t* v6, size_t n6, uint8_t* out6, void* stream, int cus);
// order (optional): out[order[slot]] instead of out[slot] (request order;
// an entry >= nout, e.g. 0xFFFFFFFF = padding, writes nothing) — the
// raw-request batches.
// rule (optional): per slot (or order[slot]) the first matching rule's
// counter index, 0xFFFFFFFF when no rule allows.
// codes (optional): the batch's strings are raw bytes (the device-layout raw
// path writes them uncoded) and class-mode programs code them through these
// per-program 256-byte maps (HttpRawDev.codes) as they walk.
int launch_http(const HttpDev& t, const void* records, size_t n, const uint8_t* arena, uint8_t* out,
                void* stream, int cus, const uint32_t* order = nullptr, uint32_t* rule = nullptr,
                uint32_t nout = 0xFFFFFFFFu, const uint8_t* codes = nullptr);
int launch_ipcache(const IpcacheDev& t, const uint32_t* v4, size_t n4, IpcVal* out4, const uint8_t* v6, size_t n6,
                   IpcVal* out6, void* stream, int cus);
// tails (optional): the split layout — reqs holds 16-byte heads, tails the
// 48-byte topic ids of each request (cg_kafka_verdicts_split_*).
int launch_kafka(const KafkaDev& t, const void* reqs, size_t n, const uint32_t* arena, uint8_t* out,
                 void* stream, int cus, const void* tails = nullptr);
// Kafka wire decode (kernels_kafka.hip): records + statuses (kKwDefer for the
// host to finish); ctr[0] arena entries reserved, ctr[1] deferred requests
// (both zeroed by the caller).
int launch_kafka_decode(const KafkaDictDev& topics, const KafkaDictDev& clients, const uint8_t* raw,
                        const uint64_t* off, size_t n, const uint16_t* redirect, const uint32_t* remote, void* recs,
                        uint32_t* arena, size_t arena_cap, unsigned long long* ctr, uint8_t* status, void* stream,
                        int cus, uint32_t* defer_list, uint8_t* zarena, size_t zcap);

// Raw HTTP/1 heads → batch (kernels_http_raw.hip; sequence in http_raw.cc).
// The scan and rank kernels run http_raw_grid(R, lists, n, cus) blocks over the
// requests in the same order.  With http_raw_lds_keys(R) the scan writes
// per-block bucket counts (counts[key * grid + block]) and raw_prefix turns
// them into per-block slot offsets (bbase) and totals (hist); otherwise the
// scan adds into a global histogram (counts = hist) and the rank takes slots
// from global cursors.  sbuf: the request-ordered string buffer
// (records per request, http_raw.cc), cst its per-request stride.  lists:
// the requests are cg_http_pack header lists instead of HTTP/1 heads (a list
// longer than kFieldsMaxList sets kRawListTooLong in *ovf_bytes).  Requests
// outside their wave's LDS stage are appended to dlist (*dcount, zeroed by
// the caller; room for n) and finished by a second kernel of the launch.
constexpr unsigned long long kRawListTooLong = 1ull << 63;
size_t http_raw_grid(const HttpRawDev& R, bool lists, size_t n, int cus);
bool http_raw_lds_keys(const HttpRawDev& R);
int launch_http_raw_scan(const HttpRawDev& R, bool lists, const uint8_t* raw, const uint64_t* off, size_t n,
                         const uint32_t* policy, const uint8_t* ingress, const uint16_t* port, uint32_t* counts,
                         void* rinfo, const uint32_t* remote, uint8_t* sbuf, uint32_t cst,
                         unsigned long long* ovf_bytes, uint32_t* dlist, uint32_t* dcount, void* stream, int cus);
int launch_http_raw_prefix(const uint32_t* bcount, uint32_t nkeys, uint32_t nblk, uint32_t* bbase, uint32_t* hist,
                           void* stream);
int launch_http_raw_rank(const HttpRawDev& R, bool lists, size_t n, const void* rinfo, uint32_t* cursor,
                         const uint32_t* bbase, uint32_t* order, void* stream, int cus);
int launch_http_raw_build(const HttpRawDev& R, const HttpRawRun* runs, uint32_t nruns, uint32_t ntiles,
                          HttpTile* ttab, uint8_t* tiles, uint32_t* order, const uint8_t* sbuf, uint8_t* arena,
                          unsigned long long* arena_cursor, void* stream, int cus);

// The device-layout path (CILIUM_GPU_RAW_LAYOUT=device; sequence, all on
// one stream with no host round trip, in http_raw.cc):
// launch_http_raw_dl_scan (scan + deferred requests) puts each request into its
// slot of the batch laid out by L (dev_types.h RawLayoutDev) or on L's walk
// list; launch_http_raw_seal pads the last tiles and writes the chunk table
// and header; then launch_http over the batch (order = L.order) and
// launch_http_raw_walk for the walk list.  lists: the requests are
// cg_http_pack header lists instead of HTTP/1 heads.
size_t http_raw_dl_grid(const HttpRawDev& R, bool lists, size_t n, int cus);
bool http_raw_seal_sorts(const HttpRawDev& R);
int launch_http_raw_dl_scan(const HttpRawDev& R, bool lists, const uint8_t* raw, const uint64_t* off, size_t n,
                            const uint32_t* policy, const uint8_t* ingress, const uint16_t* port,
                            const uint32_t* remote, const RawLayoutDev& L, void* stream, int cus);
int launch_http_raw_seal(const HttpRawDev& R, const RawLayoutDev& L, void* batch, uint32_t epoch, uint64_t ttab_off,
                         uint64_t tiles_off, uint64_t total_bytes, void* stream);
int launch_http_raw_walk(const HttpDev& T, const HttpRawDev& R, bool lists, const uint8_t* raw, const uint64_t* off,
                         const uint32_t* policy, const uint8_t* ingress, const uint16_t* port, const uint32_t* remote,
                         const RawLayoutDev& L, uint8_t* out, void* stream, int cus);

// The persistent verdict ring (ring.cc): nwg one-wave workgroups serving
// the slots of G until its stop word, idle_ticks without a call or
// life_ticks; `state` is http_ring_state_bytes() of zeroed device memory.
// LDS of the ring kernel: `cells` of program block, the list parser's tables
// when `tabs`; ring_tables_small: tables small enough to stage always
size_t ring_lds_bytes(const HttpRawDev& R, uint32_t cells, bool tabs);
bool ring_tables_small(const HttpRawDev& R);
size_t http_ring_state_bytes();
int launch_http_ring(const HttpDev& HT, const HttpRawDev& R, const HttpRingDev& G, void* state, void* stream);
// the device's wall_clock64() into *d_out (ring.cc measures its rate)
int ring_clock(unsigned long long* d_out, void* stream);

}  // namespace cg
