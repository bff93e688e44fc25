// http.h — HTTP L7 policy snapshot: NPDS JSON → programs of union DFAs.
#pragma once

#include <array>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "dev_types.h"
#include "engine.h"

namespace cg {

struct HttpSnapshot {
  std::vector<std::string> fields;  // walked fields, canonical order, lowercase
  // proxylib snapshot: field values are arbitrary bytes, given escaped (bytes
  // 0x00-0x03 as 0x03, 0x10 + b; regex.h kEscByte) and never codec-rejected
  bool raw_values = false;
  std::map<std::string, uint32_t> policy_index;
  uint32_t npolicies = 0;

  std::vector<HttpProg> progs;
  std::vector<HttpPart> parts;
  std::vector<uint32_t> cells;
  std::vector<uint32_t> phash_keys, phash_vals;
  uint32_t phash_mask = 0;
  std::vector<uint32_t> dflt;
  // (policy, ingress, port) of each program, for counter attribution
  std::vector<uint32_t> prog_key;
  // class-mode programs (kProgClass): string byte b is packed as code[b]
  std::vector<std::array<uint8_t, 256>> prog_code;
  // what each per-rule hit counter counts (HttpProg.rule_base + bit)
  std::vector<cg_http_rule_info> rule_info;

  uint32_t epoch = 0;
  uint64_t total_states = 0;
  uint64_t total_exceptions = 0;
  uint64_t total_rules = 0;
  uint64_t total_remote_slots = 0;

  DevMem d_progs, d_parts, d_cells, d_dflt, d_counters;
  HttpDev dev{};
  // raw HTTP/1 heads and header lists on the device (http_raw.cc): tables
  // set by upload when the snapshot has at most kRawMaxFields fields; raw
  // heads also need a non-proxylib snapshot
  DevMem d_phk, d_phv, d_fslots, d_fnames, d_codes, d_nkeys, d_walk;
  HttpRawDev raw{};
  bool raw_ok = false, lists_ok = false;
  LaunchFence fence;  // last member: queued kernels finish before the buffers go (engine.h)

  void upload(Engine& e);
  uint32_t lookup_prog(uint32_t policy, bool ingress, uint32_t port) const;
};

std::shared_ptr<HttpSnapshot> http_compile(const char* json, size_t len);
// A fresh batch epoch (packed batches carry the epoch of their snapshot).
uint32_t http_next_epoch();
// The compiled snapshot as a flat image and back (http_image.cc): compile
// once, publish the same tables on every GPU / process.
std::vector<uint8_t> http_image_export(const HttpSnapshot& s);
std::shared_ptr<HttpSnapshot> http_image_import(const uint8_t* p, size_t n);

// NPDS wire form (serialized DiscoveryResponse of cilium.NetworkPolicy) →
// the NPDS JSON http_compile and the proxylib translation read (npds_pb.cc).
std::string npds_pb_to_json(const uint8_t* p, size_t n, bool strict_utf8);

// The raw-head path (http_raw.cc): device tables (called by upload), and
// verdicts for n requests already in device memory, in request order, on
// `stream` with the lease's workspace (synchronizes it).  Request i is
// d_raw[d_off[i], d_off[i+1]): an HTTP/1 head (RawInput::Heads) or a
// cg_http_pack header list "name\0value\0..." (RawInput::Lists).
enum class RawInput { Heads, Lists };
void http_raw_upload(HttpSnapshot& S);
void http_verdicts_raw_on(const HttpSnapshot& s, StagingSlot& sl, int cus, RawInput in, const uint8_t* d_raw,
                          const uint64_t* d_off, size_t n, const uint32_t* d_policy, const uint8_t* d_ingress,
                          const uint16_t* d_port, const uint32_t* d_remote, uint8_t* d_out, void* stream);

// Upper bounds of a packed batch of n requests (slots, bytes).
size_t http_batch_slots(const HttpSnapshot& s, size_t n);
size_t http_batch_bytes(const HttpSnapshot& s, size_t n);

// Pack requests into a program-grouped batch (dev_types.h HttpBatchHeader).
// order[slot] = request index, or UINT32_MAX for a padding slot.
void http_pack(const HttpSnapshot& s, size_t n, const uint32_t* policy, const uint8_t* ingress,
               const uint16_t* port, const uint32_t* remote, const uint8_t* hdr_blob,
               const uint64_t* hdr_off, void* batch, size_t batch_cap, uint32_t* order, size_t* nslots,
               uint8_t* arena, size_t arena_cap, size_t* arena_used);

// Walk the snapshot's tables on the host exactly as the kernel does, for
// every slot of a batch (diagnostics / compiler tests only; the verdict API
// never calls this).  out has one byte per slot.
// rule (optional, one per slot): the global index of the first rule that
// allows the slot (the per-rule hit counter it adds to), or UINT32_MAX.
void http_eval_host(const HttpSnapshot& s, const uint8_t* batch, const uint8_t* arena, size_t arena_len,
                    uint8_t* out, uint32_t* rule = nullptr);

}  // namespace cg
