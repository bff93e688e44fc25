/*
 * cilium_gpu.h — C ABI of libciliumgpu.so, the MI355X (gfx950) batched
 * policy-verdict engine.
 *
 * This is the drop-in boundary for Cilium's data-parallel classification path
 * (SURVEY.md §8).  Every entry point is plain C: integers, pointers and sizes;
 * no C++ or torch types cross it.  Conventions kept from the reference:
 *
 *  - Return codes reuse proxylib's FilterResult numbering for the shared
 *    values (proxylib/proxylib/types.h:38-47); engine-specific codes start at
 *    16.  Nothing throws across the ABI (proxylib/proxylib/connection.go:119-135
 *    recovers panics into PARSER_ERROR; we return codes).
 *  - Buffers are caller-owned; the library never retains a caller pointer
 *    after a call returns (proxylib/proxylib.go:46-51 copies strings on entry).
 *  - Policy updates are all-or-nothing: the new tables are compiled and
 *    uploaded first, then published by a pointer swap, so a failed update
 *    leaves the previous snapshot serving (proxylib/proxylib/instance.go:180-215,
 *    envoy/cilium_network_policy.cc onConfigUpdate).
 *  - "_dev" verdict calls take DEVICE pointers and a hipStream_t (passed as
 *    void*, NULL = the handle's stream) and are asynchronous; the "_host"
 *    variants take host pointers and return when the verdicts are written.
 *
 * Each declaration cites the reference interface it replaces.
 */
#ifndef CILIUM_GPU_H
#define CILIUM_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Result codes                                                              */
/* ------------------------------------------------------------------------ */
typedef enum {
  CG_OK = 0,                  /* FILTER_OK                 types.h:39 */
  CG_POLICY_DROP = 1,         /* FILTER_POLICY_DROP        types.h:40 */
  CG_PARSER_ERROR = 2,        /* FILTER_PARSER_ERROR       types.h:41 */
  CG_UNKNOWN_PARSER = 3,      /* FILTER_UNKNOWN_PARSER     types.h:42 */
  CG_UNKNOWN_CONNECTION = 4,  /* FILTER_UNKNOWN_CONNECTION types.h:43 */
  CG_INVALID_ADDRESS = 5,     /* FILTER_INVALID_ADDRESS    types.h:44 */
  CG_INVALID_INSTANCE = 6,    /* FILTER_INVALID_INSTANCE   types.h:45 */
  CG_UNKNOWN_ERROR = 7,       /* FILTER_UNKNOWN_ERROR      types.h:46 */
  /* engine-specific */
  CG_INVALID_ARGUMENT = 16,
  CG_NO_DEVICE = 17,          /* no usable gfx950 device / HIP error at open */
  CG_DEVICE_ERROR = 18,       /* a HIP call failed */
  CG_POLICY_REJECTED = 19,    /* policy failed to parse/compile; old snapshot kept */
  CG_REVISION_MISMATCH = 20,  /* prefilter.go:131-133 "Latest revision is %d not %d" */
  CG_MAP_FULL = 21,           /* bpf map E2BIG: more keys than max_entries */
  CG_NOT_FOUND = 22,          /* key/CIDR/policy not present (ENOENT) */
  CG_NO_MAP = 23,             /* prefilter.go:137-139 "No map enabled for CIDR" */
  CG_UNSUPPORTED = 24         /* regex construct outside the supported subset */
} cg_result;

typedef struct {
  const char* key;
  const char* value;
} cg_kv;

/* ------------------------------------------------------------------------ */
/* Module lifetime — replaces proxylib OpenModule/CloseModule                */
/* (proxylib/libcilium.h:107-115, proxylib/proxylib.go:118-155).             */
/* params: "device" = HIP device ordinal (default "0").                      */
/* Returns 0 on error (same convention as OpenModule).  Host-only work       */
/* (policy compilation, table builds) works on a handle opened with          */
/* "device" = "-1" (no GPU); verdict calls on such a handle return           */
/* CG_NO_DEVICE — there is no CPU fallback.                                  */
/* ------------------------------------------------------------------------ */
uint64_t cg_open(const cg_kv* params, size_t n_params, uint8_t debug);
void cg_close(uint64_t h);
/* Last error message of the calling thread (static storage, never NULL). */
const char* cg_last_error(void);
/* Library/kernels build string, e.g. "libciliumgpu gfx950 r1". */
const char* cg_version(void);

/* ======================================================================== */
/* L4: policymap verdicts — bpf/lib/policy.h:46-163                          */
/* ======================================================================== */

/* struct policy_key, bpf/lib/common.h:180-186; Go PolicyKey,
 * pkg/maps/policymap/policymap.go:64-69.  dport in NETWORK byte order. */
typedef struct {
  uint32_t sec_label;
  uint16_t dport;     /* network byte order */
  uint8_t protocol;   /* u8proto: TCP=6, UDP=17 (pkg/u8proto/u8proto.go:27-28) */
  uint8_t egress;     /* bit0: TrafficDirection Ingress=0/Egress=1 (trafficdirection.go:20-29) */
} cg_policy_key;

/* struct policy_entry, bpf/lib/common.h:188-193; Go PolicyEntry,
 * policymap.go:73-80.  proxy_port in NETWORK byte order. */
typedef struct {
  uint16_t proxy_port; /* network byte order */
  uint16_t pad[3];
  uint64_t packets;
  uint64_t bytes;
} cg_policy_entry;

/* One packet to classify: the arguments of __policy_can_access
 * (bpf/lib/policy.h:46-49) that reach the verdict, packed to 12 bytes. */
typedef struct {
  uint32_t identity;   /* sec_label of the remote endpoint */
  uint16_t dport;      /* network byte order (tuple.dport) */
  uint8_t proto;       /* tuple.nexthdr */
  uint8_t flags;       /* CG_L4_F_* */
  uint32_t len;        /* skb->len, added to policy_entry.bytes on a hit */
} cg_l4_tuple;

#define CG_L4_F_INGRESS 0x01u   /* dir == CT_INGRESS (common.h:328); else CT_EGRESS */
#define CG_L4_F_FRAGMENT 0x02u  /* is_fragment */
#define CG_L4_F_CB_POLICY 0x04u /* skb->cb[CB_POLICY] set (policy.h:98) */

/* Verdict values written per tuple (int32), identical to the return of
 * __policy_can_access: >0 proxy_port as stored (network order, read as a
 * host u16), 0 = TC_ACT_OK, DROP_POLICY = -133 (common.h:240),
 * DROP_FRAG_NOSUPPORT = -157 (common.h:264). */
#define CG_DROP_POLICY (-133)
#define CG_DROP_FRAG_NOSUPPORT (-157)

/* Policy maps — one per endpoint, like cilium_policy_<epid>.
 * max_entries: 0 = PolicyMap MaxEntries 16384 (policymap.go:37). */
int cg_policymap_create(uint64_t h, uint32_t max_entries, uint32_t* map_id);
int cg_policymap_destroy(uint64_t h, uint32_t map_id);
/* PolicyMap.AllowKey/Allow (policymap.go:162-176): insert or update
 * proxy_port (network order) for each key.  Existing counters are kept.
 * CG_MAP_FULL if a new key would exceed max_entries (nothing applied). */
int cg_policymap_allow(uint64_t h, uint32_t map_id, const cg_policy_key* keys,
                       const uint16_t* proxy_ports_be, size_t n);
/* PolicyMap.DeleteKey/Delete (policymap.go:187-199); CG_NOT_FOUND if any key
 * is absent (nothing applied). */
int cg_policymap_delete(uint64_t h, uint32_t map_id, const cg_policy_key* keys, size_t n);
/* PolicyMap.Exists + LookupElement (policymap.go:181-185). */
int cg_policymap_lookup(uint64_t h, uint32_t map_id, const cg_policy_key* key,
                        cg_policy_entry* entry);
/* PolicyMap.DumpToSlice (policymap.go:224-255).  Writes up to cap entries,
 * sets *n to the number of entries in the map. */
int cg_policymap_dump(uint64_t h, uint32_t map_id, cg_policy_key* keys,
                      cg_policy_entry* entries, size_t cap, size_t* n);
/* PolicyMap.Flush (policymap.go:257-280). */
int cg_policymap_flush(uint64_t h, uint32_t map_id);

/* Batched policy_can_access over tuples (policy.h:46-110).  Counters of the
 * matching entry advance exactly as the BPF code's __sync_fetch_and_add
 * (policy.h:68-69,80-81,92-93).  Device pointers, async on stream. */
int cg_l4_verdicts_dev(uint64_t h, uint32_t map_id, const cg_l4_tuple* d_tuples,
                       size_t n, int32_t* d_verdicts, void* stream);
int cg_l4_verdicts_host(uint64_t h, uint32_t map_id, const cg_l4_tuple* tuples,
                        size_t n, int32_t* verdicts);

/* The verdict wrappers around __policy_can_access (bpf/lib/policy.h:126-163),
 * selected by `mode`:
 *   CG_L4_CAN_ACCESS  __policy_can_access itself: each tuple's CG_L4_F_INGRESS
 *                     and CG_L4_F_FRAGMENT flags (what cg_l4_verdicts_* do);
 *   CG_L4_INGRESS     policy_can_access_ingress (policy.h:126-146, called at
 *                     bpf_lxc.c:814,948): dir = CT_INGRESS for every tuple,
 *                     the tuple's is_fragment; any negative result becomes
 *                     DROP_POLICY (so an unmatched fragment is -133, not -157);
 *   CG_L4_EGRESS      policy_can_egress (policy.h:150-163, via
 *                     policy_can_egress{4,6} at bpf_lxc.c:220,527): dir =
 *                     CT_EGRESS, is_fragment = false; negative → DROP_POLICY.
 * OR CG_L4_IGNORE_DROP to model a datapath built with IGNORE_DROP: the
 * wrappers then return TC_ACT_OK instead of DROP_POLICY.  CG_L4_F_CB_POLICY
 * (skb->cb[CB_POLICY]) is honoured in every mode, as in policy.h:98. */
#define CG_L4_CAN_ACCESS 0u
#define CG_L4_INGRESS 1u
#define CG_L4_EGRESS 2u
#define CG_L4_IGNORE_DROP 0x100u
int cg_l4_policy_verdicts_dev(uint64_t h, uint32_t map_id, uint32_t mode, const cg_l4_tuple* d_tuples,
                              size_t n, int32_t* d_verdicts, void* stream);
int cg_l4_policy_verdicts_host(uint64_t h, uint32_t map_id, uint32_t mode, const cg_l4_tuple* tuples,
                               size_t n, int32_t* verdicts);

/* ======================================================================== */
/* LPM: XDP CIDR prefilter — bpf/bpf_xdp.c:88-184,                           */
/* pkg/datapath/prefilter/prefilter.go:57-298                                */
/* ======================================================================== */

/* A CIDR as the agent holds it (net.IPNet; cidrKey cidrmap.go:52-64). */
typedef struct {
  uint8_t family;     /* 4 or 6 */
  uint8_t prefixlen;  /* ones of the mask */
  uint8_t pad[2];
  uint8_t addr[16];   /* network byte order; v4 uses addr[0..3] */
} cg_cidr;

/* preFilterConfig (prefilter.go:49-54); NewPreFilter default is fix4|fix6
 * with dyn maps disabled (prefilter.go:281-298). */
#define CG_PF_DYN4 0x1u
#define CG_PF_DYN6 0x2u
#define CG_PF_FIX4 0x4u
#define CG_PF_FIX6 0x8u

/* XDP verdicts written per address (linux enum xdp_action). */
#define CG_XDP_DROP 1
#define CG_XDP_PASS 2

/* NewPreFilter.  max_lpm/max_hash: 0 = maxLKeys 65536 / maxHKeys 20M
 * (prefilter.go:43-44).  Revision starts at 1 (prefilter.go:291). */
int cg_prefilter_create(uint64_t h, uint32_t config, uint32_t max_lpm, uint32_t max_hash,
                        uint32_t* pf_id);
int cg_prefilter_destroy(uint64_t h, uint32_t pf_id);
/* PreFilter.Insert (prefilter.go:125-159): revision check (0 = any), per-CIDR
 * map selection (selectMap :108-122), undo on failure.  *revision_out gets the
 * new revision on success. */
int cg_prefilter_insert(uint64_t h, uint32_t pf_id, int64_t revision, const cg_cidr* cidrs,
                        size_t n, int64_t* revision_out);
/* PreFilter.Delete (prefilter.go:162-203). */
int cg_prefilter_delete(uint64_t h, uint32_t pf_id, int64_t revision, const cg_cidr* cidrs,
                        size_t n, int64_t* revision_out);
/* PreFilter.Dump (prefilter.go:99-106): entries of dyn4, fix4, dyn6, fix6
 * in that map order; *n gets the total. */
int cg_prefilter_dump(uint64_t h, uint32_t pf_id, cg_cidr* out, size_t cap, size_t* n,
                      int64_t* revision);
/* The local endpoint set cilium_lxc consulted by check_v{4,6}_endpoint
 * (bpf_xdp.c:88-95,123-130 → bpf/lib/eps.h:26-46).  Replaces the set. */
int cg_prefilter_set_endpoints(uint64_t h, uint32_t pf_id, const uint32_t* v4_be, size_t n4,
                               const uint8_t* v6, size_t n6);
/* check_v4 / check_v6 (bpf_xdp.c:97-156) over a batch.
 * v4: n4 records of {saddr, daddr} (u32 each, network order as in iphdr);
 * v6: n6 records of {saddr[16], daddr[16]}.  out: one CG_XDP_* byte each. */
int cg_prefilter_verdicts_dev(uint64_t h, uint32_t pf_id, const uint32_t* d_v4, size_t n4,
                              uint8_t* d_out4, const uint8_t* d_v6, size_t n6, uint8_t* d_out6,
                              void* stream);
int cg_prefilter_verdicts_host(uint64_t h, uint32_t pf_id, const uint32_t* v4, size_t n4,
                               uint8_t* out4, const uint8_t* v6, size_t n6, uint8_t* out6);

/* ======================================================================== */
/* ipcache: IP -> security identity (cilium_ipcache, bpf/lib/maps.h:135-159; */
/* pkg/maps/ipcache/ipcache.go:36-130; lookup bpf/lib/eps.h:48-115)         */
/* ======================================================================== */

/* RemoteEndpointInfo (bpf/lib/common.h:175-178, ipcache.go:127-130). */
typedef struct {
  uint32_t sec_label;
  uint32_t tunnel_endpoint;  /* as stored: the node IPv4 address bytes */
} cg_remote_endpoint_info;

/* identity the callers fall back to (bpf/node_config.h:35) */
#define CG_WORLD_ID 2

/* A cilium_ipcache map.  max_entries 0 = MaxEntries 512000 (ipcache.go:36). */
int cg_ipcache_create(uint64_t h, uint32_t max_entries, uint32_t* ipc_id);
int cg_ipcache_destroy(uint64_t h, uint32_t ipc_id);
/* Map.Update of {Key, RemoteEndpointInfo} pairs (ipcache.go NewKey: prefix
 * from the mask, address masked to it, family 4/6).  BPF_ANY semantics: an
 * existing key is overwritten.  All-or-nothing: CG_MAP_FULL when the batch
 * would exceed max_entries, and nothing is applied. */
int cg_ipcache_update(uint64_t h, uint32_t ipc_id, const cg_cidr* keys,
                      const cg_remote_endpoint_info* values, size_t n);
/* Map.Delete; CG_NOT_FOUND (nothing deleted) if any key is absent. */
int cg_ipcache_delete(uint64_t h, uint32_t ipc_id, const cg_cidr* keys, size_t n);
/* Exact-key lookup (bpf map lookup of a full key); CG_NOT_FOUND if absent. */
int cg_ipcache_lookup(uint64_t h, uint32_t ipc_id, const cg_cidr* key, cg_remote_endpoint_info* value);
/* Map.Dump: keys in (family, prefixlen, address) order; *n gets the total. */
int cg_ipcache_dump(uint64_t h, uint32_t ipc_id, cg_cidr* keys, cg_remote_endpoint_info* values,
                    size_t cap, size_t* n);
/* lookup_ip4_remote_endpoint / lookup_ip6_remote_endpoint over a batch,
 * resolved as bpf_lxc.c:509-518 does: the longest covering prefix's
 * {sec_label, tunnel_endpoint} if it exists and sec_label != 0, else
 * {CG_WORLD_ID, 0}.  v4: n4 u32 addresses (network order, as iphdr.daddr);
 * v6: n6 16-byte addresses.  out: one cg_remote_endpoint_info each. */
int cg_ipcache_resolve_dev(uint64_t h, uint32_t ipc_id, const uint32_t* d_v4, size_t n4,
                           cg_remote_endpoint_info* d_out4, const uint8_t* d_v6, size_t n6,
                           cg_remote_endpoint_info* d_out6, void* stream);
int cg_ipcache_resolve_host(uint64_t h, uint32_t ipc_id, const uint32_t* v4, size_t n4,
                            cg_remote_endpoint_info* out4, const uint8_t* v6, size_t n6,
                            cg_remote_endpoint_info* out6);

/* The egress flow of bpf_lxc.c:509-527 over a batch: each tuple's remote
 * identity is lookup_ip4_remote_endpoint(remote_v4[i]) resolved as the
 * datapath does (WORLD_ID on a miss or sec_label 0), then
 * policy_can_egress4 (policy.h:172-176 → policy_can_egress :150-163):
 * dir = CT_EGRESS and is_fragment = false whatever the tuple's flags say,
 * any negative result → DROP_POLICY.  The tuples' identity fields are
 * ignored.  remote_v4: network-order IPv4 addresses (iphdr.daddr).  Counters
 * advance as in cg_l4_verdicts_*. */
int cg_l4_verdicts_ipcache_dev(uint64_t h, uint32_t map_id, uint32_t ipc_id, const uint32_t* d_remote_v4,
                               const cg_l4_tuple* d_tuples, size_t n, int32_t* d_verdicts, void* stream);
int cg_l4_verdicts_ipcache_host(uint64_t h, uint32_t map_id, uint32_t ipc_id, const uint32_t* remote_v4,
                                const cg_l4_tuple* tuples, size_t n, int32_t* verdicts);
/* The IPv6 twin (bpf_lxc.c:205-220: lookup_ip6_remote_endpoint, then
 * policy_can_egress6 → policy_can_egress): remote_v6 holds n 16-byte
 * addresses in network order. */
int cg_l4_verdicts_ipcache6_dev(uint64_t h, uint32_t map_id, uint32_t ipc_id, const uint8_t* d_remote_v6,
                                const cg_l4_tuple* d_tuples, size_t n, int32_t* d_verdicts, void* stream);
int cg_l4_verdicts_ipcache6_host(uint64_t h, uint32_t map_id, uint32_t ipc_id, const uint8_t* remote_v6,
                                 const cg_l4_tuple* tuples, size_t n, int32_t* verdicts);

/* ======================================================================== */
/* proxylib generic L7 (proxylib/proxylib/policymap.go:118-260)              */
/* ======================================================================== */

/* Install the NetworkPolicy list of a proxylib instance (the id OpenModule
 * returned, include/cilium_proxylib.h) — what the reference receives over
 * NPDS (xds-path).  protobuf-JSON form with generic L7 rules:
 *   [{"name": "cp1", "ingress_per_port_policies": [{"port": 80, "rules": [
 *       {"remote_policies": [1], "l7_proto": "r2d2",
 *        "l7_rules": {"l7_rules": [{"rule": {"cmd": "READ", "file": "s.*"}}]}}]}]}]
 * Rule parsers: r2d2 (r2d2parser.go:91-123) and cassandra
 * (cassandraparser.go:97-131); a rule with another l7_proto drops its port
 * (policymap.go:186-204).  ParseError conditions → CG_POLICY_REJECTED and the
 * previous snapshot stays.  Verdict contract: exact port, port 0, else deny. */
int cg_proxylib_policy_update(uint64_t instance, const char* json, size_t len);

/* The proxylib update from the NPDS wire form (a serialized DiscoveryResponse
 * of cilium.NetworkPolicy resources, as Instance.PolicyUpdate receives it,
 * proxylib/proxylib/instance.go:180-215, with the same Validate() rules as
 * cg_http_policy_update_npds). */
int cg_proxylib_policy_update_npds(uint64_t instance, const uint8_t* discovery_response, size_t len);

/* OnData calls with request frames whose verdicts the instance has decided,
 * and the GPU batches that decided them: concurrent calls of different
 * connections share a batch (flat combining; calls > batches under load). */
int cg_proxylib_stats(uint64_t instance, uint64_t* batches, uint64_t* calls);

/* Batching window of the OnData combiner.  A call that finds no batch in
 * flight becomes the flusher; with min_calls > 1 it waits until min_calls
 * calls are queued or max_wait_us microseconds have passed, then decides
 * everything queued as one GPU batch.  Default (1, 0): decide at once.
 * No reference counterpart (Go proxylib decides each frame in the calling
 * goroutine, proxylib/proxylib/connection.go:176-179); a latency/throughput
 * knob for Envoy worker pools. */
int cg_proxylib_set_batching(uint64_t instance, uint32_t min_calls, uint32_t max_wait_us);

/* ======================================================================== */
/* HTTP L7: Envoy cilium.l7policy — envoy/cilium_network_policy.h:40-237,    */
/* envoy/cilium_l7policy.cc:127-182                                          */
/* ======================================================================== */

/* Install the full set of endpoint NetworkPolicies (the NPDS resource list,
 * envoy/cilium/npds.proto:31-182) given in protobuf-JSON form:
 *   [{"name": "...", "policy": 3,
 *     "ingress_per_port_policies": [{"port": 80, "protocol": "TCP",
 *        "rules": [{"remote_policies": [1],
 *                   "http_rules": {"http_rules": [{"headers": [
 *                       {"name": ":path", "regex_match": "..."} |
 *                       {"name": "...", "exact_match": "..."} |
 *                       {"name": "...", "present_match": true}]}]}}]}],
 *     "egress_per_port_policies": [...]}]
 * Compiles every regex to a minimized union DFA per (policy, direction,
 * port) and swaps the snapshot in; on any error (regex outside the
 * supported ECMAScript subset, duplicate port → EnvoyException
 * "PortNetworkPolicy: Duplicate port number", cilium_network_policy.h:160)
 * the previous snapshot stays and CG_POLICY_REJECTED is returned. */
int cg_http_policy_update(uint64_t h, const char* npds_json, size_t len);
/* The installed HTTP snapshot's compiled tables as a flat image (unions,
 * DFAs, remote tables, program index; a checksum) and its import on another
 * handle — another GPU or process — without recompiling: SURVEY §8(e)
 * "the host compiles once and uploads identical images to each GPU"; also the
 * serialized table cache (§5 checkpoint / resume).  Export with buf = NULL
 * returns the size in *len.  Import is all-or-nothing like an update; an
 * image from another library build is CG_POLICY_REJECTED.  Replaces the
 * per-worker re-translation of NetworkPolicyMap::onConfigUpdate
 * (envoy/cilium_network_policy.cc) with one compile per node. */
int cg_http_policy_export(uint64_t h, void* buf, size_t cap, size_t* len);
int cg_http_policy_import(uint64_t h, const void* buf, size_t len);

/* The same update from the NPDS wire form: a serialized xDS
 * envoy.api.v2.DiscoveryResponse whose resources are google.protobuf.Any
 * of type "type.googleapis.com/cilium.NetworkPolicy" (envoy/cilium/npds.proto:
 * 31-182, the StreamNetworkPolicies payload Envoy's NPDS subscription hands to
 * NetworkPolicyMap::onConfigUpdate, envoy/cilium_network_policy.cc:46-60).
 * The messages are validated as npds.pb.validate.go does (port <= 65535,
 * unique remote_policies, non-empty rule lists, Kafka name patterns); a
 * resource of another type, a malformed message or a failed validation
 * rejects the whole update (CG_POLICY_REJECTED, previous snapshot stays). */
int cg_http_policy_update_npds(uint64_t h, const uint8_t* discovery_response, size_t len);
/* Index of a policy name in the installed snapshot (for the packer);
 * CG_NOT_FOUND → requests naming it are denied (cilium_network_policy.h:232-235). */
int cg_http_policy_index(uint64_t h, const char* name, uint32_t* index);
/* Snapshot statistics: programs, DFA parts, total states, table bytes. */
int cg_http_policy_stats(uint64_t h, uint64_t* out, size_t n);

/* Per-rule hit counters (what = CG_CTR_HTTP_RULES in cg_read_counters): a
 * request Envoy allows through a rule is counted once, on the FIRST rule
 * that allows it in Envoy's evaluation order (PolicyInstance::Allowed →
 * PortNetworkPolicy::Matches: the port's own PortNetworkPolicyRules, then
 * port 0's, each rule's HttpNetworkPolicyRules in order,
 * cilium_network_policy.h:90-192).  Counter i counts the rule described by
 * entry i of cg_http_rule_info_get; a rule of port 0's scope has one counter
 * per exact-port program it is merged into and one in the wildcard-port
 * program.  Requests allowed because no HTTP policy applies (no policy for
 * the port, a port without HTTP rules) are attributed to no rule; denied
 * requests to none (their per-program denied counter counts them). */
typedef struct {
  uint32_t policy;     /* policy index (cg_http_policy_index) */
  uint32_t ingress;    /* 1 ingress, 0 egress */
  uint32_t port;       /* the program's destination port; 0 = the wildcard-port program */
  uint32_t scope;      /* 0: the rule is in this port's PortNetworkPolicy, 1: in port 0's */
  uint32_t rule;       /* PortNetworkPolicyRule index within its scope */
  uint32_t http_rule;  /* HttpNetworkPolicyRule index within it, or one of: */
} cg_http_rule_info;
#define CG_HTTP_RULE_NO_HTTP 0xFFFFFFFFu     /* the PortNetworkPolicyRule has no HTTP rules */
#define CG_HTTP_RULE_SCOPE_ALLOW 0xFFFFFFFEu /* port 0 has no HTTP rules: it allows the rest */
int cg_http_rule_info_get(uint64_t h, cg_http_rule_info* out, size_t cap, size_t* n);

/* Packed request batches.  A record is an 8-byte meta word plus its field
 * string in 16-byte units (at most CG_HTTP_SLOT_BYTES in the record; longer
 * strings go to the overflow arena).  Records are stored tile-transposed in
 * tiles of 64: a tile is its 512-byte meta block then as many string units as
 * its longest string needs (string unit u ≥ 1 of lane l at tile + 512 +
 * (u-1)*1024 + l*16), so a wavefront's 16-byte load of a unit is one
 * contiguous 1 KiB read; when no lane holds more than 8 bytes in the last
 * unit, that unit is stored as a 512-byte half unit (8 bytes per lane; tile
 * table bit 15), in tiles of programs walked from LDS one part at a time.  The
 * packer resolves each request's (policy, direction, port) evaluation
 * program on the host and groups requests by program (padding each group to
 * whole tiles), so a workgroup stages one program's DFA in LDS.  A batch is
 * a 64-byte header (its total_bytes field = the batch's size), a chunk
 * table, a tile table ({offset in 512-B granules, units | half << 15 |
 * last-unit bytes << 16} per tile), then the tiles;
 * slots are in grouped order and order[slot] gives the request index
 * (UINT32_MAX for padding).  Size the buffers with cg_http_batch_bytes /
 * cg_http_batch_slots (upper bounds for n requests under the installed
 * policy; a batch is tied to the snapshot it was packed against — after a
 * policy update it is rejected and every slot is denied). */
#define CG_HTTP_TILE 64
#define CG_HTTP_UNITS 9
#define CG_HTTP_SLOT_BYTES 128
#define CG_HTTP_META_BYTES 8
size_t cg_http_batch_bytes(uint64_t h, size_t n);
size_t cg_http_batch_slots(uint64_t h, size_t n);

/* Request flags (meta byte 7).  Meta word: [0..3] remote identity, [4..6]
 * overflow arena offset / 16, [7] flags.  An overflow arena entry is the
 * string's u32 length followed by the string. */
#define CG_HTTP_F_INGRESS 0x01u
#define CG_HTTP_F_OVERFLOW 0x02u  /* fields in the overflow arena */
#define CG_HTTP_F_MALFORMED 0x04u /* field holds a byte Envoy's codec rejects */
#define CG_HTTP_F_PAD 0x08u

/* Worker threads cg_http_pack uses for a large batch (CILIUM_GPU_PACK_THREADS,
 * else the hardware threads, at most 16). */
uint32_t cg_http_pack_threads(void);
/* Pack n requests.  Request i: policy index policy[i] (UINT32_MAX unknown),
 * direction ingress[i], destination port port[i], remote identity
 * remote[i] (source identity on ingress, destination on egress,
 * cilium_l7policy.cc:144-150), and its header list as NUL-separated
 * "name\0value\0" pairs in hdr_blob[hdr_off[i] .. hdr_off[i+1]).  Header
 * names compare case-insensitively and only the first value of a name is
 * seen (Envoy HeaderMap::get).  Records whose slot string exceeds 128 bytes
 * spill into the overflow arena: pass arena/arena_cap (may be NULL/0 to
 * query), *arena_used gets the bytes needed; one batch's arena is at most
 * 256 MiB (CG_INVALID_ARGUMENT beyond: pack such a request set as several
 * batches; cg_http_verdicts_raw_* splits by itself).  *nslots gets the batch's slot
 * count; order must hold cg_http_batch_slots(h, n) entries. */
int cg_http_pack(uint64_t h, size_t n, const uint32_t* policy, const uint8_t* ingress,
                 const uint16_t* port, const uint32_t* remote, const uint8_t* hdr_blob,
                 const uint64_t* hdr_off, void* batch, size_t batch_cap, uint32_t* order,
                 size_t* nslots, uint8_t* arena, size_t arena_cap, size_t* arena_used);

/* HTTP/1.x request heads from raw bytes (the Envoy codec
 * step in front of AccessFilter::decodeHeaders, cilium_l7policy.cc:127-170).
 * Request r is raw[raw_off[r] .. raw_off[r+1]): request-line, header fields,
 * empty line.  Writes the cg_http_pack header lists (:method, :path with the
 * query, :authority from Host, then the other headers as sent) into hdr_blob
 * / hdr_off (n+1 entries) and ok[r] = 0 (ok may be NULL) for a head the
 * codec rejects (bad request-line, non-token name, control byte in a value,
 * no final CRLF).  A rejected head's list is one entry whose value is the
 * byte 0x7F, which cg_http_pack flags CG_HTTP_F_MALFORMED: it is denied
 * under any policy, as Envoy answers 400 before the filter.  hdr_blob NULL
 * = size query (*blob_used). */
int cg_http_parse_heads(const uint8_t* raw, const uint64_t* raw_off, size_t n, uint8_t* hdr_blob,
                        size_t blob_cap, uint64_t* hdr_off, size_t* blob_used, uint8_t* ok);

/* Raw HTTP/1 request heads to verdicts on the device: the codec step of
 * cg_http_parse_heads, the packing of cg_http_pack and the verdicts of
 * cg_http_verdicts_dev in one call, with the request bytes never leaving
 * device memory (the consumer is AccessFilter::
 * decodeHeaders, envoy/cilium_l7policy.cc:127-170).  Request r is
 * d_raw[d_raw_off[r] .. d_raw_off[r+1]) with d_policy/d_ingress/d_port/
 * d_remote as in cg_http_pack; d_out[r] = 1 allow, 0 deny, request order.
 * Heads over 60 KiB are rejected (Envoy's default max_request_headers_kb).
 * Enqueued on `stream` and returns without waiting (NULL: the handle's
 * stream, waited for before the call returns):
 * slots, tiles, chunk table and header are laid out on the device, strings
 * past the 128-byte slot walked one lane each; a later call on another
 * stream waits for this one on the device.  An offset range that runs
 * backwards is an empty (rejected) request — the call has returned before
 * the device reads the offsets.  CILIUM_GPU_RAW_LAYOUT=host selects the
 * round-3 sequence instead (host layout step, synchronizes the stream,
 * CG_INVALID_ARGUMENT for backward offsets).  CG_UNSUPPORTED when the
 * snapshot walks more than 32 header fields or is a proxylib snapshot. */
int cg_http_verdicts_raw_dev(uint64_t h, const uint8_t* d_raw, const uint64_t* d_raw_off, size_t n,
                             const uint32_t* d_policy, const uint8_t* d_ingress, const uint16_t* d_port,
                             const uint32_t* d_remote, uint8_t* d_out, void* stream);

/* cg_http_verdicts_raw_dev from host memory (staged in, verdicts copied out). */
int cg_http_verdicts_raw_host(uint64_t h, const uint8_t* raw, const uint64_t* raw_off, size_t n,
                              const uint32_t* policy, const uint8_t* ingress, const uint16_t* port,
                              const uint32_t* remote, uint8_t* out);

/* Parsed header lists to verdicts on the device: the input of cg_http_pack
 * (request i's "name\0value\0" pairs in d_hdr_blob[d_hdr_off[i] ..
 * d_hdr_off[i+1]), names case-insensitive, first value wins, the codec's
 * value check — the header map AccessFilter::decodeHeaders sees,
 * envoy/cilium_l7policy.cc:127-182) grouped, sorted and packed by the raw
 * path's kernels instead of on the host, then cg_http_verdicts_dev; d_out[i]
 * = 1 allow, 0 deny, request order.  Proxylib snapshots take escaped values
 * as cg_http_pack does.  One request's list holds at most 65535 bytes
 * (Envoy's default header limit is 60 KiB): a longer one is denied here (the
 * host entry and the round-3 sequence refuse the call, CG_INVALID_ARGUMENT).
 * Stream and synchronization as cg_http_verdicts_raw_dev; CG_UNSUPPORTED when
 * the snapshot walks more than 32 header fields. */
int cg_http_verdicts_fields_dev(uint64_t h, const uint8_t* d_hdr_blob, const uint64_t* d_hdr_off, size_t n,
                                const uint32_t* d_policy, const uint8_t* d_ingress, const uint16_t* d_port,
                                const uint32_t* d_remote, uint8_t* d_out, void* stream);

/* cg_http_verdicts_fields_dev from host memory (staged in, verdicts copied
 * out): the drop-in for cg_http_pack + cg_http_verdicts_host.  A call of at
 * most 1024 lists (Envoy-sized: decodeHeaders decides one request,
 * envoy/cilium_l7policy.cc:127-182) is packed on the calling thread and
 * decided with one staged copy in, one launch and one copy out; larger ones
 * are grouped and packed on the GPU.  Any snapshot works at any size: when
 * the device packer does not take it (more than 32 header fields walked),
 * larger calls are packed on the calling thread too, 1M lists at a time. */
int cg_http_verdicts_fields_host(uint64_t h, const uint8_t* hdr_blob, const uint64_t* hdr_off, size_t n,
                                 const uint32_t* policy, const uint8_t* ingress, const uint16_t* port,
                                 const uint32_t* remote, uint8_t* out);

/* The persistent verdict ring: Envoy-sized calls (AccessFilter::decodeHeaders
 * decides one request, envoy/cilium_l7policy.cc:127-182) without a launch,
 * staged copies or a stream synchronization per call.  cg_http_ring_open
 * starts `workgroups` one-wave workgroups (1..256) that poll `slots`
 * (1..64 * workgroups) request slots in pinned host memory; a call of
 * cg_http_ring_verdicts claims a slot, writes its header lists there, rings
 * the slot's doorbell and spins until the kernel has written the verdicts.
 * Same inputs, outputs and verdicts as cg_http_verdicts_fields_host (which
 * decides calls past a slot: more than 256 lists or 32 KiB of list bytes,
 * and snapshots walking more than 32 header fields).  The kernel serves the
 * handle's current policy: a cg_http_policy_update restarts it before the
 * next call; it leaves by itself after 50 ms without a call (the next call
 * starts it again, ~20 us).  cg_http_ring_close (or cg_close) stops it. */
int cg_http_ring_open(uint64_t h, uint32_t workgroups, uint32_t slots);
int cg_http_ring_verdicts(uint64_t h, const uint8_t* hdr_blob, const uint64_t* hdr_off, size_t n,
                          const uint32_t* policy, const uint8_t* ingress, const uint16_t* port,
                          const uint32_t* remote, uint8_t* out);
/* Calls served by the ring's kernels and launches made, cumulative. */
int cg_http_ring_stats(uint64_t h, uint64_t* served, uint64_t* launches);
int cg_http_ring_close(uint64_t h);

/* NetworkPolicyMap::Allowed per slot (cilium_network_policy.h:223-237):
 * d_out[slot] = 1 allow, 0 deny (→ 403), in batch slot order.  d_arena may
 * be NULL when no record overflowed.  Per-(policy,direction,port) allowed/
 * denied counters advance (metrics policy_l7_forwarded/denied_total,
 * pkg/metrics/metrics.go:270-296). */
int cg_http_verdicts_dev(uint64_t h, const void* d_batch, size_t nslots, const uint8_t* d_arena,
                         uint8_t* d_out, void* stream);
/* Host convenience: uploads the batch, runs the kernel and writes out[i]
 * for request i (un-permuting through order). */
int cg_http_verdicts_host(uint64_t h, const void* batch, size_t nslots, const uint32_t* order,
                          size_t n, const uint8_t* arena, size_t arena_len, uint8_t* out);
/* The same verdicts with each request's first matching rule beside it:
 * d_rule[slot] = the per-rule counter index it adds to (cg_http_rule_info_get
 * order: the PortNetworkPolicyRule / HTTP rule that allowed it, Envoy's
 * evaluation order), or UINT32_MAX when no rule allows it (denied, or
 * allowed because no HTTP policy applies).  Replaces the access log's rule
 * attribution (pkg/proxy/accesslog/record.go:36-47) and the policy trace
 * (pkg/policy/policy.go:29-70) for every request of a batch. */
int cg_http_verdicts_rules_dev(uint64_t h, const void* d_batch, size_t nslots, const uint8_t* d_arena,
                               uint8_t* d_out, uint32_t* d_rule, void* stream);
int cg_http_verdicts_rules_host(uint64_t h, const void* batch, size_t nslots, const uint32_t* order,
                                size_t n, const uint8_t* arena, size_t arena_len, uint8_t* out,
                                uint32_t* rule);

/* ======================================================================== */
/* Kafka L7: pkg/kafka/policy.go:144-225 via pkg/proxy/kafka.go:117-153      */
/* ======================================================================== */

/* Install Kafka redirect rule sets, JSON form of L7DataMap per redirect:
 *   [{"name": "...", "selectors": [
 *       {"identities": [1, 2] or null for the wildcard selector,
 *        "rules": [{"role": "...", "apiKey": "...", "apiVersion": "...",
 *                   "clientID": "...", "topic": "..."}]}]}]
 * Each PortRuleKafka is Sanitize()d (pkg/policy/api/rule_validation.go:232-275);
 * a failure rejects the whole update. */
int cg_kafka_policy_update(uint64_t h, const char* json, size_t len);
int cg_kafka_policy_index(uint64_t h, const char* name, uint32_t* index);

/* Packed Kafka request: 64 bytes. */
#define CG_KAFKA_MAX_TOPICS 12
typedef struct {
  int16_t api_key;      /* RequestMessage.kind */
  int16_t api_version;  /* RequestMessage.version */
  uint8_t kind;         /* CG_KAFKA_K_*: which typed request ReadRequest produced */
  uint8_t n_topics;     /* topics in topic_ids (> CG_KAFKA_MAX_TOPICS: in the arena at
                           topic_ids[0]; CG_KAFKA_TOPICS_IN_ARENA: count in topic_ids[1]) */
  uint16_t policy;      /* redirect index (UINT16_MAX unknown → deny) */
  uint32_t remote;      /* source identity (0 = unknown: wildcard rules only) */
  uint32_t client_id;   /* interned ClientID (CG_KAFKA_UNKNOWN_STR if not a rule string) */
  uint32_t topic_ids[CG_KAFKA_MAX_TOPICS]; /* interned topics; overflow: [0] = arena offset */
} cg_kafka_request;

#define CG_KAFKA_TOPICS_IN_ARENA 255  /* n_topics value for 255+ topics */
#define CG_KAFKA_K_NIL 0      /* request == nil (unparsed kinds) */
#define CG_KAFKA_K_TYPED 1    /* Produce/Fetch/Offset/Metadata/OffsetCommit/OffsetFetch */
#define CG_KAFKA_K_CONSUMER_METADATA 2
#define CG_KAFKA_UNKNOWN_STR 0xFFFFFFFFu

/* Intern a string against the installed Kafka snapshot's topic / clientID
 * dictionaries (what=0 topic, 1 clientID). */
int cg_kafka_intern(uint64_t h, uint32_t what, const char* s, size_t len, uint32_t* id);

/* Kafka requests from their wire bytes: ReadRequest (pkg/kafka/request.go:
 * 186-229) with the vendored optiopay/kafka decoders it calls (proto
 * ReadReq and Read{Produce,Fetch,Offset,Metadata,ConsumerMetadata,
 * OffsetCommit,OffsetFetch}Req, messages.go:124-166,504,767,1033,1173,1389,
 * 1591,1810; produce message sets parsed in full with CRC32 checks and
 * gzip / snappy payloads inflated, as pkg/proxy/kafka.go:449-451 configures).
 * Request i is raw[raw_off[i] .. raw_off[i+1]): the connection's bytes from
 * the start of the request (ReadReq reads 4 + size of them).  Writes one
 * cg_kafka_request per request (topics and clientID interned against the
 * installed snapshot, redirect[i] / remote[i] copied) and status[i]:
 * CG_KAFKA_DECODE_OK, or CG_KAFKA_DECODE_ERROR when ReadRequest returns an
 * error — the proxy closes the connection (kafka.go:340-347); such a
 * record is marked to be denied (policy UINT16_MAX).  Topic lists longer
 * than CG_KAFKA_MAX_TOPICS go to `arena` (arena_cap u32 entries); *arena_used
 * gets the entries the batch needs, and the call fails with CG_MAP_FULL
 * when that exceeds arena_cap (arena_cap >= raw bytes / 2 always suffices).
 * raw_off must be non-decreasing; raw holds raw_off[n] bytes.  The decode
 * runs on the GPU (cg_kafka_decode_dev on staged copies). */
#define CG_KAFKA_DECODE_OK 0
#define CG_KAFKA_DECODE_ERROR 1
int cg_kafka_decode_host(uint64_t h, const uint8_t* raw, const uint64_t* raw_off, size_t n,
                         const uint16_t* redirect, const uint32_t* remote, cg_kafka_request* reqs,
                         uint32_t* arena, size_t arena_cap, size_t* arena_used, uint8_t* status);

/* Kafka decode accounting of the handle, cumulative: compressed message
 * payloads (gzip / snappy, optiopay proto/messages.go:460-480) decoded on
 * the GPU, and requests the device handed to the host decoder (a nested
 * compressed set, a second gzip member, a payload past the per-call inflate
 * arena).  Either pointer may be NULL. */
int cg_kafka_decode_stats(uint64_t h, uint64_t* device_inflated, uint64_t* host_deferred);

/* Compressed payloads the device handed to the host decoder without
 * reserving inflate-arena space, cumulative: the per-call arena
 * (kKafkaInflateArena) was full, or the size the payload declares (gzip
 * ISIZE, snappy length) is more than its bytes can decode to (DEFLATE
 * 1032:1, snappy 32:1), so a sender's claim cannot use up the arena.  The
 * host decoder gives these requests their outcome either way. */
int cg_kafka_inflate_stats(uint64_t h, uint64_t* unreserved);

/* The same decode on the GPU (one lane per request, raw bytes in HBM),
 * records and statuses in device memory.  d_raw_off holds n + 1 offsets.
 * Requests carrying gzip / snappy messages are finished by the host
 * decoder (the device reports them, the call decodes them on the CPU and
 * patches their records before returning), so this call synchronizes.
 * d_arena: arena_cap u32 entries of device memory for long topic lists;
 * *arena_used and CG_MAP_FULL as for cg_kafka_decode_host.  A decreasing
 * offset pair is read as an empty request. */
int cg_kafka_decode_dev(uint64_t h, const uint8_t* d_raw, const uint64_t* d_raw_off, size_t n,
                        const uint16_t* d_redirect, const uint32_t* d_remote, cg_kafka_request* d_reqs,
                        uint32_t* d_arena, size_t arena_cap, size_t* arena_used, uint8_t* d_status,
                        void* stream);

/* Raw requests → verdicts in one call (decode on the GPU, then the verdict
 * kernel): out[i] = 1 forward, 0 deny (ErrTopicAuthorizationFailed),
 * 2 = ReadRequest failed (connection closed). */
#define CG_KAFKA_V_DENY 0
#define CG_KAFKA_V_ALLOW 1
#define CG_KAFKA_V_CLOSE 2
int cg_kafka_verdicts_raw_host(uint64_t h, const uint8_t* raw, const uint64_t* raw_off, size_t n,
                               const uint16_t* redirect, const uint32_t* remote, uint8_t* out);

/* kafkaRedirect.canAccess per request: out[i] = 1 allow, 0 deny. */
int cg_kafka_verdicts_dev(uint64_t h, const cg_kafka_request* d_reqs, size_t n,
                          const uint32_t* d_arena, uint8_t* d_out, void* stream);
int cg_kafka_verdicts_host(uint64_t h, const cg_kafka_request* reqs, size_t n,
                           const uint32_t* arena, size_t arena_len, uint8_t* out);
/* The same verdicts over the record split in two arrays: d_heads[i] = the
 * first 16 bytes of cg_kafka_request i, d_topics[12 i .. 12 i + 11] = its
 * topic_ids.  Most requests are settled from the head alone (the decision
 * summaries), so HBM moves 16 bytes per request instead of a 64-byte record
 * line; topic tails are read only for the requests that need their topics. */
typedef struct {
  int16_t api_key;
  int16_t api_version;
  uint8_t kind;
  uint8_t n_topics;
  uint16_t policy;
  uint32_t remote;
  uint32_t client_id;
} cg_kafka_request_head;
int cg_kafka_verdicts_split_dev(uint64_t h, const cg_kafka_request_head* d_heads, const uint32_t* d_topics,
                                size_t n, const uint32_t* d_arena, uint8_t* d_out, void* stream);

/* ======================================================================== */
/* Counters                                                                  */
/* ======================================================================== */
/* what: 0 = HTTP per-program {allowed, denied} u64 pairs,
 *       1 = Kafka per-redirect {allowed, denied} u64 pairs,
 *       2 = prefilter {drop, pass} u64 pair for pf_or_map,
 *       3 = HTTP per-rule first-match hits (cg_http_rule_info_get order),
 *       4 = the HTTP all-reduce vector: the per-program pairs, the stale-
 *           batch count, then the per-rule hits (one contiguous device
 *           buffer, summed across GPUs by RCCL).
 * Writes min(cap, available) u64 values, *n = available. */
#define CG_CTR_HTTP_PROGRAMS 0u
#define CG_CTR_KAFKA 1u
#define CG_CTR_PREFILTER 2u
#define CG_CTR_HTTP_RULES 3u
#define CG_CTR_HTTP_ALLREDUCE 4u
int cg_read_counters(uint64_t h, uint32_t what, uint32_t pf_or_map, uint64_t* out, size_t cap,
                     size_t* n);
/* Same, into a device buffer (for an RCCL all-reduce across GPUs). */
int cg_counters_device_ptr(uint64_t h, uint32_t what, uint32_t pf_or_map, void** d_ptr,
                           size_t* n);
/* Async device-to-device copy of up to n counters into d_dst on stream. */
int cg_counters_copy_dev(uint64_t h, uint32_t what, uint32_t pf_or_map, void* d_dst, size_t n,
                         void* stream);
int cg_reset_counters(uint64_t h);

/* Synchronize the handle's stream. */
int cg_sync(uint64_t h);

/* Regex syntax check, no compilation: flavour CG_REGEX_GO = Go 1.10
 * regexp.Compile's grammar (PortRuleHTTP.Sanitize,
 * pkg/policy/api/http.go:66-84; proxylib's regexp.MustCompile,
 * proxylib/r2d2/r2d2parser.go:103), CG_REGEX_ECMA = std::regex's (what
 * Envoy compiles for regex_match, envoy/cilium_network_policy.h:68-71).
 * Returns CG_OK or CG_POLICY_REJECTED (message in cg_last_error). */
enum { CG_REGEX_ECMA = 0, CG_REGEX_GO = 1 };
int cg_regex_validate(const char* re, size_t re_len, uint32_t flavour);

/* ======================================================================== */
/* Diagnostics (CPU test-suite only; no verdict entry point calls these)    */
/* ======================================================================== */
/* Compile `re` with the engine's regex compiler and run the DFA on s
 * (search = 0: std::regex_match, ECMAScript; 1: Go regexp.MatchString). */
int cg_diag_regex_match(const char* re, size_t re_len, const uint8_t* s, size_t len,
                        uint32_t search, uint8_t* result);
/* Walk the compiled HTTP / Kafka tables on the host, exactly as the kernels
 * do, to test the compilers without a GPU. */
int cg_diag_http_eval_host(uint64_t h, const void* batch, size_t nslots, const uint32_t* order,
                           size_t n, const uint8_t* arena, size_t arena_len, uint8_t* out);
/* The same walk, reporting per request the per-rule hit counter it adds to
 * (cg_http_rule_info_get index), or UINT32_MAX when no rule allows it. */
int cg_diag_http_rules_host(uint64_t h, const void* batch, size_t nslots, const uint32_t* order,
                            size_t n, const uint8_t* arena, size_t arena_len, uint32_t* rule);
int cg_diag_kafka_eval_host(uint64_t h, const cg_kafka_request* reqs, size_t n,
                            const uint32_t* arena, size_t arena_len, uint8_t* out);
/* cg_kafka_decode_host's decode on the CPU (the host decoder that also
 * finishes compressed produce requests), for cross-checking the GPU. */
int cg_diag_kafka_decode_host(uint64_t h, const uint8_t* raw, const uint64_t* raw_off, size_t n,
                              const uint16_t* redirect, const uint32_t* remote, cg_kafka_request* reqs,
                              uint32_t* arena, size_t arena_cap, size_t* arena_used, uint8_t* status);
int cg_diag_l4_eval_host(uint64_t h, uint32_t map_id, const cg_l4_tuple* tuples, size_t n,
                         int32_t* verdicts);
/* The ipcache tables walked on the host exactly as ipcache_kernel does. */
int cg_diag_ipcache_eval_host(uint64_t h, uint32_t ipc_id, const uint32_t* v4, size_t n4,
                              cg_remote_endpoint_info* out4, const uint8_t* v6, size_t n6,
                              cg_remote_endpoint_info* out6);
int cg_diag_prefilter_eval_host(uint64_t h, uint32_t pf_id, const uint32_t* v4, size_t n4,
                                uint8_t* out4, const uint8_t* v6, size_t n6, uint8_t* out6);

#ifdef __cplusplus
}
#endif
#endif /* CILIUM_GPU_H */
