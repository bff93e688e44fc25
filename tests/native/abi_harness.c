/* abi_harness.c — the C-ABI boundary driven by a C compiler.
 *
 * Compiled by gcc (C11) against include/cilium_gpu.h and linked to
 * cilium_amd/libciliumgpu.so by tests/test_abi.py (CPU suite).  It pins the
 * struct layouts a cgo or Envoy binding relies on (the BPF map ABI of
 * bpf/lib/common.h:175-193 and the engine's packed records) and calls the
 * control-plane entry points plus the host table walkers on a device = -1
 * handle: policymap (pkg/maps/policymap/policymap.go:164-255), prefilter
 * (pkg/datapath/prefilter/prefilter.go:125-203), ipcache, NPDS HTTP policy
 * (pkg/envoy/server.go → cilium_network_policy.h) with cg_http_pack, and the
 * Kafka policy.  Verdict entry points must answer CG_NO_DEVICE there: the
 * engine has no CPU fallback.  Exit status 0 = every check held.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cilium_gpu.h"

/* struct policy_key (common.h:180-186): 8 bytes */
_Static_assert(sizeof(cg_policy_key) == 8, "policy_key");
_Static_assert(offsetof(cg_policy_key, sec_label) == 0, "policy_key.sec_label");
_Static_assert(offsetof(cg_policy_key, dport) == 4, "policy_key.dport");
_Static_assert(offsetof(cg_policy_key, protocol) == 6, "policy_key.protocol");
_Static_assert(offsetof(cg_policy_key, egress) == 7, "policy_key.egress");
/* struct policy_entry (common.h:188-193): 24 bytes */
_Static_assert(sizeof(cg_policy_entry) == 24, "policy_entry");
_Static_assert(offsetof(cg_policy_entry, packets) == 8, "policy_entry.packets");
_Static_assert(offsetof(cg_policy_entry, bytes) == 16, "policy_entry.bytes");
/* packed L4 tuple: 12 bytes */
_Static_assert(sizeof(cg_l4_tuple) == 12, "l4_tuple");
_Static_assert(offsetof(cg_l4_tuple, dport) == 4, "l4_tuple.dport");
_Static_assert(offsetof(cg_l4_tuple, proto) == 6, "l4_tuple.proto");
_Static_assert(offsetof(cg_l4_tuple, flags) == 7, "l4_tuple.flags");
_Static_assert(offsetof(cg_l4_tuple, len) == 8, "l4_tuple.len");
/* cidrKey (cidrmap.go:52-64) as the engine takes it: 20 bytes */
_Static_assert(sizeof(cg_cidr) == 20, "cidr");
_Static_assert(offsetof(cg_cidr, prefixlen) == 1, "cidr.prefixlen");
_Static_assert(offsetof(cg_cidr, addr) == 4, "cidr.addr");
/* RemoteEndpointInfo (common.h:175-178): 8 bytes */
_Static_assert(sizeof(cg_remote_endpoint_info) == 8, "remote_endpoint_info");
_Static_assert(offsetof(cg_remote_endpoint_info, tunnel_endpoint) == 4, "remote_endpoint_info.tunnel");
/* packed Kafka request: 64 bytes, topics from offset 16 */
_Static_assert(sizeof(cg_kafka_request) == 64, "kafka_request");
_Static_assert(offsetof(cg_kafka_request, kind) == 4, "kafka_request.kind");
_Static_assert(offsetof(cg_kafka_request, policy) == 6, "kafka_request.policy");
_Static_assert(offsetof(cg_kafka_request, remote) == 8, "kafka_request.remote");
_Static_assert(offsetof(cg_kafka_request, client_id) == 12, "kafka_request.client_id");
_Static_assert(offsetof(cg_kafka_request, topic_ids) == 16, "kafka_request.topic_ids");
_Static_assert(sizeof(cg_http_rule_info) == 24, "http_rule_info");
_Static_assert(sizeof(cg_kafka_request_head) == 16, "kafka_request_head");
_Static_assert(offsetof(cg_kafka_request_head, client_id) == offsetof(cg_kafka_request, client_id), "head prefix");
_Static_assert(sizeof(cg_kv) == 2 * sizeof(void*), "kv");

static int failures = 0;
#define CHECK(cond, ...)                                  \
  do {                                                    \
    if (!(cond)) {                                        \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                       \
      fprintf(stderr, " (%s)\n", cg_last_error());        \
      ++failures;                                         \
    }                                                     \
  } while (0)

static uint16_t be16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }

static void test_policymap(uint64_t h) {
  uint32_t map = 0;
  CHECK(cg_policymap_create(h, 0, &map) == CG_OK, "policymap_create");
  /* {identity 300, dport 80, TCP, ingress} -> proxy 0 (allow);
   * {identity 301, 0, 0, ingress} (L3) -> proxy 8080 (ignored: TC_ACT_OK);
   * {0, 443, TCP, ingress} (L4 wildcard) -> proxy 10000 */
  cg_policy_key keys[3] = {{300, be16(80), 6, 0}, {301, 0, 0, 0}, {0, be16(443), 6, 0}};
  uint16_t proxy[3] = {0, be16(8080), be16(10000)};
  CHECK(cg_policymap_allow(h, map, keys, proxy, 3) == CG_OK, "policymap_allow");
  cg_policy_entry e;
  memset(&e, 0, sizeof(e));
  CHECK(cg_policymap_lookup(h, map, &keys[2], &e) == CG_OK && e.proxy_port == be16(10000), "lookup");
  cg_policy_key missing = {999, be16(1), 17, 0};
  CHECK(cg_policymap_lookup(h, map, &missing, &e) == CG_NOT_FOUND, "lookup missing");
  /* __policy_can_access (policy.h:46-110) via the host table walk */
  cg_l4_tuple t[5] = {
      {300, be16(80), 6, CG_L4_F_INGRESS, 100},   /* exact key: allow, proxy 0 */
      {301, be16(22), 6, CG_L4_F_INGRESS, 100},   /* L3 key: TC_ACT_OK */
      {302, be16(443), 6, CG_L4_F_INGRESS, 100},  /* L4 wildcard: its proxy port */
      {302, be16(80), 6, CG_L4_F_INGRESS, 100},   /* nothing: DROP_POLICY */
      {300, be16(80), 6, CG_L4_F_INGRESS | CG_L4_F_FRAGMENT, 100}, /* fragment: DROP_FRAG_NOSUPPORT */
  };
  int32_t v[5];
  CHECK(cg_diag_l4_eval_host(h, map, t, 5, v) == CG_OK, "diag_l4_eval_host");
  CHECK(v[0] == 0 && v[1] == 0 && v[2] == (int32_t)be16(10000) && v[3] == CG_DROP_POLICY &&
            v[4] == CG_DROP_FRAG_NOSUPPORT,
        "l4 verdicts %d %d %d %d %d", v[0], v[1], v[2], v[3], v[4]);
  CHECK(cg_l4_verdicts_host(h, map, t, 5, v) == CG_NO_DEVICE, "no CPU fallback for L4 verdicts");
  size_t n = 0;
  cg_policy_key dk[4];
  cg_policy_entry de[4];
  CHECK(cg_policymap_dump(h, map, dk, de, 4, &n) == CG_OK && n == 3, "dump n=%zu", n);
  CHECK(cg_policymap_delete(h, map, &keys[0], 1) == CG_OK, "delete");
  CHECK(cg_policymap_delete(h, map, &keys[0], 1) == CG_NOT_FOUND, "delete again");
  CHECK(cg_policymap_destroy(h, map) == CG_OK, "destroy");
}

static void test_prefilter(uint64_t h) {
  uint32_t pf = 0;
  CHECK(cg_prefilter_create(h, CG_PF_DYN4 | CG_PF_FIX4 | CG_PF_FIX6, 0, 0, &pf) == CG_OK, "prefilter_create");
  cg_cidr c[2];
  memset(c, 0, sizeof(c));
  c[0].family = 4, c[0].prefixlen = 24, c[0].addr[0] = 10, c[0].addr[1] = 1, c[0].addr[2] = 2;
  c[1].family = 4, c[1].prefixlen = 32, c[1].addr[0] = 192, c[1].addr[1] = 168, c[1].addr[3] = 7;
  int64_t rev = 0;
  CHECK(cg_prefilter_insert(h, pf, 1, c, 2, &rev) == CG_OK && rev == 2, "insert rev=%lld", (long long)rev);
  CHECK(cg_prefilter_insert(h, pf, 1, c, 1, &rev) == CG_REVISION_MISMATCH, "stale revision");
  const uint32_t ep = 0x0100000A; /* 10.0.0.1 in network order */
  CHECK(cg_prefilter_set_endpoints(h, pf, &ep, 1, NULL, 0) == CG_OK, "set_endpoints");
  /* {saddr, daddr}: inside the /24 -> drop; the /32 -> drop; elsewhere to
   * the local endpoint -> pass; elsewhere to a foreign address -> drop */
  uint32_t v4[8] = {0x0502010A, ep, 0x0700A8C0, ep, 0x01010101, ep, 0x01010101, 0x02020202};
  uint8_t out[4];
  CHECK(cg_diag_prefilter_eval_host(h, pf, v4, 4, out, NULL, 0, NULL) == CG_OK, "diag_prefilter");
  CHECK(out[0] == CG_XDP_DROP && out[1] == CG_XDP_DROP && out[2] == CG_XDP_PASS && out[3] == CG_XDP_DROP,
        "prefilter verdicts %d %d %d %d", out[0], out[1], out[2], out[3]);
  CHECK(cg_prefilter_verdicts_host(h, pf, v4, 4, out, NULL, 0, NULL) == CG_NO_DEVICE, "no CPU fallback (LPM)");
  CHECK(cg_prefilter_destroy(h, pf) == CG_OK, "prefilter_destroy");
}

static void test_ipcache(uint64_t h) {
  uint32_t ipc = 0;
  CHECK(cg_ipcache_create(h, 0, &ipc) == CG_OK, "ipcache_create");
  cg_cidr k[2];
  memset(k, 0, sizeof(k));
  k[0].family = 4, k[0].prefixlen = 16, k[0].addr[0] = 10, k[0].addr[1] = 1;
  k[1].family = 4, k[1].prefixlen = 32, k[1].addr[0] = 10, k[1].addr[1] = 1, k[1].addr[3] = 9;
  cg_remote_endpoint_info val[2] = {{5000, 0}, {6000, 0x0101A8C0}};
  CHECK(cg_ipcache_update(h, ipc, k, val, 2) == CG_OK, "ipcache_update");
  const uint32_t a[3] = {0x0900010A, 0x0800010A, 0x01010101};
  cg_remote_endpoint_info o[3];
  CHECK(cg_diag_ipcache_eval_host(h, ipc, a, 3, o, NULL, 0, NULL) == CG_OK, "diag_ipcache");
  /* longest prefix wins; no prefix: WORLD */
  CHECK(o[0].sec_label == 6000 && o[1].sec_label == 5000 && o[2].sec_label == CG_WORLD_ID, "ipcache %u %u %u",
        o[0].sec_label, o[1].sec_label, o[2].sec_label);
  CHECK(cg_ipcache_destroy(h, ipc) == CG_OK, "ipcache_destroy");
}

/* examples/demo/sw_policy_http.real.json as NPDS: egress port 80, any remote,
 * GET /v1/ | POST /v1/request-landing/ | PUT /v1/exhaust-port/ + X-Has-Force */
static const char* kStarwars =
    "[{\"name\":\"spaceship\",\"policy\":257,\"egress_per_port_policies\":[{\"port\":80,\"rules\":[{"
    "\"http_rules\":{\"http_rules\":["
    "{\"headers\":[{\"name\":\":method\",\"regex_match\":\"GET\"},{\"name\":\":path\",\"regex_match\":\"/v1/\"}]},"
    "{\"headers\":[{\"name\":\":method\",\"regex_match\":\"POST\"},"
    "{\"name\":\":path\",\"regex_match\":\"/v1/request-landing/\"}]},"
    "{\"headers\":[{\"name\":\":method\",\"regex_match\":\"PUT\"},"
    "{\"name\":\":path\",\"regex_match\":\"/v1/exhaust-port/\"},"
    "{\"name\":\"X-Has-Force\",\"exact_match\":\"true\"}]}]}}]}]}]";

static void test_http(uint64_t h) {
  CHECK(cg_http_policy_update(h, kStarwars, strlen(kStarwars)) == CG_OK, "http_policy_update");
  uint32_t pol = 0;
  CHECK(cg_http_policy_index(h, "spaceship", &pol) == CG_OK, "http_policy_index");
  CHECK(cg_http_policy_update(h, "[{\"name\":", 9) == CG_POLICY_REJECTED, "bad JSON rejected");
  /* the previous snapshot keeps serving: four requests */
  static const char blob[] =
      ":method\0GET\0:path\0/v1/\0"
      ":method\0PUT\0:path\0/v1/exhaust-port/\0"
      ":method\0PUT\0:path\0/v1/exhaust-port/\0x-has-force\0true\0"
      ":method\0DELETE\0:path\0/v1/\0";
  const uint64_t off[5] = {0, 23, 59, 112, 138};
  const uint32_t policy[4] = {pol, pol, pol, pol};
  const uint8_t ingress[4] = {0, 0, 0, 0};
  const uint16_t port[4] = {80, 80, 80, 80};
  const uint32_t remote[4] = {1000, 1000, 1000, 1000};
  const size_t cap = cg_http_batch_bytes(h, 4), slots = cg_http_batch_slots(h, 4);
  void* batch = malloc(cap);
  uint32_t* order = malloc(slots * sizeof(uint32_t));
  size_t nslots = 0, arena_used = 0;
  CHECK(cg_http_pack(h, 4, policy, ingress, port, remote, (const uint8_t*)blob, off, batch, cap, order, &nslots,
                     NULL, 0, &arena_used) == CG_OK,
        "http_pack");
  uint8_t out[4] = {9, 9, 9, 9};
  CHECK(cg_diag_http_eval_host(h, batch, nslots, order, 4, NULL, 0, out) == CG_OK, "diag_http_eval_host");
  CHECK(out[0] == 1 && out[1] == 0 && out[2] == 1 && out[3] == 0, "http verdicts %d %d %d %d", out[0], out[1],
        out[2], out[3]);
  CHECK(cg_http_verdicts_host(h, batch, nslots, order, 4, NULL, 0, out) == CG_NO_DEVICE, "no CPU fallback (HTTP)");
  size_t img = 0;
  CHECK(cg_http_policy_export(h, NULL, 0, &img) == CG_OK && img > 16, "export size");
  void* buf = malloc(img);
  CHECK(cg_http_policy_export(h, buf, img, &img) == CG_OK, "export");
  CHECK(cg_http_policy_import(h, buf, img) == CG_OK, "import");
  ((uint8_t*)buf)[img / 2] ^= 1;
  CHECK(cg_http_policy_import(h, buf, img) == CG_POLICY_REJECTED, "damaged image rejected");
  free(buf);
  free(batch);
  free(order);
  CHECK(cg_regex_validate("(?i)^/v1/\\pL+", 14, CG_REGEX_GO) == CG_OK, "Go syntax");
  CHECK(cg_regex_validate("(?i)^/v1/", 9, CG_REGEX_ECMA) == CG_POLICY_REJECTED, "ECMAScript refuses (?i)");
}

static void test_kafka(uint64_t h) {
  static const char* pol =
      "[{\"name\":\"k\",\"selectors\":[{\"identities\":[7],\"rules\":["
      "{\"role\":\"produce\",\"topic\":\"allowedTopic\"},{\"apiKey\":\"metadata\"}]}]}]";
  CHECK(cg_kafka_policy_update(h, pol, strlen(pol)) == CG_OK, "kafka_policy_update");
  uint32_t idx = 0, topic = 0;
  CHECK(cg_kafka_policy_index(h, "k", &idx) == CG_OK, "kafka_policy_index");
  CHECK(cg_kafka_intern(h, 0, "allowedTopic", 12, &topic) == CG_OK, "kafka_intern");
  cg_kafka_request r[2];
  memset(r, 0, sizeof(r));
  r[0].api_key = 0, r[0].kind = CG_KAFKA_K_TYPED, r[0].n_topics = 1, r[0].policy = (uint16_t)idx, r[0].remote = 7;
  r[0].client_id = CG_KAFKA_UNKNOWN_STR, r[0].topic_ids[0] = topic;
  r[1] = r[0];
  r[1].topic_ids[0] = CG_KAFKA_UNKNOWN_STR; /* disallowedTopic */
  uint8_t out[2] = {9, 9};
  CHECK(cg_diag_kafka_eval_host(h, r, 2, NULL, 0, out) == CG_OK, "diag_kafka_eval_host");
  /* pkg/proxy/kafka_test.go:184-258: produce to allowedTopic passes,
   * to disallowedTopic fails */
  CHECK(out[0] == 1 && out[1] == 0, "kafka verdicts %d %d", out[0], out[1]);
  CHECK(cg_kafka_verdicts_host(h, r, 2, NULL, 0, out) == CG_NO_DEVICE, "no CPU fallback (Kafka)");
}

int main(void) {
  const cg_kv params[1] = {{"device", "-1"}};
  const uint64_t h = cg_open(params, 1, 0);
  if (!h) {
    fprintf(stderr, "cg_open failed: %s\n", cg_last_error());
    return 2;
  }
  printf("%s\n", cg_version());
  test_policymap(h);
  test_prefilter(h);
  test_ipcache(h);
  test_http(h);
  test_kafka(h);
  cg_close(h);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("abi_harness: all checks passed\n");
  return 0;
}
