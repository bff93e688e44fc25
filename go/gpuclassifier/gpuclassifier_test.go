package gpuclassifier

import (
	"net"
	"testing"
)

// The control plane on a host-only handle (device -1); verdict calls there
// must answer NoDevice (no CPU fallback).  Run with the library built:
//
//	python cilium_amd/build.py && cd go && go test ./gpuclassifier
func TestHostOnlyHandle(t *testing.T) {
	e, err := Open(-1)
	if err != nil {
		t.Fatal(err)
	}
	defer e.Close()
	pm, err := e.NewPolicyMap(0)
	if err != nil {
		t.Fatal(err)
	}
	if err := pm.Allow(300, 80, 6, Ingress, 0); err != nil {
		t.Fatal(err)
	}
	if !pm.Exists(PolicyKey{Identity: 300, DestPort: hton16(80), Nexthdr: 6}) {
		t.Fatal("key not found after Allow")
	}
	keys, _, err := pm.DumpToSlice()
	if err != nil || len(keys) != 1 {
		t.Fatalf("dump: %v %d", err, len(keys))
	}
	if _, err := pm.Verdicts([]L4Tuple{{Identity: 300, DPort: hton16(80), Proto: 6, Flags: L4Ingress}}); err == nil ||
		err.(*Error).Code != NoDevice {
		t.Fatalf("verdicts on a host-only handle: %v", err)
	}
	pf, err := e.NewPreFilter(PrefilterDyn4|PrefilterFix4, 0, 0)
	if err != nil {
		t.Fatal(err)
	}
	_, n, _ := net.ParseCIDR("10.1.2.0/24")
	if rev, err := pf.Insert(1, []net.IPNet{*n}); err != nil || rev != 2 {
		t.Fatalf("insert: %v %d", err, rev)
	}
	if _, err := pf.Insert(1, []net.IPNet{*n}); err == nil || err.(*Error).Code != RevisionMismatch {
		t.Fatalf("stale revision: %v", err)
	}
	h := PortRuleHTTP{Path: "(?i)^/v1/", Method: "GET"}
	if err := h.Sanitize(); err != nil {
		t.Fatal(err)
	}
	if err := (&PortRuleHTTP{Path: "a**"}).Sanitize(); err == nil {
		t.Fatal("Sanitize accepted a** (Go rejects nested repetition)")
	}
	pol := []byte(`[{"name":"sw","egress_per_port_policies":[{"port":80,"rules":[{"http_rules":{"http_rules":[` +
		`{"headers":[{"name":":method","regex_match":"GET"},{"name":":path","regex_match":"/v1/"}]}]}}]}]}]`)
	if err := e.UpdateNetworkPoliciesJSON(pol); err != nil {
		t.Fatal(err)
	}
	if _, err := e.PolicyIndex("sw"); err != nil {
		t.Fatal(err)
	}
	if err := e.UpdateKafka([]KafkaRedirect{{Name: "k", Selectors: []KafkaSelectorRules{
		{Identities: []uint32{7}, Rules: []PortRuleKafka{{Role: "produce", Topic: "allowedTopic"}}}}}}); err != nil {
		t.Fatal(err)
	}
}
