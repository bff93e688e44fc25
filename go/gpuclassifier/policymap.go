package gpuclassifier

// #include "cilium_gpu.h"
import "C"

import "unsafe"

// PolicyMap mirrors policymap.PolicyMap (pkg/maps/policymap/policymap.go:
// 164-280) on the device: one per endpoint, 16384 entries by default.
type PolicyMap struct {
	e  *Engine
	id C.uint32_t
}

// NewPolicyMap creates a map; maxEntries 0 = MaxEntries 16384 (policymap.go:37).
func (e *Engine) NewPolicyMap(maxEntries uint32) (*PolicyMap, error) {
	var id C.uint32_t
	if err := call(func() C.int { return C.cg_policymap_create(e.h, C.uint32_t(maxEntries), &id) }); err != nil {
		return nil, err
	}
	return &PolicyMap{e: e, id: id}, nil
}

// Destroy frees the map's tables once queued launches are done with them.
func (pm *PolicyMap) Destroy() error { return call(func() C.int { return C.cg_policymap_destroy(pm.e.h, pm.id) }) }

func hton16(v uint16) uint16 { return v<<8 | v>>8 }

func cKey(k PolicyKey) C.cg_policy_key {
	return C.cg_policy_key{sec_label: C.uint32_t(k.Identity), dport: C.uint16_t(k.DestPort),
		protocol: C.uint8_t(k.Nexthdr), egress: C.uint8_t(k.TrafficDirection)}
}

// AllowKey is PolicyMap.AllowKey (policymap.go:162-166): proxyPort in host
// byte order; existing counters are kept.
func (pm *PolicyMap) AllowKey(k PolicyKey, proxyPort uint16) error {
	ck := cKey(k)
	pp := C.uint16_t(hton16(proxyPort))
	return call(func() C.int { return C.cg_policymap_allow(pm.e.h, pm.id, &ck, &pp, 1) })
}

// Allow is PolicyMap.Allow (policymap.go:168-176): dport and proxyPort in
// host byte order.
func (pm *PolicyMap) Allow(id uint32, dport uint16, proto uint8, dir TrafficDirection, proxyPort uint16) error {
	return pm.AllowKey(PolicyKey{Identity: id, DestPort: hton16(dport), Nexthdr: proto,
		TrafficDirection: uint8(dir)}, proxyPort)
}

// AllowKeys installs a batch (all-or-nothing; MapFull beyond max entries).
// proxyPorts are in network byte order, as syncPolicyMap writes them.
func (pm *PolicyMap) AllowKeys(keys []PolicyKey, proxyPortsBE []uint16) error {
	if len(keys) == 0 || len(keys) != len(proxyPortsBE) {
		return &Error{Code: InvalidArgument, Msg: "keys and proxy ports differ in length"}
	}
	return call(func() C.int { return C.cg_policymap_allow(pm.e.h, pm.id, (*C.cg_policy_key)(unsafe.Pointer(&keys[0])),
		(*C.uint16_t)(unsafe.Pointer(&proxyPortsBE[0])), C.size_t(len(keys))) })
}

// DeleteKey is PolicyMap.DeleteKey (policymap.go:187-193).
func (pm *PolicyMap) DeleteKey(k PolicyKey) error {
	ck := cKey(k)
	return call(func() C.int { return C.cg_policymap_delete(pm.e.h, pm.id, &ck, 1) })
}

// Lookup is Exists + LookupElement (policymap.go:181-185).
func (pm *PolicyMap) Lookup(k PolicyKey) (PolicyEntry, error) {
	ck := cKey(k)
	var ce C.cg_policy_entry
	if err := call(func() C.int { return C.cg_policymap_lookup(pm.e.h, pm.id, &ck, &ce) }); err != nil {
		return PolicyEntry{}, err
	}
	return PolicyEntry{ProxyPort: uint16(ce.proxy_port), Packets: uint64(ce.packets), Bytes: uint64(ce.bytes)}, nil
}

// Exists is PolicyMap.Exists (policymap.go:181-185).
func (pm *PolicyMap) Exists(k PolicyKey) bool {
	_, err := pm.Lookup(k)
	return err == nil
}

// DumpToSlice is PolicyMap.DumpToSlice (policymap.go:224-255).
func (pm *PolicyMap) DumpToSlice() ([]PolicyKey, []PolicyEntry, error) {
	var n C.size_t
	if err := call(func() C.int { return C.cg_policymap_dump(pm.e.h, pm.id, nil, nil, 0, &n) }); err != nil {
		return nil, nil, err
	}
	keys := make([]PolicyKey, int(n))
	entries := make([]PolicyEntry, int(n))
	if n == 0 {
		return keys, entries, nil
	}
	if err := call(func() C.int { return C.cg_policymap_dump(pm.e.h, pm.id, (*C.cg_policy_key)(unsafe.Pointer(&keys[0])),
		(*C.cg_policy_entry)(unsafe.Pointer(&entries[0])), n, &n) }); err != nil {
		return nil, nil, err
	}
	return keys, entries, nil
}

// Flush is PolicyMap.Flush (policymap.go:257-280).
func (pm *PolicyMap) Flush() error { return call(func() C.int { return C.cg_policymap_flush(pm.e.h, pm.id) }) }

// VerdictsDev runs __policy_can_access (policy.h:46-110) over n device
// tuples into device verdicts on a hipStream_t (nil: the handle's stream),
// asynchronously.
func (pm *PolicyMap) VerdictsDev(tuples unsafe.Pointer, n int, verdicts unsafe.Pointer, stream unsafe.Pointer) error {
	return call(func() C.int { return C.cg_l4_verdicts_dev(pm.e.h, pm.id, (*C.cg_l4_tuple)(tuples), C.size_t(n),
		(*C.int32_t)(verdicts), stream) })
}

// Verdicts is VerdictsDev from host memory (staged in, verdicts copied out).
func (pm *PolicyMap) Verdicts(tuples []L4Tuple) ([]int32, error) {
	out := make([]int32, len(tuples))
	if len(tuples) == 0 {
		return out, nil
	}
	err := call(func() C.int { return C.cg_l4_verdicts_host(pm.e.h, pm.id, (*C.cg_l4_tuple)(unsafe.Pointer(&tuples[0])),
		C.size_t(len(tuples)), (*C.int32_t)(unsafe.Pointer(&out[0]))) })
	return out, err
}
