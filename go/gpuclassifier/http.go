package gpuclassifier

// #include <stdlib.h>
// #include "cilium_gpu.h"
import "C"

import "unsafe"

// UpdateNPDS installs the serialized NPDS DiscoveryResponse (resources:
// Any-wrapped cilium.NetworkPolicy, envoy/cilium/npds.proto:31-182) — what
// XDSServer.UpdateNetworkPolicy publishes (pkg/envoy/server.go:628) and
// Envoy's NetworkPolicyMap::onConfigUpdate compiles.  All-or-nothing: on
// PolicyRejected the previous snapshot keeps serving.
func (e *Engine) UpdateNPDS(discoveryResponse []byte) error {
	return call(func() C.int { return C.cg_http_policy_update_npds(e.h, bytesPtr(discoveryResponse), C.size_t(len(discoveryResponse))) })
}

// UpdateNetworkPoliciesJSON installs the protobuf-JSON form of the same
// resource list (a JSON array of cilium.NetworkPolicy, OrigName field names).
func (e *Engine) UpdateNetworkPoliciesJSON(policies []byte) error {
	cs := C.CBytes(policies)
	defer C.free(cs)
	return call(func() C.int { return C.cg_http_policy_update(e.h, (*C.char)(cs), C.size_t(len(policies))) })
}

// PolicyIndex is the index requests name a policy by (NetworkPolicy.name).
func (e *Engine) PolicyIndex(name string) (uint32, error) {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var idx C.uint32_t
	err := call(func() C.int { return C.cg_http_policy_index(e.h, cs, &idx) })
	return uint32(idx), err
}

// ExportHTTPPolicy returns the compiled tables as an image; ImportHTTPPolicy
// installs one on another handle (one compile per node, SURVEY §8(e)).
func (e *Engine) ExportHTTPPolicy() ([]byte, error) {
	var n C.size_t
	if err := call(func() C.int { return C.cg_http_policy_export(e.h, nil, 0, &n) }); err != nil {
		return nil, err
	}
	img := make([]byte, int(n))
	err := call(func() C.int { return C.cg_http_policy_export(e.h, unsafe.Pointer(&img[0]), n, &n) })
	return img, err
}

// ImportHTTPPolicy installs an image (all-or-nothing; PolicyRejected for a
// damaged image or one of another library build).
func (e *Engine) ImportHTTPPolicy(img []byte) error {
	if len(img) == 0 {
		return &Error{Code: InvalidArgument, Msg: "empty image"}
	}
	return call(func() C.int { return C.cg_http_policy_import(e.h, unsafe.Pointer(&img[0]), C.size_t(len(img))) })
}

// ShareHTTPPolicy copies this handle's compiled HTTP policy to the others.
func (e *Engine) ShareHTTPPolicy(others []*Engine) error {
	img, err := e.ExportHTTPPolicy()
	if err != nil {
		return err
	}
	for _, o := range others {
		if err := o.ImportHTTPPolicy(img); err != nil {
			return err
		}
	}
	return nil
}

// HTTPRequest is what AccessFilter::decodeHeaders hands to
// NetworkPolicyMap::Allowed (envoy/cilium_l7policy.cc:127-182): the policy,
// direction, destination port, remote identity (source on ingress,
// destination on egress, :144-150) and the header map.
type HTTPRequest struct {
	Policy  uint32 // PolicyIndex; ^uint32(0) = unknown (deny)
	Ingress bool
	Port    uint16
	Remote  uint32
	Headers [][2]string // names case-insensitive; the first value of a name wins
}

// HTTPVerdicts decides a batch (header lists grouped, packed and evaluated
// on the GPU): true = allow, false = deny (→ 403).
func (e *Engine) HTTPVerdicts(reqs []HTTPRequest) ([]bool, error) {
	n := len(reqs)
	out := make([]bool, n)
	if n == 0 {
		return out, nil
	}
	var blob []byte
	off := make([]uint64, n+1)
	policy := make([]uint32, n)
	ingress := make([]uint8, n)
	port := make([]uint16, n)
	remote := make([]uint32, n)
	for i, r := range reqs {
		for _, h := range r.Headers {
			blob = append(blob, h[0]...)
			blob = append(blob, 0)
			blob = append(blob, h[1]...)
			blob = append(blob, 0)
		}
		off[i+1] = uint64(len(blob))
		policy[i], port[i], remote[i] = r.Policy, r.Port, r.Remote
		if r.Ingress {
			ingress[i] = 1
		}
	}
	if len(blob) == 0 {
		blob = []byte{0}
	}
	v := make([]uint8, n)
	err := call(func() C.int { return C.cg_http_verdicts_fields_host(e.h, bytesPtr(blob), (*C.uint64_t)(unsafe.Pointer(&off[0])),
		C.size_t(n), (*C.uint32_t)(unsafe.Pointer(&policy[0])), (*C.uint8_t)(unsafe.Pointer(&ingress[0])),
		(*C.uint16_t)(unsafe.Pointer(&port[0])), (*C.uint32_t)(unsafe.Pointer(&remote[0])), bytesPtr(v)) })
	for i := range v {
		out[i] = v[i] != 0
	}
	return out, err
}

// HTTPVerdictsRawDev decides raw HTTP/1 request heads already in device
// memory (the Envoy codec step, packing and verdicts on the GPU).
func (e *Engine) HTTPVerdictsRawDev(raw, rawOff, policy, ingress, port, remote, out unsafe.Pointer, n int,
	stream unsafe.Pointer) error {
	return call(func() C.int { return C.cg_http_verdicts_raw_dev(e.h, (*C.uint8_t)(raw), (*C.uint64_t)(rawOff), C.size_t(n),
		(*C.uint32_t)(policy), (*C.uint8_t)(ingress), (*C.uint16_t)(port), (*C.uint32_t)(remote), (*C.uint8_t)(out),
		stream) })
}

// HTTPRuleInfo is what each per-rule hit counter counts (cg_http_rule_info).
type HTTPRuleInfo struct {
	Policy, Ingress, Port, Scope, Rule, HTTPRule uint32
}

// HTTPRules returns the rule table the per-rule counters follow.
func (e *Engine) HTTPRules() ([]HTTPRuleInfo, error) {
	var n C.size_t
	if err := call(func() C.int { return C.cg_http_rule_info_get(e.h, nil, 0, &n) }); err != nil {
		return nil, err
	}
	out := make([]HTTPRuleInfo, int(n))
	if n == 0 {
		return out, nil
	}
	err := call(func() C.int { return C.cg_http_rule_info_get(e.h, (*C.cg_http_rule_info)(unsafe.Pointer(&out[0])), n, &n) })
	return out, err
}

// HTTPStats is cg_http_policy_stats's u64 vector.
func (e *Engine) HTTPStats() ([]uint64, error) {
	out := make([]uint64, 16)
	err := call(func() C.int { return C.cg_http_policy_stats(e.h, (*C.uint64_t)(unsafe.Pointer(&out[0])), C.size_t(len(out))) })
	return out, err
}
