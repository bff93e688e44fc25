package gpuclassifier

// #include "cilium_gpu.h"
import "C"

import (
	"net"
	"unsafe"
)

// WorldID is the identity a miss resolves to (bpf/node_config.h:35).
const WorldID = uint32(C.CG_WORLD_ID)

// RemoteEndpointInfo is ipcache.RemoteEndpointInfo
// (pkg/maps/ipcache/ipcache.go:127-130).
type RemoteEndpointInfo struct {
	SecurityIdentity uint32
	TunnelEndpoint   [4]byte
}

// IPCache mirrors ipcache.Map (ipcache.go:36-130) on the device; lookups are
// lookup_ip{4,6}_remote_endpoint (bpf/lib/eps.h:48-115).
type IPCache struct {
	e  *Engine
	id C.uint32_t
}

// NewIPCache: maxEntries 0 = MaxEntries 512000 (ipcache.go:36).
func (e *Engine) NewIPCache(maxEntries uint32) (*IPCache, error) {
	var id C.uint32_t
	if err := call(func() C.int { return C.cg_ipcache_create(e.h, C.uint32_t(maxEntries), &id) }); err != nil {
		return nil, err
	}
	return &IPCache{e: e, id: id}, nil
}

// Destroy frees the ipcache's tables.
func (m *IPCache) Destroy() error { return call(func() C.int { return C.cg_ipcache_destroy(m.e.h, m.id) }) }

// Update is Map.Update of one prefix (BPF_ANY).
func (m *IPCache) Update(n net.IPNet, v RemoteEndpointInfo) error {
	c := cidrs([]net.IPNet{n})
	val := C.cg_remote_endpoint_info{sec_label: C.uint32_t(v.SecurityIdentity),
		tunnel_endpoint: *(*C.uint32_t)(unsafe.Pointer(&v.TunnelEndpoint[0]))}
	return call(func() C.int { return C.cg_ipcache_update(m.e.h, m.id, &c[0], &val, 1) })
}

// Delete is Map.Delete of one prefix.
func (m *IPCache) Delete(n net.IPNet) error {
	c := cidrs([]net.IPNet{n})
	return call(func() C.int { return C.cg_ipcache_delete(m.e.h, m.id, &c[0], 1) })
}

// ResolveDev resolves device addresses as bpf_lxc.c:509-518 does.
func (m *IPCache) ResolveDev(v4 unsafe.Pointer, n4 int, out4 unsafe.Pointer, v6 unsafe.Pointer, n6 int,
	out6 unsafe.Pointer, stream unsafe.Pointer) error {
	return call(func() C.int { return C.cg_ipcache_resolve_dev(m.e.h, m.id, (*C.uint32_t)(v4), C.size_t(n4),
		(*C.cg_remote_endpoint_info)(out4), (*C.uint8_t)(v6), C.size_t(n6), (*C.cg_remote_endpoint_info)(out6),
		stream) })
}

// EgressVerdictsDev is bpf_lxc.c:509-527 in one kernel: each tuple's remote
// identity from its IPv4 destination, then policy_can_egress4.
func (m *IPCache) EgressVerdictsDev(pm *PolicyMap, remoteV4 unsafe.Pointer, tuples unsafe.Pointer, n int,
	verdicts unsafe.Pointer, stream unsafe.Pointer) error {
	return call(func() C.int { return C.cg_l4_verdicts_ipcache_dev(m.e.h, pm.id, m.id, (*C.uint32_t)(remoteV4), (*C.cg_l4_tuple)(tuples),
		C.size_t(n), (*C.int32_t)(verdicts), stream) })
}
