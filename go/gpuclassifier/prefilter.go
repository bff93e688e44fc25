package gpuclassifier

// #include "cilium_gpu.h"
import "C"

import (
	"net"
	"unsafe"
)

// PreFilter config bits (preFilterConfig, pkg/datapath/prefilter/prefilter.go:49-54).
const (
	PrefilterDyn4 = uint32(C.CG_PF_DYN4)
	PrefilterDyn6 = uint32(C.CG_PF_DYN6)
	PrefilterFix4 = uint32(C.CG_PF_FIX4)
	PrefilterFix6 = uint32(C.CG_PF_FIX6)
	XDPDrop       = uint8(C.CG_XDP_DROP)
	XDPPass       = uint8(C.CG_XDP_PASS)
)

// PreFilter mirrors prefilter.PreFilter (prefilter.go:57-298): revisioned
// Insert/Delete with undo, the four maps selected per CIDR (selectMap
// :108-122), and check_v4 / check_v6 (bpf/bpf_xdp.c:97-156) on the GPU.
type PreFilter struct {
	e  *Engine
	id C.uint32_t
}

// NewPreFilter: config 0 = NewPreFilter's default fix4|fix6 (prefilter.go:
// 281-298); maxLPM / maxHash 0 = maxLKeys 65536 / maxHKeys 20M (:43-44).
func (e *Engine) NewPreFilter(config, maxLPM, maxHash uint32) (*PreFilter, error) {
	if config == 0 {
		config = PrefilterFix4 | PrefilterFix6
	}
	var id C.uint32_t
	if err := call(func() C.int { return C.cg_prefilter_create(e.h, C.uint32_t(config), C.uint32_t(maxLPM), C.uint32_t(maxHash),
		&id) }); err != nil {
		return nil, err
	}
	return &PreFilter{e: e, id: id}, nil
}

// Destroy frees the prefilter's tables.
func (pf *PreFilter) Destroy() error { return call(func() C.int { return C.cg_prefilter_destroy(pf.e.h, pf.id) }) }

func cidrs(nets []net.IPNet) []C.cg_cidr {
	out := make([]C.cg_cidr, len(nets))
	for i, n := range nets {
		ones, _ := n.Mask.Size()
		out[i].prefixlen = C.uint8_t(ones)
		if ip4 := n.IP.To4(); ip4 != nil {
			out[i].family = 4
			for k := 0; k < 4; k++ {
				out[i].addr[k] = C.uint8_t(ip4[k])
			}
		} else {
			out[i].family = 6
			for k := 0; k < 16; k++ {
				out[i].addr[k] = C.uint8_t(n.IP[k])
			}
		}
	}
	return out
}

// Insert is PreFilter.Insert (prefilter.go:125-159): revision 0 = any;
// RevisionMismatch is the reference's "Latest revision is %d not %d"
// (:131-133), NoMap its "No map enabled for CIDR" (:137-139).  Returns the
// new revision.
func (pf *PreFilter) Insert(revision int64, nets []net.IPNet) (int64, error) {
	c := cidrs(nets)
	var rev C.int64_t
	var p *C.cg_cidr
	if len(c) > 0 {
		p = &c[0]
	}
	err := call(func() C.int { return C.cg_prefilter_insert(pf.e.h, pf.id, C.int64_t(revision), p, C.size_t(len(c)), &rev) })
	return int64(rev), err
}

// Delete is PreFilter.Delete (prefilter.go:162-203).
func (pf *PreFilter) Delete(revision int64, nets []net.IPNet) (int64, error) {
	c := cidrs(nets)
	var rev C.int64_t
	var p *C.cg_cidr
	if len(c) > 0 {
		p = &c[0]
	}
	err := call(func() C.int { return C.cg_prefilter_delete(pf.e.h, pf.id, C.int64_t(revision), p, C.size_t(len(c)), &rev) })
	return int64(rev), err
}

// SetEndpoints replaces the local endpoint set cilium_lxc
// (bpf_xdp.c:88-95,123-130 → bpf/lib/eps.h:26-46).
func (pf *PreFilter) SetEndpoints(v4 []net.IP, v6 []net.IP) error {
	a4 := make([]uint32, len(v4))
	for i, ip := range v4 {
		b := ip.To4()
		a4[i] = uint32(b[0]) | uint32(b[1])<<8 | uint32(b[2])<<16 | uint32(b[3])<<24 // network order in memory
	}
	a6 := make([]byte, 16*len(v6))
	for i, ip := range v6 {
		copy(a6[16*i:], ip.To16())
	}
	var p4 *C.uint32_t
	if len(a4) > 0 {
		p4 = (*C.uint32_t)(unsafe.Pointer(&a4[0]))
	}
	return call(func() C.int { return C.cg_prefilter_set_endpoints(pf.e.h, pf.id, p4, C.size_t(len(a4)), bytesPtr(a6), C.size_t(len(v6))) })
}

// VerdictsDev runs check_v4 / check_v6 over device records ({saddr, daddr}
// u32 pairs; 32-byte v6 pairs) into one CG_XDP_* byte each.
func (pf *PreFilter) VerdictsDev(v4 unsafe.Pointer, n4 int, out4 unsafe.Pointer, v6 unsafe.Pointer, n6 int,
	out6 unsafe.Pointer, stream unsafe.Pointer) error {
	return call(func() C.int { return C.cg_prefilter_verdicts_dev(pf.e.h, pf.id, (*C.uint32_t)(v4), C.size_t(n4), (*C.uint8_t)(out4),
		(*C.uint8_t)(v6), C.size_t(n6), (*C.uint8_t)(out6), stream) })
}
