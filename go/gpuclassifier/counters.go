package gpuclassifier

// #include "cilium_gpu.h"
import "C"

import "unsafe"

// Counter sets (cg_read_counters): the per-entry packets/bytes of the BPF
// policy map (policy.h:68-69) come with DumpToSlice; these are the L7 and
// prefilter ones (policy_l7_forwarded/denied_total, pkg/metrics/metrics.go:
// 270-296).
const (
	CountersHTTPPrograms  = uint32(C.CG_CTR_HTTP_PROGRAMS)
	CountersKafka         = uint32(C.CG_CTR_KAFKA)
	CountersPrefilter     = uint32(C.CG_CTR_PREFILTER)
	CountersHTTPRules     = uint32(C.CG_CTR_HTTP_RULES)
	CountersHTTPAllReduce = uint32(C.CG_CTR_HTTP_ALLREDUCE)
)

// ReadCounters returns a counter vector; pfOrMap names the prefilter for
// CountersPrefilter.
func (e *Engine) ReadCounters(what, pfOrMap uint32) ([]uint64, error) {
	var n C.size_t
	if err := call(func() C.int { return C.cg_read_counters(e.h, C.uint32_t(what), C.uint32_t(pfOrMap), nil, 0, &n) }); err != nil {
		return nil, err
	}
	out := make([]uint64, int(n))
	if n == 0 {
		return out, nil
	}
	err := call(func() C.int { return C.cg_read_counters(e.h, C.uint32_t(what), C.uint32_t(pfOrMap), (*C.uint64_t)(unsafe.Pointer(&out[0])),
		n, &n) })
	return out, err
}

// CountersDevice is the device buffer of a counter vector, for an RCCL
// all-reduce across the node's GPUs (SURVEY §8(e)).
func (e *Engine) CountersDevice(what, pfOrMap uint32) (unsafe.Pointer, int, error) {
	var p unsafe.Pointer
	var n C.size_t
	err := call(func() C.int { return C.cg_counters_device_ptr(e.h, C.uint32_t(what), C.uint32_t(pfOrMap), &p, &n) })
	return p, int(n), err
}

// ResetCounters zeroes every counter of the handle.
func (e *Engine) ResetCounters() error { return call(func() C.int { return C.cg_reset_counters(e.h) }) }
