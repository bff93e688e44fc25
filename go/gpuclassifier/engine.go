// Package gpuclassifier binds libciliumgpu.so, the MI355X batched
// policy-verdict engine (include/cilium_gpu.h), for the Go agent.
//
// It is the cgo layer of SURVEY §7 step 3: the reference's types keep their
// field names and JSON tags (types.go), and each method names the reference
// call site it replaces.  The package imports nothing from the reference (the
// agent converts its own values with the mirror types), so it builds against
// the header and the library alone:
//
//	go build ./gpuclassifier   (with CGO_ENABLED=1, gcc, libciliumgpu.so)
//
// Ownership and errors follow the C ABI: every buffer is caller-owned and is
// not retained after a call returns; every failure is an *Error carrying the
// cg_result code and cg_last_error's message.  There is no CPU fallback: a
// handle opened on device -1 compiles policies and builds tables, and its
// verdict calls return CG_NO_DEVICE.
package gpuclassifier

// #cgo CFLAGS: -I${SRCDIR}/../../include
// #cgo LDFLAGS: -L${SRCDIR}/../../cilium_amd -lciliumgpu -Wl,-rpath,${SRCDIR}/../../cilium_amd
// #include <stdlib.h>
// #include "cilium_gpu.h"
import "C"

import (
	"fmt"
	"runtime"
	"strconv"
	"unsafe"
)

// Result codes (cg_result); the first eight share proxylib's FilterResult
// numbering (proxylib/proxylib/types.h:38-47).
const (
	OK                = int(C.CG_OK)
	PolicyDrop        = int(C.CG_POLICY_DROP)
	ParserError       = int(C.CG_PARSER_ERROR)
	UnknownParser     = int(C.CG_UNKNOWN_PARSER)
	UnknownConnection = int(C.CG_UNKNOWN_CONNECTION)
	InvalidAddress    = int(C.CG_INVALID_ADDRESS)
	InvalidInstance   = int(C.CG_INVALID_INSTANCE)
	UnknownError      = int(C.CG_UNKNOWN_ERROR)
	InvalidArgument   = int(C.CG_INVALID_ARGUMENT)
	NoDevice          = int(C.CG_NO_DEVICE)
	DeviceError       = int(C.CG_DEVICE_ERROR)
	PolicyRejected    = int(C.CG_POLICY_REJECTED)
	RevisionMismatch  = int(C.CG_REVISION_MISMATCH)
	MapFull           = int(C.CG_MAP_FULL)
	NotFound          = int(C.CG_NOT_FOUND)
	NoMap             = int(C.CG_NO_MAP)
	Unsupported       = int(C.CG_UNSUPPORTED)
)

// Error is a failed engine call.
type Error struct {
	Code int
	Msg  string
}

func (e *Error) Error() string { return fmt.Sprintf("libciliumgpu [%d]: %s", e.Code, e.Msg) }

// call runs one engine call and, on failure, reads cg_last_error on the same
// OS thread: the message is thread-local in the library (runtime.cc), and a
// goroutine may move between threads from one cgo call to the next.
func call(f func() C.int) error {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	rc := f()
	if rc == C.CG_OK {
		return nil
	}
	return &Error{Code: int(rc), Msg: C.GoString(C.cg_last_error())}
}

// Engine is one handle bound to one GPU (cg_open).  Handles are safe for
// concurrent use; policy updates publish atomically.
type Engine struct{ h C.uint64_t }

// Open replaces proxylib OpenModule (proxylib/libcilium.h:107-115): device
// is the HIP ordinal, -1 for a host-only handle.
func Open(device int) (*Engine, error) {
	k, v := C.CString("device"), C.CString(strconv.Itoa(device))
	defer C.free(unsafe.Pointer(k))
	defer C.free(unsafe.Pointer(v))
	kv := C.cg_kv{key: k, value: v}
	var h C.uint64_t
	err := call(func() C.int {
		if h = C.cg_open(&kv, 1, 0); h == 0 { // OpenModule convention: 0 = error
			return C.CG_NO_DEVICE
		}
		return C.CG_OK
	})
	if err != nil {
		return nil, err
	}
	return &Engine{h: h}, nil
}

// Close releases the handle (CloseModule).
func (e *Engine) Close() {
	if e.h != 0 {
		C.cg_close(e.h)
		e.h = 0
	}
}

// Version is the library's build string.
func Version() string { return C.GoString(C.cg_version()) }

// Sync waits for the handle's stream.
func (e *Engine) Sync() error { return call(func() C.int { return C.cg_sync(e.h) }) }

// RegexValidate checks a pattern without compiling it: go = Go 1.10
// regexp.Compile's syntax (PortRuleHTTP.Sanitize,
// pkg/policy/api/http.go:66-84), else std::regex ECMAScript (what Envoy
// compiles for regex_match).
func RegexValidate(re string, goSyntax bool) error {
	flavour := C.uint32_t(C.CG_REGEX_ECMA)
	if goSyntax {
		flavour = C.CG_REGEX_GO
	}
	cs := C.CString(re)
	defer C.free(unsafe.Pointer(cs))
	return call(func() C.int { return C.cg_regex_validate(cs, C.size_t(len(re)), flavour) })
}

// bytesPtr is the address of a byte slice's first element, nil when empty.
func bytesPtr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}
