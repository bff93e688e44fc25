/*
 * cilium_proxylib.h — the proxylib C ABI exported by libciliumgpu.so, so
 * that Envoy's cilium proxylib filter can dlopen the engine unchanged
 * (envoy/cilium_proxylib.cc:18-61 resolves these symbol names).
 *
 * Same symbols, argument order and types as the reference's cgo exports
 * (proxylib/libcilium.h:77-115, types proxylib/proxylib/types.h:22-50,
 * implementation proxylib/proxylib.go:56-155).  Frames are parsed on the
 * host (r2d2 line framing, proxylib/r2d2/r2d2parser.go:148-199); the policy
 * verdicts of all request frames of one OnData call run as one batch in the
 * engine's http_kernel on the GPU.
 *
 * Policies: the reference streams them over xDS (NPDS gRPC, xds-path); here
 * they are installed with cg_proxylib_policy_update (include/cilium_gpu.h)
 * on the instance id OpenModule returned.
 */
#ifndef CILIUM_PROXYLIB_H
#define CILIUM_PROXYLIB_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  const char* p;
  ptrdiff_t n;
} GoString;

typedef struct {
  void* data;
  int64_t len;
  int64_t cap;
} GoSlice;

typedef enum {
  FILTEROP_MORE,
  FILTEROP_PASS,
  FILTEROP_DROP,
  FILTEROP_INJECT,
  FILTEROP_ERROR,
} FilterOpType;

typedef enum {
  FILTEROP_ERROR_INVALID_OP_LENGTH = 1,
  FILTEROP_ERROR_INVALID_FRAME_TYPE,
  FILTEROP_ERROR_INVALID_FRAME_LENGTH,
} FilterOpError;

typedef struct {
  uint64_t op;      /* FilterOpType */
  int64_t n_bytes;  /* > 0 */
} FilterOp;

typedef enum {
  FILTER_OK,
  FILTER_POLICY_DROP,
  FILTER_PARSER_ERROR,
  FILTER_UNKNOWN_PARSER,
  FILTER_UNKNOWN_CONNECTION,
  FILTER_INVALID_ADDRESS,
  FILTER_INVALID_INSTANCE,
  FILTER_UNKNOWN_ERROR,
} FilterResult;

/* OnNewConnection (libcilium.h:77, proxylib.go:56-76).  origBuf/replyBuf
 * are caller-owned inject buffers ([]byte with fixed capacity). */
FilterResult OnNewConnection(uint64_t instanceId, GoString proto, uint64_t connectionId, uint8_t ingress,
                             uint32_t srcId, uint32_t dstId, GoString srcAddr, GoString dstAddr,
                             GoString policyName, GoSlice* origBuf, GoSlice* replyBuf);
/* OnData (libcilium.h:101, connection.go:118-174): data is a [][]byte,
 * filterOps a []FilterOp appended to up to its capacity. */
FilterResult OnData(uint64_t connectionId, uint8_t reply, uint8_t endStream, GoSlice* data, GoSlice* filterOps);
/* Close (libcilium.h:104). */
void Close(uint64_t connectionId);
/* OpenModule (libcilium.h:110, proxylib.go:118-150): params is a [][2]string
 * of access-log-path, xds-path, node-id; any other key → 0 (error).  The GPU
 * is CILIUM_GPU_DEVICE (default 0; -1 = a host-only instance that parses
 * frames and installs policies but cannot evaluate them). */
uint64_t OpenModule(GoSlice params, uint8_t debug);
/* CloseModule (libcilium.h:114). */
void CloseModule(uint64_t id);

#ifdef __cplusplus
}
#endif

#endif /* CILIUM_PROXYLIB_H */
