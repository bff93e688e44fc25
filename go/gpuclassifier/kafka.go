package gpuclassifier

// #include <stdlib.h>
// #include "cilium_gpu.h"
import "C"

import (
	"encoding/json"
	"unsafe"
)

// KafkaRequest is the packed 64-byte record kafkaRedirect.canAccess decides
// (pkg/proxy/kafka.go:117-153 over pkg/kafka/policy.go:144-225).
type KafkaRequest struct {
	APIKey     int16
	APIVersion int16
	Kind       uint8 // KafkaKindNil / KafkaKindTyped / KafkaKindConsumerMetadata
	NTopics    uint8
	Policy     uint16 // redirect index (KafkaPolicyIndex); 0xFFFF = unknown (deny)
	Remote     uint32 // source identity (0 = unknown: wildcard rules only)
	ClientID   uint32 // KafkaIntern(1, ...), KafkaUnknownString if not a rule string
	TopicIDs   [12]uint32
}

const (
	KafkaKindNil              = uint8(C.CG_KAFKA_K_NIL)
	KafkaKindTyped            = uint8(C.CG_KAFKA_K_TYPED)
	KafkaKindConsumerMetadata = uint8(C.CG_KAFKA_K_CONSUMER_METADATA)
	KafkaUnknownString        = uint32(C.CG_KAFKA_UNKNOWN_STR)
)

// UpdateKafka installs the rule sets of the Kafka redirects
// (Redirect.updateRules, pkg/proxy/redirect.go:68-82); every PortRuleKafka
// is Sanitize()d and a failure rejects the whole update.
func (e *Engine) UpdateKafka(redirects []KafkaRedirect) error {
	b, err := json.Marshal(redirects)
	if err != nil {
		return err
	}
	cs := C.CBytes(b)
	defer C.free(cs)
	return call(func() C.int { return C.cg_kafka_policy_update(e.h, (*C.char)(cs), C.size_t(len(b))) })
}

// KafkaPolicyIndex is the redirect index requests carry.
func (e *Engine) KafkaPolicyIndex(name string) (uint16, error) {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var idx C.uint32_t
	err := call(func() C.int { return C.cg_kafka_policy_index(e.h, cs, &idx) })
	return uint16(idx), err
}

// KafkaIntern maps a topic (what = 0) or clientID (what = 1) to its id.
func (e *Engine) KafkaIntern(what uint32, s string) uint32 {
	cs := C.CString(s)
	defer C.free(unsafe.Pointer(cs))
	var id C.uint32_t
	if call(func() C.int { return C.cg_kafka_intern(e.h, C.uint32_t(what), cs, C.size_t(len(s)), &id) }) != nil {
		return KafkaUnknownString
	}
	return uint32(id)
}

// KafkaVerdicts decides packed requests: true = forward, false = deny
// (ErrTopicAuthorizationFailed, pkg/proxy/kafka.go:249-260).
func (e *Engine) KafkaVerdicts(reqs []KafkaRequest) ([]bool, error) {
	out := make([]bool, len(reqs))
	if len(reqs) == 0 {
		return out, nil
	}
	v := make([]uint8, len(reqs))
	err := call(func() C.int { return C.cg_kafka_verdicts_host(e.h, (*C.cg_kafka_request)(unsafe.Pointer(&reqs[0])), C.size_t(len(reqs)),
		nil, 0, bytesPtr(v)) })
	for i := range v {
		out[i] = v[i] != 0
	}
	return out, err
}

// KafkaVerdictsRaw decodes wire requests (ReadRequest, pkg/kafka/request.go:
// 186-229) and decides them: KafkaAllow / KafkaDeny / KafkaClose (the
// decode failed: the proxy closes the connection).
func (e *Engine) KafkaVerdictsRaw(raw []byte, rawOff []uint64, redirect []uint16, remote []uint32) ([]uint8, error) {
	n := len(rawOff) - 1
	out := make([]uint8, n)
	if n <= 0 {
		return out, nil
	}
	err := call(func() C.int { return C.cg_kafka_verdicts_raw_host(e.h, bytesPtr(raw), (*C.uint64_t)(unsafe.Pointer(&rawOff[0])),
		C.size_t(n), (*C.uint16_t)(unsafe.Pointer(&redirect[0])), (*C.uint32_t)(unsafe.Pointer(&remote[0])),
		bytesPtr(out)) })
	return out, err
}

const (
	KafkaDeny  = uint8(C.CG_KAFKA_V_DENY)
	KafkaAllow = uint8(C.CG_KAFKA_V_ALLOW)
	KafkaClose = uint8(C.CG_KAFKA_V_CLOSE)
)
