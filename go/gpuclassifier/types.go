package gpuclassifier

// Mirror types of the reference's classification inputs (SURVEY §8(b)):
// same field names, meanings and JSON tags, defined here so that this
// package imports nothing from the agent.

// TrafficDirection is policymap.TrafficDirection
// (pkg/maps/policymap/trafficdirection.go:20-29).
type TrafficDirection uint8

const (
	Ingress TrafficDirection = 0
	Egress  TrafficDirection = 1
)

// PolicyKey is policymap.PolicyKey (policymap.go:64-69).  DestPort is in
// network byte order, as in the BPF map.
type PolicyKey struct {
	Identity         uint32 `align:"sec_label"`
	DestPort         uint16 `align:"dport"`
	Nexthdr          uint8  `align:"protocol"`
	TrafficDirection uint8  `align:"egress"`
}

// PolicyEntry is policymap.PolicyEntry (policymap.go:73-80).  ProxyPort is in
// network byte order.
type PolicyEntry struct {
	ProxyPort uint16 `align:"proxy_port"`
	Pad0      uint16
	Pad1      uint16
	Pad2      uint16
	Packets   uint64 `align:"packets"`
	Bytes     uint64 `align:"bytes"`
}

// PortRuleHTTP is api.PortRuleHTTP (pkg/policy/api/http.go:28-60).
type PortRuleHTTP struct {
	Path    string   `json:"path,omitempty"`
	Method  string   `json:"method,omitempty"`
	Host    string   `json:"host,omitempty"`
	Headers []string `json:"headers,omitempty"`
}

// Sanitize is PortRuleHTTP.Sanitize (http.go:66-84): Path and Method must be
// valid Go regexps; Host and Headers are not checked.
func (h *PortRuleHTTP) Sanitize() error {
	if h.Path != "" {
		if err := RegexValidate(h.Path, true); err != nil {
			return err
		}
	}
	if h.Method != "" {
		if err := RegexValidate(h.Method, true); err != nil {
			return err
		}
	}
	return nil
}

// PortRuleKafka is api.PortRuleKafka (pkg/policy/api/kafka.go:26-107);
// the engine runs Sanitize (rule_validation.go:232-275) on every rule it is
// given.
type PortRuleKafka struct {
	Role       string `json:"role,omitempty"`
	APIKey     string `json:"apiKey,omitempty"`
	APIVersion string `json:"apiVersion,omitempty"`
	ClientID   string `json:"clientID,omitempty"`
	Topic      string `json:"topic,omitempty"`
}

// PortRuleL7 is api.PortRuleL7 (pkg/policy/api/l7.go:24).
type PortRuleL7 map[string]string

// L7Rules is api.L7Rules (pkg/policy/api/l4.go:65-85).
type L7Rules struct {
	HTTP    []PortRuleHTTP  `json:"http,omitempty"`
	Kafka   []PortRuleKafka `json:"kafka,omitempty"`
	L7Proto string          `json:"l7proto,omitempty"`
	L7      []PortRuleL7    `json:"l7,omitempty"`
}

// KafkaSelectorRules is one entry of a redirect's L7DataMap
// (pkg/policy/l4.go:32) with its selector resolved to identities (nil: the
// wildcard selector), as Redirect.updateRules copies it
// (pkg/proxy/redirect.go:68-82).
type KafkaSelectorRules struct {
	Identities []uint32        `json:"identities"`
	Rules      []PortRuleKafka `json:"rules"`
}

// KafkaRedirect is the rule set of one Kafka redirect.
type KafkaRedirect struct {
	Name      string               `json:"name"`
	Selectors []KafkaSelectorRules `json:"selectors"`
}

// L4Tuple is one packet's __policy_can_access arguments
// (bpf/lib/policy.h:46-49), 12 bytes; dport in network byte order.
type L4Tuple struct {
	Identity uint32
	DPort    uint16
	Proto    uint8
	Flags    uint8 // L4Ingress | L4Fragment | L4CBPolicy
	Len      uint32
}

// L4 tuple flags and verdict values (policy.h, common.h:240,264).
const (
	L4Ingress         = 0x01
	L4Fragment        = 0x02
	L4CBPolicy        = 0x04
	DropPolicy        = -133
	DropFragNoSupport = -157
)

// FilterResult is proxylib's (proxylib/proxylib/types.go:24-102).
type FilterResult int

const (
	FilterOK FilterResult = iota
	FilterPolicyDrop
	FilterParserError
	FilterUnknownParser
	FilterUnknownConnection
	FilterInvalidAddress
	FilterInvalidInstance
	FilterUnknownError
)

// OpType is proxylib's FilterOpType.
type OpType uint64

const (
	MORE OpType = iota
	PASS
	DROP
	INJECT
	ERROR
)
