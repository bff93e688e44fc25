package gpuclassifier

import "net"

// Classifier is the drop-in interface the agent programs against
// (BASELINE north_star): the L4 policy map, the XDP prefilter, the ipcache,
// the Envoy HTTP policy and the Kafka redirect rules, each behind the
// reference's own types, decided in batches on the GPU.
type Classifier interface {
	NewPolicyMap(maxEntries uint32) (*PolicyMap, error)
	NewPreFilter(config, maxLPM, maxHash uint32) (*PreFilter, error)
	NewIPCache(maxEntries uint32) (*IPCache, error)
	UpdateNPDS(discoveryResponse []byte) error
	UpdateNetworkPoliciesJSON(policies []byte) error
	PolicyIndex(name string) (uint32, error)
	HTTPVerdicts(reqs []HTTPRequest) ([]bool, error)
	UpdateKafka(redirects []KafkaRedirect) error
	KafkaVerdicts(reqs []KafkaRequest) ([]bool, error)
	ReadCounters(what, pfOrMap uint32) ([]uint64, error)
	Close()
}

var _ Classifier = (*Engine)(nil)

// L4 is the policy-map side of Classifier, as pkg/maps/policymap's callers
// use it (pkg/endpoint/endpoint.go:2621-2720 syncPolicyMap).
type L4 interface {
	AllowKey(k PolicyKey, proxyPort uint16) error
	DeleteKey(k PolicyKey) error
	Exists(k PolicyKey) bool
	DumpToSlice() ([]PolicyKey, []PolicyEntry, error)
	Flush() error
	Verdicts(tuples []L4Tuple) ([]int32, error)
}

var _ L4 = (*PolicyMap)(nil)

// Prefilter is the PreFilter side (daemon/prefilter.go:66-86 calls Insert).
type Prefilter interface {
	Insert(revision int64, nets []net.IPNet) (int64, error)
	Delete(revision int64, nets []net.IPNet) (int64, error)
	SetEndpoints(v4 []net.IP, v6 []net.IP) error
}

var _ Prefilter = (*PreFilter)(nil)
