"""cilium_amd — MI355X-native batched policy-verdict engine for Cilium's
classification path (L4 policymap, XDP CIDR prefilter, HTTP and Kafka L7).

The verdicts are computed by hand-written HIP kernels for gfx950 in
``libciliumgpu.so`` (sources in ``csrc/``), reached through the C ABI in
``include/cilium_gpu.h``.  Build with ``python -m cilium_amd.build``.
"""
from . import policy  # noqa: F401  (pure-Python rule types; no native dependency)

__all__ = ["policy", "Classifier", "PolicyMap", "PreFilter"]


def __getattr__(name):
    # The native library is loaded lazily so that rule types import without it.
    if name in ("Classifier", "PolicyMap", "PreFilter"):
        from . import classifier
        return getattr(classifier, name)
    raise AttributeError(name)
