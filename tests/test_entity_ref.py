"""Entity selectors pinned to pkg/policy/api/entity_test.go:26-75
(TestEntityMatches, TestEntitySliceMatches) after InitEntities("cluster1")."""
import pytest

from cilium_amd import resolve as R


def _labels(*strs):
    """labels.ParseLabelArray: "source:key=value" (source and value optional)."""
    out = {}
    for s in strs:
        k, _, v = s.partition("=")
        out[k] = v
    return out


def _matches(entities, lbls):
    return any(sel.matches(lbls) for e in entities for sel in R._ENTITY_SELECTORS[e])


CL = f"k8s:{R.POLICY_LABEL_CLUSTER}=cluster1"
CASES = [  # (entities, labels, expect) — entity_test.go line
    (["host"], ["reserved:host"], True), (["host"], ["reserved:host", "id:foo"], True),            # :29-30
    (["host"], ["reserved:world"], False), (["host"], ["id=foo"], False),                           # :31-32
    (["all"], ["reserved:host"], True), (["all"], ["reserved:world"], True), (["all"], ["id=foo"], True),  # :34-36
    (["cluster"], ["reserved:host"], True), (["cluster"], ["reserved:init"], True),                # :38-39
    (["cluster"], ["reserved:world"], False),                                                       # :40
    (["cluster"], [CL, "id=foo"], True), (["cluster"], [CL, "id=foo", "id=bar"], True),            # :43-44
    (["cluster"], ["id=foo"], False),                                                               # :45
    (["world"], ["reserved:host"], False), (["world"], ["reserved:world"], True),                   # :47-48
    (["world"], ["id=foo"], False), (["world"], ["id=foo", "id=bar"], False),                       # :49-50
    (["host", "world"], ["reserved:host"], True), (["host", "world"], ["reserved:world"], True),    # :57-58
    (["host", "world"], ["id=foo"], False),                                                         # :59
]


@pytest.fixture
def cluster1():
    R.init_entities("cluster1")
    yield
    R.init_entities()


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{'+'.join(c[0])}:{','.join(c[1])}")
def test_entity_matches(cluster1, case):
    entities, lbls, want = case
    assert _matches(entities, _labels(*lbls)) == want


def test_selects_all_endpoints():
    """selector_test.go:32-47 (EndpointSelectorSlice.SelectsAllEndpoints)."""
    bar, foo = R.EndpointSelector.of({"bar": ""}), R.EndpointSelector.of({"foo": ""})
    assert R.selects_all([])
    assert R.selects_all([R.WILDCARD])
    assert R.selects_all([R.WILDCARD, bar])
    assert not R.selects_all([bar, foo])
