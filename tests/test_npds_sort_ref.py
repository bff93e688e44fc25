"""NPDS sort order (pkg/envoy/sort.go) pinned to pkg/envoy/sort_test.go:29-254:
each slice, given in reverse, sorts back into the test's expected order under
the restated comparators (resolve.py _hm_key, _http_rule_cmp, _pnpr_cmp,
_pnp_cmp).  The objects are the test's, in the engine's NPDS JSON form."""
import functools

from cilium_amd import resolve as R

HM = [{"name": "aaa", "regex_match": "aaa"}, {"name": "bbb", "regex_match": "aaa"},   # HeaderMatcher1..4 (:29-47)
      {"name": "bbb", "regex_match": "bbb"}, {"name": "bbb", "regex_match": "bbb"}]
HR = [[], [HM[0]], [HM[0], HM[1]], [HM[0], HM[2]]]                                     # HTTPNetworkPolicyRule1..4 (:68-80)


def _pnpr(remotes, http=None):
    r = {"remote_policies": list(remotes)}
    if http is not None:
        r["http_rules"] = {"http_rules": [{"headers": h} for h in http]}
    return r


PNPR = [_pnpr([]), _pnpr([1]), _pnpr([1, 2]), _pnpr([], [HR[0]]), _pnpr([1, 2], [HR[0]]),  # :101-160
        _pnpr([1, 2], [HR[0], HR[1]]), _pnpr([1, 2], [HR[0], HR[2]])]
PNP = [{"protocol": "TCP", "port": 10001, "rules": []}, {"protocol": "UDP", "port": 10001, "rules": []},  # :189-231
       {"protocol": "UDP", "port": 10002, "rules": []}, {"protocol": "UDP", "port": 10002, "rules": [PNPR[0]]},
       {"protocol": "UDP", "port": 10002, "rules": [PNPR[0], PNPR[1]]},
       {"protocol": "UDP", "port": 10002, "rules": [PNPR[0], PNPR[2]]}]


def test_sort_header_matchers():  # :49-66
    assert sorted(reversed(HM), key=R._hm_key) == HM


def test_sort_http_network_policy_rules():  # :82-99
    assert sorted(reversed(HR), key=functools.cmp_to_key(R._http_rule_cmp)) == HR


def test_sort_port_network_policy_rules():  # :164-187
    assert sorted(reversed(PNPR), key=functools.cmp_to_key(R._pnpr_cmp)) == PNPR


def test_sort_port_network_policies():  # :233-254
    assert sorted(reversed(PNP), key=functools.cmp_to_key(R._pnp_cmp)) == PNP
