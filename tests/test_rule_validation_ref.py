"""Rule.Sanitize pinned to pkg/policy/api/rule_validation_test.go:28-352
(TestL7RulesWithNonTCPProtocols, TestL7Rules): each rule of the test, in
the policy JSON form, accepted or refused with the test's message."""
import pytest

from cilium_amd import resolve as R

GET = {"http": [{"method": "GET", "path": "/"}]}


def _rule(ports, rules):
    return {"endpointSelector": {}, "ingress": [{"fromEndpoints": [{}], "toPorts": [
        {"ports": [{"port": p, "protocol": pr} for p, pr in ports], **({"rules": rules} if rules else {})}]}]}


CASES = [  # (source lines, rule, error message or None)
    (":30-52", _rule([("80", "TCP"), ("81", "TCP")], GET), None),
    (":54-75", _rule([("80", "UDP")], GET), "L7 rules can only apply exclusively to TCP, not UDP"),
    (":77-99", _rule([("80", "ANY")], GET), "L7 rules can only apply exclusively to TCP, not ANY"),
    (":101-124", _rule([("80", "TCP"), ("12345", "UDP")], GET), "L7 rules can only apply exclusively to TCP, not UDP"),
    (":126-149", _rule([("80", "UDP"), ("12345", "TCP")], GET), "L7 rules can only apply exclusively to TCP, not UDP"),
    (":280-303", _rule([("80", "TCP"), ("81", "TCP")],
                       {"l7proto": "test.lineparser", "l7": [{"method": "PUT", "path": "/"},
                                                            {"method": "GET", "path": "/"}]}), None),
    (":305-325", _rule([("80", "TCP"), ("81", "TCP")], {"l7proto": "test.lineparser"}), None),
    (":327-351", _rule([("80", "TCP"), ("81", "TCP")],
                       {"l7proto": "test.lineparser", "l7": [{"method": "PUT", "": "Foo"}]}), "Empty key not allowed"),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
def test_rule_sanitize(case):
    _, rule, err = case
    r = R.Rule.from_json(rule)
    if err is None:
        r.sanitize()
    else:
        with pytest.raises(ValueError) as ei:
            r.sanitize()
        assert str(ei.value) == err


@pytest.mark.parametrize("sel", [R.WILDCARD, R.EndpointSelector.of({"bar": ""})], ids=["wildcard", "bar"])
def test_create_l4_filter(sel):
    """l4_test.go:58-83 (TestCreateL4Filter): one L7 rule entry whether the
    selector is the wildcard or label-based, ingress and egress."""
    from cilium_amd.policy import L7Rules, PortRuleHTTP
    rules = L7Rules(HTTP=[PortRuleHTTP(Path="/public", Method="GET")])
    assert len(R.create_l4_ingress_filter([sel], [], rules, 80, "TCP").L7RulesPerEp) == 1
    assert len(R.create_l4_egress_filter([sel], rules, 80, "TCP").L7RulesPerEp) == 1


def test_invalid_policies_runtime():
    """test/runtime/Policies.go:1614-1657 ("Invalid Policies"): both imports
    fail.  The truncated document is not JSON; the 50-port rule as the test
    renders it (objects without commas) is not JSON either, and written as a
    list it breaks the 40-port limit (rule_validation.go:317-319)."""
    import json
    with pytest.raises(json.JSONDecodeError):
        json.loads('[{"endpointSelector": {"matchLabels":{"id.httpd1":""}},')
    ports = "".join(f'{{"port": "{i}", "protocol": "tcp"}}' for i in range(50))
    doc = ('[{"endpointSelector": {"matchLabels": {"foo": ""}}, "ingress": [{"fromEndpoints": '
           '[{"matchLabels": {"reserved:host": ""}}, {"matchLabels": {"bar": ""}}], "toPorts": [{"ports": [%s]}]}]}]')
    with pytest.raises(json.JSONDecodeError):
        json.loads(doc % ports)
    rules = json.loads(doc % ", ".join(f'{{"port": "{i}", "protocol": "tcp"}}' for i in range(50)))
    with pytest.raises(ValueError) as ei:
        R.Repository([R.Rule.from_json(r) for r in rules])
    assert str(ei.value) == "too many ports, the max is 40"
