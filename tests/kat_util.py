"""Helpers turning the golden KAT fixtures into engine / oracle inputs."""
import ipaddress
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def http_requests(reqs, policy_index):
    """KAT request dicts → packer / oracle input arrays."""
    parts, off = [], [0]
    for r in reqs:
        b = b"".join(k.encode() + b"\0" + v.encode() + b"\0" for k, v in r["headers"])
        parts.append(b)
        off.append(off[-1] + len(b))
    return dict(policy=np.array([policy_index(r["policy"]) for r in reqs], np.uint32),
                ingress=np.array([r["ingress"] for r in reqs], np.uint8),
                port=np.array([r["port"] for r in reqs], np.uint16),
                remote=np.array([r["remote"] for r in reqs], np.uint32),
                hdr_blob=np.frombuffer(b"".join(parts) or b"\0", np.uint8).copy(),
                hdr_off=np.array(off, np.uint64))


def kafka_case(c):
    """One MatchesRule KAT → (redirect policy, request field lists)."""
    pol = [{"name": "r", "selectors": [{"identities": None, "rules": c["rules"]}]}]
    q = c["request"]
    req = dict(redirect=[0], remote=[0], api_key=[q["api_key"]], api_version=[q["api_version"]], kind=[q["kind"]],
               client_id=[q["client_id"].encode()], topics=[[t.encode() for t in q["topics"]]])
    return pol, req


def lpm_case(c):
    """A covers-KAT as a prefilter query: source = addr, destination = a local
    endpoint, so covered → XDP_DROP (1) and not covered → XDP_PASS (2)."""
    from cilium_amd.classifier import PreFilter
    pfx = PreFilter.cidrs([c["prefix"]])
    a = int(ipaddress.ip_address(c["addr"]))
    ep = 0x0A000001  # 10.0.0.1
    v4 = np.array([[int.from_bytes(a.to_bytes(4, "big"), "little"), int.from_bytes(ep.to_bytes(4, "big"), "little")]],
                  np.uint32)
    ep4 = np.array([int.from_bytes(ep.to_bytes(4, "big"), "little")], np.uint32)
    return pfx, v4, ep4
