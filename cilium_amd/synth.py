"""Synthetic workloads for the BASELINE.json configs (seeded, deterministic).

Each generator follows SURVEY.md §8(d): star-wars HTTP (config 1), L4
policymap (2), CIDR prefilter (3), Kafka (4) and the 10K-rule HTTP set (5).
Requests are returned in the engine's input formats (header blobs for the
HTTP packer, numpy records for L4/LPM, field lists for Kafka).
"""
from __future__ import annotations

import os

import numpy as np

from .policy import (PortRuleHTTP, PortRuleKafka, get_http_rule, htons, network_policy, port_network_policy,
                     port_network_policy_rule)

SEED = 0xC111A
METHODS = [b"GET", b"POST", b"PUT", b"DELETE", b"HEAD", b"PATCH"]


def _blob(reqs: list[list[tuple[bytes, bytes]]]) -> tuple[np.ndarray, np.ndarray]:
    parts = []
    off = [0]
    for hs in reqs:
        b = b"".join(k + b"\0" + v + b"\0" for k, v in hs)
        parts.append(b)
        off.append(off[-1] + len(b))
    return np.frombuffer(b"".join(parts) or b"\0", np.uint8).copy(), np.asarray(off, np.uint64)


# ------------------------------------------------------- config 1: star-wars
SPACESHIP_ID = 257
DEATHSTAR_ID = 258
OTHER_ID = 300


def starwars_rules() -> list[PortRuleHTTP]:
    """examples/demo/sw_policy_http.real.json:13-31."""
    return [PortRuleHTTP(Method="GET", Path="/v1/"),
            PortRuleHTTP(Method="POST", Path="/v1/request-landing/"),
            PortRuleHTTP(Method="PUT", Path="/v1/exhaust-port/", Headers=["X-Has-Force: true"])]


def starwars_policy() -> list[dict]:
    """Two endpoint policies: the spaceship's egress (toPorts without
    toEndpoints → any destination) and the deathstar's ingress restricted to
    the spaceship identity (the L3-dependent variant)."""
    hs = [get_http_rule(r)[0] for r in starwars_rules()]
    return [
        network_policy("spaceship", SPACESHIP_ID,
                       egress=[port_network_policy(80, [port_network_policy_rule([], hs)])]),
        network_policy("deathstar", DEATHSTAR_ID,
                       ingress=[port_network_policy(80, [port_network_policy_rule([SPACESHIP_ID], hs)])]),
    ]


def starwars_requests(n: int, seed: int = SEED):
    rng = np.random.default_rng(seed)
    paths = [b"/v1/", b"/v1/request-landing/", b"/v1/exhaust-port/"]
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", np.uint8)
    reqs = []
    pol = rng.integers(0, 2, n).astype(np.uint32)
    ingress = (pol == 1).astype(np.uint8)
    remote = np.where(rng.random(n) < 0.5, SPACESHIP_ID, OTHER_ID).astype(np.uint32)
    remote = np.where(pol == 0, DEATHSTAR_ID, remote).astype(np.uint32)
    port = np.full(n, 80, np.uint16)
    port[rng.random(n) < 0.05] = 8080
    m = rng.integers(0, len(METHODS), n)
    pk = rng.integers(0, 4, n)
    hdr = rng.random(n) < 0.5
    hv = rng.integers(0, 3, n)
    for i in range(n):
        if pk[i] < 3:
            path = paths[pk[i]]
        else:
            L = int(rng.integers(1, 25))
            path = b"/v1/" + letters[rng.integers(0, len(letters), L)].tobytes()
        hs = [(b":method", METHODS[m[i]]), (b":path", path), (b":authority", b"deathstar.empire.svc")]
        if hdr[i]:
            hs.append((b"X-Has-Force", [b"true", b"True", b"false"][hv[i]]))
        reqs.append(hs)
    blob, off = _blob(reqs)
    return dict(policy=pol, ingress=ingress, port=port, remote=remote, hdr_blob=blob, hdr_off=off)


# -------------------------------------------------- config 5: 10K-rule HTTP
HTTP10K_METHODS = ["GET", "POST", "PUT", "DELETE", "GET|HEAD", "P(UT|OST)"]
WORDS = ["alpha", "bravo", "charlie", "delta", "echo", "foxtrot", "golf", "hotel", "india", "juliet", "kilo",
         "lima", "mike", "november", "oscar", "papa"]


def http10k_rules(n_rules: int = 10000, n_ports: int = 64, n_ids: int = 1000, n_selectors: int = 256,
                  seed: int = SEED):
    """Rules spread over ports and selectors (each selector = a set of
    identities).  Returns (npds policies, rule metadata used by the request
    generator)."""
    rng = np.random.default_rng(seed)
    ports = (8000 + np.arange(n_ports)).tolist()
    ids = (1000 + np.arange(n_ids)).tolist()
    sel_ids = [sorted(rng.choice(ids, size=int(rng.integers(4, 9)), replace=False).tolist())
               for _ in range(n_selectors)]
    meta = []
    by_scope: dict[tuple[int, int], list] = {}
    for k in range(n_rules):
        port = ports[int(rng.integers(0, n_ports))]
        sel = int(rng.integers(0, n_selectors))
        method = HTTP10K_METHODS[int(rng.integers(0, len(HTTP10K_METHODS)))]
        kind = int(rng.integers(0, 3))
        word = WORDS[int(rng.integers(0, len(WORDS)))]
        if kind == 0:
            path = f"/api/v[0-9]+/svc{k}/.*"
        elif kind == 1:
            path = f"/static/{k}/[a-z]+\\.(js|css)"
        else:
            path = f"/svc{k}/{word}"
        host = f"svc{k}\\.example\\.com" if rng.random() < 0.2 else ""
        headers = [f"X-Tenant-{k % 7}: t{k % 13}"] if rng.random() < 0.1 else []
        r = PortRuleHTTP(Method=method, Path=path, Host=host, Headers=headers)
        meta.append(dict(k=k, port=port, sel=sel, kind=kind, word=word, rule=r))
        by_scope.setdefault((port, sel), []).append(r)
    per_port: dict[int, list] = {}
    for (port, sel), rules in sorted(by_scope.items()):
        per_port.setdefault(port, []).append(
            port_network_policy_rule(sel_ids[sel], [get_http_rule(r)[0] for r in rules]))
    policies = [network_policy("ep-10k", 4242,
                               ingress=[port_network_policy(p, per_port[p]) for p in sorted(per_port)])]
    return policies, dict(meta=meta, sel_ids=sel_ids, ports=ports, ids=ids)


def _example(meta: dict, rng, hit: bool) -> list[tuple[bytes, bytes]]:
    k, kind, word = meta["k"], meta["kind"], meta["word"]
    method = meta["rule"].Method
    mchoices = {"GET": ["GET"], "POST": ["POST"], "PUT": ["PUT"], "DELETE": ["DELETE"], "GET|HEAD": ["GET", "HEAD"],
                "P(UT|OST)": ["PUT", "POST"]}[method]
    m = mchoices[int(rng.integers(0, len(mchoices)))]
    letters = "abcdefghijklmnopqrstuvwxyz"
    if kind == 0:
        tail = "".join(letters[int(x)] for x in rng.integers(0, 26, int(rng.integers(0, 40))))
        path = f"/api/v{int(rng.integers(1, 10))}/svc{k}/{tail}"
    elif kind == 1:
        stem = "".join(letters[int(x)] for x in rng.integers(0, 26, int(rng.integers(1, 24))))
        path = f"/static/{k}/{stem}.{'js' if rng.random() < 0.5 else 'css'}"
    else:
        path = f"/svc{k}/{word}"
    host = f"svc{k}.example.com" if meta["rule"].Host else f"h{int(rng.integers(0, 100))}.example.com"
    hs = [(b":method", m.encode()), (b":path", path.encode()), (b":authority", host.encode())]
    for h in meta["rule"].Headers:
        name, val = h.split(" ", 1)
        hs.append((name.rstrip(":").encode(), val.encode()))
    if not hit:
        # near miss: one field mutated
        which = int(rng.integers(0, 4))
        if which == 0:
            hs[0] = (b":method", b"PATCH")
        elif which == 1:
            p = bytearray(hs[1][1])
            pos = int(rng.integers(1, len(p)))
            p[pos] = ord("~")
            hs[1] = (b":path", bytes(p))
        elif which == 2:
            hs[1] = (b":path", hs[1][1] + b"/x")
        else:
            hs[2] = (b":authority", b"evil.example.com")
    return hs


def http10k_requests(n: int, info: dict, seed: int = SEED, distinct: int = 200_000):
    """n requests: 50% crafted to hit a random rule, 50% near-miss mutations.
    `distinct` unique header blocks are generated and tiled to n."""
    rng = np.random.default_rng(seed ^ 0x5EED)
    meta, sel_ids = info["meta"], info["sel_ids"]
    d = min(n, distinct)
    reqs = []
    port = np.zeros(d, np.uint16)
    remote = np.zeros(d, np.uint32)
    rix = rng.integers(0, len(meta), d)
    hit = rng.random(d) < 0.5
    for i in range(d):
        mt = meta[int(rix[i])]
        reqs.append(_example(mt, rng, bool(hit[i])))
        port[i] = mt["port"]
        ids = sel_ids[mt["sel"]]
        remote[i] = ids[int(rng.integers(0, len(ids)))]
    blob, off = _blob(reqs)
    rep = (n + d - 1) // d
    if rep > 1:
        lens = np.diff(off)
        blob = np.tile(blob, rep)
        off = np.concatenate([[0], np.cumsum(np.tile(lens, rep))]).astype(np.uint64)
        port = np.tile(port, rep)
        remote = np.tile(remote, rep)
    off = off[:n + 1]
    blob = blob[:int(off[-1])] if n else blob[:1]
    return dict(policy=np.zeros(n, np.uint32), ingress=np.ones(n, np.uint8), port=port[:n], remote=remote[:n],
                hdr_blob=blob, hdr_off=off)


# ------------------------------------------------------ config 2: L4 table
def l4_table(n_entries: int = 16384, n_ids: int = 16384, seed: int = SEED):
    """70% {id,port,proto,dir}, 20% {id,0,0,dir}, 10% {0,port,proto,dir}."""
    rng = np.random.default_rng(seed)
    from .classifier import POLICY_KEY_DTYPE
    ids = np.concatenate([np.arange(1, 6), 256 + np.arange(n_ids)]).astype(np.uint32)
    keys = set()
    out = []
    while len(out) < n_entries:
        r = rng.random()
        d = int(rng.integers(0, 2))
        if r < 0.7:
            k = (int(rng.choice(ids)), htons(int(rng.integers(1, 65536))), int(rng.choice([6, 17])), d)
        elif r < 0.9:
            k = (int(rng.choice(ids)), 0, 0, d)
        else:
            k = (0, htons(int(rng.integers(1, 65536))), int(rng.choice([6, 17])), d)
        if k in keys:
            continue
        keys.add(k)
        out.append(k)
    arr = np.zeros(len(out), POLICY_KEY_DTYPE)
    arr["sec_label"] = [k[0] for k in out]
    arr["dport"] = [k[1] for k in out]
    arr["protocol"] = [k[2] for k in out]
    arr["egress"] = [k[3] for k in out]
    ports = np.where(rng.random(len(out)) < 0.8, 0, rng.integers(10000, 11000, len(out))).astype(np.uint16)
    ports_be = ((ports & 0xFF) << 8 | ports >> 8).astype(np.uint16)
    return arr, ports_be


def l4_tuples(n: int, keys: np.ndarray, n_ids: int = 16384, seed: int = SEED):
    """identity uniform over the table's ids + 10 unknown, dport 50% from table
    ports (Zipf s=1.1) / 50% uniform, proto 50/50, dir 50/50, fragment 1%,
    len 64-1500."""
    rng = np.random.default_rng(seed ^ 0x7)
    from .classifier import L4_TUPLE_DTYPE
    t = np.zeros(n, L4_TUPLE_DTYPE)
    ids = np.concatenate([np.arange(1, 6), 256 + np.arange(n_ids), 900000 + np.arange(10)]).astype(np.uint32)
    t["identity"] = ids[rng.integers(0, len(ids), n)]
    tports = keys["dport"][keys["dport"] != 0]
    if len(tports) == 0:
        tports = np.array([htons(80)], np.uint16)
    z = np.minimum(rng.zipf(1.1, n) - 1, len(tports) - 1)
    uni = rng.integers(1, 65536, n).astype(np.uint16)
    uni_be = ((uni & 0xFF) << 8 | uni >> 8).astype(np.uint16)
    t["dport"] = np.where(rng.random(n) < 0.5, tports[z], uni_be)
    t["proto"] = np.where(rng.random(n) < 0.5, 6, 17)
    flags = (rng.random(n) < 0.5).astype(np.uint8)  # ingress
    flags |= ((rng.random(n) < 0.01).astype(np.uint8) << 1)  # fragment
    flags |= ((rng.random(n) < 0.01).astype(np.uint8) << 2)  # cb_policy
    t["flags"] = flags
    t["len"] = rng.integers(64, 1501, n)
    return t


# ---------------------------------------------------- config 3: prefilter
def lpm_prefixes(n_v4: int = 700_000, n_v6: int = 300_000, seed: int = SEED):
    """Prefix-length mix of SURVEY §8(d) config 3; returns cg_cidr records."""
    from .classifier import CIDR_DTYPE
    rng = np.random.default_rng(seed)
    out = np.zeros(n_v4 + n_v6, CIDR_DTYPE)
    r = rng.random(n_v4)
    plen4 = np.where(r < 0.55, 24, np.where(r < 0.85, rng.integers(16, 24, n_v4),
                                            np.where(r < 0.90, rng.integers(8, 16, n_v4), 32)))
    a4 = rng.integers(0, 2 ** 32, n_v4, dtype=np.uint64).astype(np.uint32)
    mask = np.where(plen4 == 0, 0, (0xFFFFFFFF << (32 - plen4)) & 0xFFFFFFFF).astype(np.uint32)
    a4 &= mask
    out["family"][:n_v4] = 4
    out["prefixlen"][:n_v4] = plen4
    out["addr"][:n_v4, :4] = a4.astype(">u4").view(np.uint8).reshape(-1, 4)
    r = rng.random(n_v6)
    plen6 = np.where(r < 0.40, rng.integers(32, 49, n_v6), np.where(r < 0.85, rng.integers(49, 65, n_v6),
                                                                   np.where(r < 0.90, rng.integers(65, 128, n_v6),
                                                                            128)))
    a6 = rng.integers(0, 256, (n_v6, 16), dtype=np.uint8)
    for i in range(16):  # mask host bits
        keep = np.clip(plen6 - 8 * i, 0, 8)
        a6[:, i] &= ((0xFF << (8 - keep)) & 0xFF).astype(np.uint8)
    out["family"][n_v4:] = 6
    out["prefixlen"][n_v4:] = plen6
    out["addr"][n_v4:] = a6
    return out


def lpm_addresses(n: int, prefixes: np.ndarray, n_eps: int = 65536, seed: int = SEED):
    """70% v4 / 30% v6; 50% drawn inside a random prefix; destinations are
    local endpoints 50% of the time.  Returns (v4 (n4,2) u32, v6 (n6,32) u8,
    ep4 u32, ep6 (m,16) u8)."""
    rng = np.random.default_rng(seed ^ 0x3)
    p4 = prefixes[prefixes["family"] == 4]
    p6 = prefixes[prefixes["family"] == 6]
    n4 = int(n * 0.7)
    n6 = n - n4
    ep4 = rng.integers(0, 2 ** 32, n_eps // 2, dtype=np.uint64).astype(np.uint32)
    ep6 = rng.integers(0, 256, (n_eps // 2, 16), dtype=np.uint8)
    # v4
    s4 = rng.integers(0, 2 ** 32, n4, dtype=np.uint64).astype(np.uint32)
    inside = rng.random(n4) < 0.5
    pick = p4[rng.integers(0, len(p4), n4)]
    base = pick["addr"][:, :4].copy().view(">u4").reshape(-1).astype(np.uint32)
    host_bits = (32 - pick["prefixlen"].astype(np.int64))
    hm = np.where(host_bits >= 32, 0xFFFFFFFF, (1 << host_bits) - 1).astype(np.uint32)
    s4 = np.where(inside, base | (s4 & hm), s4).astype(np.uint32)
    d4 = np.where(rng.random(n4) < 0.5, ep4[rng.integers(0, len(ep4), n4)],
                  rng.integers(0, 2 ** 32, n4, dtype=np.uint64).astype(np.uint32)).astype(np.uint32)
    v4 = np.empty((n4, 2), np.uint32)
    v4[:, 0] = s4.astype(">u4").view("<u4")  # network order as in iphdr
    v4[:, 1] = d4.astype(">u4").view("<u4")
    ep4_be = ep4.astype(">u4").view("<u4")
    # v6
    s6 = rng.integers(0, 256, (n6, 16), dtype=np.uint8)
    inside = rng.random(n6) < 0.5
    pick = p6[rng.integers(0, len(p6), n6)]
    for i in range(16):
        keep = np.clip(pick["prefixlen"].astype(np.int64) - 8 * i, 0, 8)
        m = ((0xFF << (8 - keep)) & 0xFF).astype(np.uint8)
        s6[:, i] = np.where(inside, (pick["addr"][:, i] & m) | (s6[:, i] & ~m), s6[:, i])
    d6 = np.where((rng.random(n6) < 0.5)[:, None], ep6[rng.integers(0, len(ep6), n6)],
                  rng.integers(0, 256, (n6, 16), dtype=np.uint8))
    v6 = np.concatenate([s6, d6], axis=1).astype(np.uint8)
    return v4, v6, ep4_be, ep6


# ------------------------------------------- ipcache
def ipcache_entries(n: int = 512_000, n_nodes: int = 4096, seed: int = SEED):
    """IP → identity entries shaped like a cluster's ipcache (MaxEntries
    512000, pkg/maps/ipcache/ipcache.go:36): 70% IPv4 / 30% IPv6.  80% of
    the v4 (70% of the v6) entries are pod /32 (/128) addresses inside one
    of `n_nodes` per-node pod CIDRs (/24, /64) with the node's tunnel
    endpoint; the rest are CIDR-policy prefixes (/8–/28, /32–/120) with
    tunnel 0.  1% of the entries carry identity 0 (resolved to WORLD_ID).
    Returns (cg_cidr records, (n, 2) u32 {sec_label, tunnel_endpoint}),
    duplicate keys removed."""
    from .classifier import CIDR_DTYPE
    rng = np.random.default_rng(seed ^ 0x1CAC)
    n4 = int(n * 0.7)
    n6 = n - n4
    keys = np.zeros(n4 + n6, CIDR_DTYPE)
    vals = np.zeros((n4 + n6, 2), np.uint32)
    node_tun = (np.uint32(0x0AFF0000) + np.arange(n_nodes, dtype=np.uint32)).astype(">u4").view("<u4")
    # v4
    pod = rng.random(n4) < 0.8
    node = rng.integers(0, n_nodes, n4)
    node24 = (0x0A000000 | (rng.permutation(1 << 16)[:n_nodes].astype(np.uint32) << 8)).astype(np.uint32)
    a_pod = node24[node] | rng.integers(1, 255, n4).astype(np.uint32)
    plen_c = rng.integers(16, 29, n4)
    a_c = rng.integers(0, 2 ** 32, n4, dtype=np.uint64).astype(np.uint32)
    a_c &= ((0xFFFFFFFF << (32 - plen_c)) & 0xFFFFFFFF).astype(np.uint32)
    keys["family"][:n4] = 4
    keys["prefixlen"][:n4] = np.where(pod, 32, plen_c)
    keys["addr"][:n4, :4] = np.where(pod, a_pod, a_c).astype(">u4").view(np.uint8).reshape(-1, 4)
    vals[:n4, 1] = np.where(pod, node_tun[node], 0)
    # v6
    pod = rng.random(n6) < 0.7
    node = rng.integers(0, n_nodes, n6)
    node64 = rng.integers(0, 256, (n_nodes, 8), dtype=np.uint8)
    node64[:, 0] = 0xFD
    a6 = rng.integers(0, 256, (n6, 16), dtype=np.uint8)
    plen6 = np.where(pod, 128, rng.integers(32, 121, n6))
    a6[:, :8] = np.where(pod[:, None], node64[node], a6[:, :8])
    for i in range(16):
        keep = np.clip(plen6 - 8 * i, 0, 8)
        a6[:, i] &= ((0xFF << (8 - keep)) & 0xFF).astype(np.uint8)
    keys["family"][n4:] = 6
    keys["prefixlen"][n4:] = plen6
    keys["addr"][n4:] = a6
    vals[n4:, 1] = np.where(pod, node_tun[node], 0)
    vals[:, 0] = rng.integers(256, 256 + 65536, n4 + n6).astype(np.uint32)
    vals[rng.random(n4 + n6) < 0.01, 0] = 0
    _, first = np.unique(keys.view(np.uint8).reshape(len(keys), -1), axis=0, return_index=True)
    first.sort()
    return keys[first], vals[first]


def ipcache_addresses(n: int, keys: np.ndarray, seed: int = SEED):
    """70% v4 / 30% v6 destination addresses; half drawn inside a random
    entry (random host bits), half uniform.  Returns (v4 u32 network order,
    v6 (n6, 16) u8)."""
    rng = np.random.default_rng(seed ^ 0x1CAD)
    k4 = keys[keys["family"] == 4]
    k6 = keys[keys["family"] == 6]
    n4 = int(n * 0.7)
    n6 = n - n4
    a4 = rng.integers(0, 2 ** 32, n4, dtype=np.uint64).astype(np.uint32)
    if len(k4):
        inside = rng.random(n4) < 0.5
        pick = k4[rng.integers(0, len(k4), n4)]
        base = pick["addr"][:, :4].copy().view(">u4").reshape(-1).astype(np.uint32)
        host = 32 - pick["prefixlen"].astype(np.int64)
        hm = np.where(host >= 32, 0xFFFFFFFF, (1 << host) - 1).astype(np.uint32)
        a4 = np.where(inside, base | (a4 & hm), a4).astype(np.uint32)
    a6 = rng.integers(0, 256, (n6, 16), dtype=np.uint8)
    if len(k6):
        inside = rng.random(n6) < 0.5
        pick = k6[rng.integers(0, len(k6), n6)]
        for i in range(16):
            keep = np.clip(pick["prefixlen"].astype(np.int64) - 8 * i, 0, 8)
            m = ((0xFF << (8 - keep)) & 0xFF).astype(np.uint8)
            a6[:, i] = np.where(inside, (pick["addr"][:, i] & m) | (a6[:, i] & ~m), a6[:, i])
    return a4.astype(">u4").view("<u4").copy(), a6


# -------------------------------------------------------- config 4: Kafka
def kafka_policy(n_rules: int = 1000, n_topics: int = 1000, n_clients: int = 100, n_ids: int = 64,
                 seed: int = SEED):
    """Rules mixing {apiKey}, {role}, {apiKey,topic}, {role,topic},
    {apiVersion}, {clientID} (examples/policies/l7/kafka/*.yaml patterns)."""
    rng = np.random.default_rng(seed)
    topics = [f"topic-{i}" for i in range(n_topics)]
    clients = [f"client-{i}" for i in range(n_clients)]
    keys = list(__import__("cilium_amd.policy", fromlist=["KAFKA_API_KEY_MAP"]).KAFKA_API_KEY_MAP)
    sels = []
    ids = (2000 + np.arange(n_ids)).tolist()
    n_sel = 16
    for s in range(n_sel + 1):
        rules = []
        for _ in range(n_rules // (n_sel + 1)):
            kind = int(rng.integers(0, 6))
            r = PortRuleKafka()
            if kind == 0:
                r.APIKey = keys[int(rng.integers(0, len(keys)))]
            elif kind == 1:
                r.Role = ["produce", "consume"][int(rng.integers(0, 2))]
            elif kind == 2:
                r.APIKey = ["produce", "fetch", "metadata"][int(rng.integers(0, 3))]
                r.Topic = topics[int(rng.integers(0, n_topics))]
            elif kind == 3:
                r.Role = ["produce", "consume"][int(rng.integers(0, 2))]
                r.Topic = topics[int(rng.integers(0, n_topics))]
            elif kind == 4:
                r.APIKey = keys[int(rng.integers(0, len(keys)))]
                r.APIVersion = str(int(rng.integers(0, 6)))
            else:
                r.ClientID = clients[int(rng.integers(0, n_clients))]
                r.APIKey = ["produce", "fetch"][int(rng.integers(0, 2))]
            rules.append(r)
        if s == n_sel:
            sels.append({"identities": None, "rules": rules[: max(1, len(rules) // 8)]})
        else:
            sels.append({"identities": sorted(rng.choice(ids, 8, replace=False).tolist()), "rules": rules})
    return [{"name": "kafka-redirect-9092", "selectors": sels}], dict(topics=topics, clients=clients, ids=ids)


def kafka_requests(n: int, info: dict, seed: int = SEED):
    """apiKey weighted (produce 35%, fetch 35%, metadata 15%, other 15% over the
    34 keys), version 0-5, 1-4 topics, clientID from 100."""
    rng = np.random.default_rng(seed ^ 0x9)
    topics, clients, ids = info["topics"], info["clients"], info["ids"]
    r = rng.random(n)
    key = np.where(r < 0.35, 0, np.where(r < 0.70, 1, np.where(r < 0.85, 3, rng.integers(0, 38, n)))).astype(np.int16)
    ver = rng.integers(0, 6, n).astype(np.int16)
    typed = np.isin(key, [0, 1, 2, 3, 8, 9])
    kind = np.where(typed, 1, np.where(key == 10, 2, 0)).astype(np.uint8)
    remote = np.where(rng.random(n) < 0.9, np.asarray(ids)[rng.integers(0, len(ids), n)],
                      rng.integers(0, 10, n)).astype(np.uint32)
    nt = np.where(typed, rng.integers(1, 5, n), 0)
    cl = rng.integers(0, len(clients), n)
    client = [clients[int(c)].encode() for c in cl]
    tix = rng.integers(0, len(topics) + 20, (n, 4))
    tps = []
    for i in range(n):
        ts = []
        for j in range(int(nt[i])):
            t = int(tix[i, j])
            ts.append(topics[t].encode() if t < len(topics) else f"unknown-{t}".encode())
        tps.append(ts)
    return dict(redirect=np.zeros(n, np.uint32), remote=remote, api_key=key, api_version=ver, kind=kind,
                client_id=client, topics=tps)


# ------------------------------------------- config 5, vectorized generator
def _assemble(parts: list, n: int) -> tuple[np.ndarray, np.ndarray, list]:
    """Concatenate per-row byte segments: parts = [(data [n, W] uint8, lens
    [n])]; returns (blob, offsets, start offset of each part per row)."""
    total = np.zeros(n, np.int64)
    for _, ln in parts:
        total += ln
    off = np.zeros(n + 1, np.int64)
    np.cumsum(total, out=off[1:])
    out = np.empty(int(off[-1]), np.uint8)
    pos = off[:-1].copy()
    starts = []
    for data, ln in parts:
        starts.append(pos.copy())
        w = data.shape[1]
        if w:
            mask = np.arange(w)[None, :] < ln[:, None]
            out[(pos[:, None] + np.arange(w)[None, :])[mask]] = data[mask]
        pos += ln
    return out, off.astype(np.uint64), starts


def _table(strs: list) -> tuple[np.ndarray, np.ndarray]:
    enc = [s.encode() if isinstance(s, str) else s for s in strs]
    w = max((len(s) for s in enc), default=0)
    t = np.zeros((len(enc), max(w, 1)), np.uint8)
    for i, s in enumerate(enc):
        t[i, :len(s)] = np.frombuffer(s, np.uint8)
    return t, np.array([len(s) for s in enc], np.int64)


def _const(s: bytes, n: int):
    return np.broadcast_to(np.frombuffer(s, np.uint8), (n, len(s))), np.full(n, len(s), np.int64)


def _pick(table, idx):
    t, ln = table
    return t[idx], ln[idx]


def http10k_requests_fast(n: int, info: dict, seed: int = SEED, raw: bool = False, chunk: int = 1 << 20):
    """n distinct config-5 requests drawn as http10k_requests draws them (50%
    crafted to hit a random rule, 50% near misses with one field mutated),
    built with vectorized numpy instead of a per-request loop.  Returns the
    header-list form (hdr_blob / hdr_off, as cg_http_pack takes it) or, with
    raw=True, raw HTTP/1.1 heads (raw_blob / raw_off: request line, Host,
    the rule's header, blank line)."""
    meta, sel_ids = info["meta"], info["sel_ids"]
    K = len(meta)
    kind = np.array([m["kind"] for m in meta], np.int64)
    port_of = np.array([m["port"] for m in meta], np.uint16)
    sel_of = np.array([m["sel"] for m in meta], np.int64)
    has_host = np.array([bool(m["rule"].Host) for m in meta])
    mopts = {"GET": ["GET"], "POST": ["POST"], "PUT": ["PUT"], "DELETE": ["DELETE"], "GET|HEAD": ["GET", "HEAD"],
             "P(UT|OST)": ["PUT", "POST"]}
    mnames = ["GET", "POST", "PUT", "DELETE", "HEAD", "PATCH"]
    m_a = np.array([mnames.index(mopts[m["rule"].Method][0]) for m in meta], np.int64)
    m_b = np.array([mnames.index(mopts[m["rule"].Method][-1]) for m in meta], np.int64)
    methods = _table(mnames)
    ks = _table([str(m["k"]) for m in meta])
    words = _table([m["word"] for m in meta])
    hdr_names = _table([m["rule"].Headers[0].split(" ", 1)[0].rstrip(":") if m["rule"].Headers else "" for m in meta])
    hdr_vals = _table([m["rule"].Headers[0].split(" ", 1)[1] if m["rule"].Headers else "" for m in meta])
    has_hdr = np.array([bool(m["rule"].Headers) for m in meta])
    hosts_rule = _table([f"svc{m['k']}.example.com" for m in meta])
    hosts_rand = _table([f"h{i}.example.com" for i in range(100)])
    evil = b"evil.example.com"
    sel_tab = np.zeros((len(sel_ids), max(len(s) for s in sel_ids)), np.uint32)
    sel_len = np.array([len(s) for s in sel_ids], np.int64)
    for i, s in enumerate(sel_ids):
        sel_tab[i, :len(s)] = s
    def one_chunk(c0: int):
        rng = np.random.default_rng([seed ^ 0xFA57, c0])
        c = min(chunk, n - c0)
        rix = rng.integers(0, K, c)
        hit = rng.random(c) < 0.5
        which = np.where(hit, -1, rng.integers(0, 4, c))
        kd = kind[rix]
        midx = np.where(rng.random(c) < 0.5, m_a[rix], m_b[rix])
        midx = np.where(which == 0, mnames.index("PATCH"), midx)
        letters = rng.integers(97, 123, (c, 40)).astype(np.uint8)
        tail_len = np.where(kd == 0, rng.integers(0, 40, c), np.where(kd == 1, rng.integers(1, 24, c), 0))
        digit = (rng.integers(1, 10, c) + 48).astype(np.uint8).reshape(c, 1)
        js = rng.random(c) < 0.5
        z = np.zeros(c, np.int64)
        one = np.ones(c, np.int64)
        # path = pre1 [digit] pre2 k "/" [tail | word] [ext] [mutation "/x"]
        pre1 = np.where(kd == 0, 6, np.where(kd == 1, 8, 4))  # "/api/v" | "/static/" | "/svc"
        pre1_tab = _table(["/api/v", "/static/", "/svc"])
        kd_i = np.where(kd == 0, 0, np.where(kd == 1, 1, 2))
        p1, _ = _pick(pre1_tab, kd_i)
        p2 = _const(b"/svc", c)
        ext_tab = _table(["", ".js", ".css"])
        ext_i = np.where(kd == 1, np.where(js, 1, 2), 0)
        kt, kl = _pick(ks, rix)
        wt, wl = _pick(words, rix)
        path_parts = [(p1, pre1), (digit, np.where(kd == 0, 1, 0)), (p2[0], np.where(kd == 0, 4, 0)),
                      (kt, kl), (_const(b"/", c)[0], one),
                      (letters, tail_len), (wt, np.where(kd == 2, wl, 0)), _pick(ext_tab, ext_i),
                      (_const(b"/x", c)[0], np.where(which == 2, 2, 0))]
        hr_t, hr_l = _pick(hosts_rule, rix)
        hx_t, hx_l = _pick(hosts_rand, rng.integers(0, 100, c))
        w = max(hr_t.shape[1], hx_t.shape[1], len(evil))
        ht = np.zeros((c, w), np.uint8)
        hl = np.where(has_host[rix], hr_l, hx_l)
        ht[:, :hr_t.shape[1]] = np.where(has_host[rix][:, None], hr_t, 0)
        ht[:, :hx_t.shape[1]] |= np.where(has_host[rix][:, None], 0, hx_t).astype(np.uint8)
        ev = which == 3
        ht[ev] = 0
        ht[ev, :len(evil)] = np.frombuffer(evil, np.uint8)
        hl = np.where(ev, len(evil), hl)
        mt, ml = _pick(methods, midx)
        hn_t, hn_l = _pick(hdr_names, rix)
        hv_t, hv_l = _pick(hdr_vals, rix)
        hh = has_hdr[rix]
        if raw:
            parts = [(mt, ml), _const(b" ", c)] + path_parts + [_const(b" HTTP/1.1\r\nHost: ", c), (ht, hl),
                                                                 _const(b"\r\n", c),
                                                                 (hn_t, np.where(hh, hn_l, 0)),
                                                                 (_const(b": ", c)[0], np.where(hh, 2, 0)),
                                                                 (hv_t, np.where(hh, hv_l, 0)),
                                                                 (_const(b"\r\n", c)[0], np.where(hh, 2, 0)),
                                                                 _const(b"\r\n", c)]
            path_first = 2
        else:
            parts = [_const(b":method\0", c), (mt, ml), _const(b"\0:path\0", c)] + path_parts + \
                    [_const(b"\0:authority\0", c), (ht, hl), _const(b"\0", c),
                     (hn_t, np.where(hh, hn_l, 0)), (_const(b"\0", c)[0], np.where(hh, 1, 0)),
                     (hv_t, np.where(hh, hv_l, 0)), (_const(b"\0", c)[0], np.where(hh, 1, 0))]
            path_first = 3
        blob, off, starts = _assemble(parts, c)
        # near miss 1: one path byte (after the first) becomes '~'
        plen = sum(ln for _, ln in path_parts)
        m1 = which == 1
        if m1.any():
            at = starts[path_first][m1] + 1 + (rng.random(int(m1.sum())) * (plen[m1] - 1)).astype(np.int64)
            blob[at] = ord("~")
        s = sel_of[rix]
        rem = sel_tab[s, (rng.random(c) * sel_len[s]).astype(np.int64)]
        return blob, off, port_of[rix], rem

    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
        res = list(ex.map(one_chunk, range(0, n, chunk)))
    blobs, offs, base, ports, remotes = [], [], 0, [], []
    for blob, off, pt, rem in res:
        blobs.append(blob)
        offs.append(off[:-1] + np.uint64(base))
        base += int(off[-1])
        ports.append(pt)
        remotes.append(rem)
    off = np.concatenate(offs + [np.array([base], np.uint64)]).astype(np.uint64)
    blob = np.concatenate(blobs) if blobs else np.zeros(1, np.uint8)
    key = ("raw_blob", "raw_off") if raw else ("hdr_blob", "hdr_off")
    return {"policy": np.zeros(n, np.uint32), "ingress": np.ones(n, np.uint8),
            "port": np.concatenate(ports) if ports else np.zeros(0, np.uint16),
            "remote": np.concatenate(remotes).astype(np.uint32) if remotes else np.zeros(0, np.uint32),
            key[0]: blob, key[1]: off}
