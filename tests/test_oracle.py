"""Pin the CPU oracle against the reference's own known answers (tests/golden) and PCRE."""

import numpy as np
import pytest

from gpumatch import blob, confgen, records, workloads
from helpers import golden, kat_request, upstream_table, vs_blob
from oracle_py import Oracle, murmur2, pcre_match

ADV = golden("advanced_routing.json")


@pytest.mark.parametrize("case", ADV["cases"], ids=lambda c: f"{c['vs']}-{c['expect_upstream']}")
def test_e2e_advanced_routing_kats(case):
    """tests/suite/test_virtual_server_advanced_routing.py:10-93."""
    vs = ADV["virtual_servers"][case["vs"]]
    b = vs_blob([vs])
    o = Oracle(b)
    reqs, arena = records.from_dicts([kat_request(ADV["host"], ADV["uri"], case["request"])])
    v, _ = o.match(reqs, arena)
    assert v[0]["action"] == 0, v[0]
    ups = upstream_table(b)
    name = f"vs_default_{vs['metadata']['name']}_{case['expect_upstream']}"
    assert ups[v[0]["upstream_id"]] == name


def _value_vs(value):
    return {"metadata": {"name": "mv", "namespace": "default"},
            "spec": {"host": "mv.example.com",
                     "upstreams": [{"name": "m", "service": "m", "port": 80}, {"name": "d", "service": "d", "port": 80}],
                     "routes": [{"path": "/", "rules": {"conditions": [{"header": "x-v"}],
                                                        "matches": [{"values": [value], "upstream": "m"}],
                                                        "defaultUpstream": "d"}}]}}


@pytest.mark.parametrize("case", golden("match_values.json")["cases"], ids=lambda c: f"{c['value']}|{c['subject']}")
def test_docs_match_value_semantics(case):
    """docs/virtualserver-and-virtualserverroute.md:264-271."""
    b = vs_blob([_value_vs(case["value"])])
    o = Oracle(b)
    reqs, arena = records.from_dicts([{"host": "mv.example.com", "uri": "/x", "headers": [("X-V", case["subject"])]}])
    v, _ = o.match(reqs, arena)
    ups = upstream_table(b)
    assert ups[v[0]["upstream_id"]] == ("vs_default_mv_m" if case["match"] else "vs_default_mv_d")
    assert v[0]["match_idx"] == (0 if case["match"] else 0xFF)


def _py_murmur2(data: bytes) -> int:
    m = 0x5BD1E995
    h = len(data) & 0xFFFFFFFF
    i = 0
    while len(data) - i >= 4:
        k = int.from_bytes(data[i:i + 4], "little")
        k = (k * m) & 0xFFFFFFFF; k ^= k >> 24; k = (k * m) & 0xFFFFFFFF
        h = (h * m) & 0xFFFFFFFF; h ^= k
        i += 4
    rem = len(data) - i
    if rem == 3: h ^= data[i + 2] << 16
    if rem >= 2: h ^= data[i + 1] << 8
    if rem >= 1: h ^= data[i]; h = (h * m) & 0xFFFFFFFF
    h ^= h >> 13; h = (h * m) & 0xFFFFFFFF; h ^= h >> 15
    return h


def test_murmur2_restatements_agree():
    rng = np.random.default_rng(1)
    assert murmur2(b"") == 0 == _py_murmur2(b"")
    for L in list(range(0, 40)) + [64, 100]:
        d = bytes(rng.integers(0, 256, L, dtype=np.uint8))
        assert murmur2(d) == _py_murmur2(d)


def test_split_clients_ratio_and_bounds():
    """tests/suite/test_virtual_server_split_traffic.py:46-66 (90/10, +-0.2) and the
    split_clients bound arithmetic (percent * 0xffffffff / 10000, first part with h < bound)."""
    sp = golden("split_traffic.json")
    vs = sp["virtual_server"]
    b = vs_blob([vs])
    o = Oracle(b)
    n = 20000
    rng = np.random.default_rng(7)
    rids = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    path = vs["spec"]["routes"][0]["path"]
    items = [{"host": vs["spec"]["host"], "uri": path, "rid": bytes(r)} for r in rids]
    reqs, arena = records.from_dicts(items)
    v, _ = o.match(reqs, arena)
    weights = [s["weight"] for s in vs["spec"]["routes"][0]["splits"]]
    frac = (v["split_bucket"] == 0).mean()
    assert abs(frac - weights[0] / 100) <= sp["tolerance"]
    bounds, last = [], 0
    for w in weights:
        last += w * 100 * 0xFFFFFFFF // 10000
        bounds.append(last & 0xFFFFFFFF)
    for i in range(200):
        h = _py_murmur2(bytes(rids[i]).hex().encode())
        exp = next((k for k, bd in enumerate(bounds) if h < bd), 0xFF)
        assert v[i]["split_bucket"] == exp


def test_cafe_server_selection_and_redirects():
    b = workloads.c1_blob()
    o = Oracle(b)
    items = [
        {"host": "cafe.example.com", "uri": "/tea", "https": True},         # proxied
        {"host": "cafe.example.com", "uri": "/tea"},                       # ssl-redirect 301
        {"host": "CAFE.Example.COM:443", "uri": "/coffee/x", "https": True},  # case + port stripped
        {"host": "cafe.example.com.", "uri": "/coffee", "https": True},      # trailing dot stripped
        {"host": "cafe.example.com", "uri": "/", "https": True},             # no location -> 404
        {"host": "other.example.com", "uri": "/tea", "https": True},         # default server -> 404
        {"host": "a..b", "uri": "/tea", "https": True},                      # invalid host -> 400
        {"host": None, "uri": "/tea"},                                       # absent host -> default
    ]
    reqs, arena = records.from_dicts(items)
    v, _ = o.match(reqs, arena)
    assert list(v["action"]) == [0, 1, 0, 0, 4, 2, 5, 2]
    assert list(v["status"]) == [0, 301, 0, 0, 404, 404, 400, 404]
    assert v[0]["server_id"] == v[2]["server_id"] == v[3]["server_id"] != v[5]["server_id"]


def test_location_lookup_semantics():
    """Appendix A.3: exact, longest prefix, ^~, regex order, auto_redirect (examples/rewrites
    README: /tea is redirected to /tea/)."""
    conf = """
    http {
      upstream u1 { server 1.1.1.1; }
      upstream u2 { server 1.1.1.2; }
      server {
        listen 80 default_server;
        server_name t.example.com;
        location = /exact { proxy_pass http://u1; }
        location /tea/ { proxy_pass http://u1; }
        location /img/ { return 403; }
        location ^~ /static { proxy_pass http://u2; }
        location ~ \\.php$ { proxy_pass http://u2; }
        location ~* \\.JPG$ { proxy_pass http://u1; }
        location / { proxy_pass http://u1; }
      }
    }"""
    b = blob.make_blob(conf, {})
    o = Oracle(b)
    cases = [("/exact", 0, 0), ("/exact/", 6, 0), ("/tea", 1, 3), ("/tea/x", 1, 0), ("/img", 2, 4 - 4),
             ("/static/a.php", 3, 0), ("/a.php", 4, 0), ("/b.jpg", 5, 0), ("/b.jpgx", 6, 0), ("/img/x", 2, 2)]
    items = [{"host": "t.example.com", "uri": u} for u, _, _ in cases]
    reqs, arena = records.from_dicts(items)
    v, _ = o.match(reqs, arena)
    for (u, loc, act), x in zip(cases, v):
        if u == "/img":
            assert x["action"] == 0 and x["location_id"] == 6, u   # no auto_redirect without proxy_pass
            continue
        assert x["location_id"] == loc, (u, x)
        assert x["action"] == act, (u, x)


@pytest.mark.parametrize("pat,subj,exp", [
    (r"^a\s$", b"a\x0b", 1),            # PCRE 8.39: \s includes VT
    (r"a$", b"a\n", 1),                 # $ before a final newline
    (r"a$", b"a\n\n", 0),
    (r"a.b", b"a\nb", 0),               # . excludes \n
    (r"[^x]", b"\n", 1),
    (r"^$", b"", 1),
])
def test_pcre_semantics_pinned(pat, subj, exp):
    assert pcre_match(pat, subj) == exp
