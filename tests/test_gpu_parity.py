"""Parity of the gfx950 path (libgpumatch.so kernels) with the CPU oracle: bit-exact verdicts and
hit-id lists on the same seeded inputs, plus the reference's known answers run on the GPU."""

import numpy as np
import pytest

from gpumatch import blob, engine, records, sigs, workloads
from helpers import assert_verdicts_equal, golden, kat_request, upstream_table, vs_blob
from oracle_py import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    return engine.Engine(0)


def run_both(eng, b, reqs, arena, gen=5, hit_cap=None):
    eng.load(b, gen)
    got, gh = eng.match_host(reqs, arena, hit_cap)
    exp, eh = Oracle(b, gen).match(reqs, arena)
    return got, gh, exp, eh


def test_c1_cafe_parity(eng):
    reqs, arena = records.gen_c1(300_000)
    got, gh, exp, eh = run_both(eng, workloads.c1_blob(), reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "C1")
    assert len(set(exp["action"].tolist())) >= 4   # the sample exercises several verdict kinds


def test_c2_advanced_routing_parity(eng):
    reqs, arena = records.gen_c2(100_000)
    got, gh, exp, eh = run_both(eng, workloads.c2_blob(), reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "C2")
    assert (exp["route_kind"] == 2).any() and (exp["route_kind"] == 3).any()
    assert (exp["match_idx"] != 0xFF).any() and (exp["split_bucket"] == 1).any()


def test_c5_mergeable_parity(eng):
    reqs, arena = workloads.gen_c5(200_000)
    got, gh, exp, eh = run_both(eng, workloads.c5_blob(), reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "C5")


@pytest.mark.parametrize("mode", ["block", "monitoring", "off"])
def test_c4_waf_parity_small_set(eng, mode):
    ss = workloads.c4_sigset(800, 200)
    reqs, arena = records.gen_c4(20_000, ss, plant_rate=0.05)
    got, gh, exp, eh = run_both(eng, workloads.c4_blob(ss, mode), reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, f"C4-{mode}")
    if mode != "off":
        assert len(eh) > 500
    else:
        assert len(eh) == 0


@pytest.mark.parametrize("sample", [False, True])
def test_c4_waf_parity_10k_rules(eng, sample):
    """The bench's rule set, with and without a traffic sample in the generation (the sample
    only steers the prefilter's key choice; verdicts must not depend on it)."""
    ss = workloads.c4_sigset()
    reqs, arena = records.gen_c4(6_000, ss, plant_rate=0.05)
    smp = workloads.c4_sample(ss, 500) if sample else None
    got, gh, exp, eh = run_both(eng, workloads.c4_blob(ss, sample=smp), reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "C4-10k")
    assert (exp["action"] == 6).sum() > 100


def test_c4_stress_variant_parity(eng):
    """The C4 stress variant (workloads.c4_stress_generation): vocabulary literals that benign
    traffic speaks, 10% factorless (always-run) regexes, SQL / HTML text -- 6000 requests
    against the oracle."""
    ss, b = workloads.c4_stress_generation()
    reqs, arena = records.gen_c4(6_000, ss, seed=workloads.C4_STRESS_POOL_SEED, plant_rate=0.05, stress=True)
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "C4-stress")
    assert (exp["n_hits"] > 0).mean() > 0.2
    st = eng.stats()
    assert st["n_sig_regex_always"] == 200 and st["last_candidates"] > 10 * len(reqs)


def always_rules(n=150, seed=11):
    """Factorless (always-run) regexes of mixed shapes: short literals, counted classes, anchors
    (^, $ with nginx's "before a final newline"), alternations, an empty-matching pattern and
    case-insensitive ones, over every zone set -- enough of them for several union-DFA groups and
    LDS slices (gm_compile.cpp, k_waf_always_multi)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    L = "abcdefghij"
    out = [sigs.Rule("re", False, "uahb", r"z*"), sigs.Rule("re", False, "b", r"^$"),
           sigs.Rule("re", True, "ah", r"^q[0-9]"), sigs.Rule("re", False, "b", r"[a-c]{2}$")]
    for i in range(n - len(out)):
        t = int(rng.integers(0, 8))
        a, b2 = (L[int(x)] for x in rng.integers(0, len(L), 2))
        k = int(rng.integers(1, 5))
        pat = [f"{a}{b2}[0-9]{{{k}}}", f"[0-9]{{{k},}}{a}x", f"({a}{b2}|{b2}{a})-{k}", f"{a}[^{b2}]{{{k}}}{a}",
               f"^{a}{b2}", f"{a}{k}$", f"={a}\\s*{b2}", f"<{a}[a-z]{{0,{k}}}>"][t]
        out.append(sigs.Rule("re", bool(rng.random() < 0.4), ["uahb", "ua", "b", "h", "u"][int(rng.integers(0, 5))], pat))
    return out


def always_items(n, seed=12):
    rng = np.random.Generator(np.random.PCG64(seed))
    L = b"abcdefghij0123456789-=<> xzqABCJ\n"
    items = []
    for i in range(n):
        def txt(lo, hi):
            return bytes(L[int(x)] for x in rng.integers(0, len(L), int(rng.integers(lo, hi))))
        body = txt(0, 300) if rng.random() < 0.8 else b""
        if rng.random() < 0.2:
            body += b"\n"
        args = txt(0, 40).replace(b"\n", b"").decode() if rng.random() < 0.7 else ""
        items.append({"host": "cafe.example.com", "uri": "/tea/" + txt(0, 20).replace(b"\n", b"").decode(),
                      "args": args, "https": True, "body": body,
                      "headers": [("X-T", txt(0, 30).replace(b"\n", b"").decode())]})
    return items


def test_always_union_groups(eng):
    """Always-run regexes answered by union DFAs in LDS slices: every (request, rule) hit equal to
    the oracle's PCRE answers (empty zones, a final newline, anchors, zone sets)."""
    b = workloads.c4_blob(sigs.SigSet(always_rules()))
    reqs, arena = records.from_dicts(always_items(20_000))
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "always")
    st = eng.stats()
    assert st["n_alw_groups"] >= 4 and st["n_alw_slices"] >= 2 and st["n_alw_single"] == 0
    assert len(eh) > 20_000   # dense hits: the empty-matching pattern alone hits every request


def test_waf_edge_cases(eng):
    rules = [sigs.Rule("lit", True, "uahb", b"evil"), sigs.Rule("lit", False, "b", b"CaseSensitive"),
             sigs.Rule("lit", True, "u", b"/tea/x"), sigs.Rule("re", True, "ah", r"sel\s*ect\d+"),
             sigs.Rule("re", False, "b", r"^start"), sigs.Rule("re", False, "b", r"end$"),
             sigs.Rule("re", False, "uahb", r"[0-9]{3}x"),           # no >= 4-byte factor: always-run
             sigs.Rule("lit", True, "h", b"evil"),                    # duplicate literal, other zone
             sigs.Rule("re", False, "a", r"(a)\1")]                   # PCRE-only: rejected
    b = workloads.c4_blob(sigs.SigSet(rules))
    items = [
        {"host": "cafe.example.com", "uri": "/tea/x", "https": True, "body": b"xxEVILxx"},
        {"host": "cafe.example.com", "uri": "/tea/a", "https": True, "body": b"casesensitive CaseSensitive"},
        {"host": "cafe.example.com", "uri": "/tea/a", "https": True, "body": b"casesensitive"},
        {"host": "cafe.example.com", "uri": "/tea/a", "https": True, "args": "q=SEL  ECT42"},
        {"host": "cafe.example.com", "uri": "/tea/a", "https": True, "body": b"start...end\n"},
        {"host": "cafe.example.com", "uri": "/tea/a", "https": True, "body": b"x start end\n\n"},
        {"host": "cafe.example.com", "uri": "/tea/ev", "args": "il=1", "https": True},   # no cross-zone match
        {"host": "cafe.example.com", "uri": "/coffee", "https": True, "headers": [("X-A", "123x evil")]},
        {"host": "cafe.example.com", "uri": "/tea", "https": False, "body": b"evil"},      # redirected: no WAF
        {"host": "cafe.example.com", "uri": "/tea/", "https": True, "body": b"ev"},
        {"host": "cafe.example.com", "uri": "/tea/q", "https": True, "body": b"evi"},     # tail of arena
    ]
    reqs, arena = records.from_dicts(items)
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "edge")
    assert got[0]["n_hits"] == 2 and got[1]["n_hits"] == 1 and got[2]["n_hits"] == 0
    assert got[6]["n_hits"] == 0 and got[8]["n_hits"] == 0


def test_waf_scan_every_alignment(eng):
    """Literals planted at every residue mod 1024 of the arena (every lane of a scan wave, every
    byte of a lane, windows straddling lanes 62/63 and chunk ends) plus one ending exactly at the
    arena's last byte."""
    rules = [sigs.Rule("lit", True, "b", b"qzxjv"), sigs.Rule("lit", False, "b", b"WXYZ"),
             sigs.Rule("re", True, "b", r"kqpz=[0-9]{3}")]
    b = workloads.c4_blob(sigs.SigSet(rules))
    rng = np.random.Generator(np.random.PCG64(7))
    items = []
    pos = 0
    for i in range(3000):
        tok = [b"QzXjV", b"WXYZ", b"kqpz=123"][i % 3]
        blen = int(rng.integers(16, 2200))
        at = int(rng.integers(0, blen - len(tok)))
        body = bytearray(b"a" * blen)
        body[at:at + len(tok)] = tok
        items.append({"host": "cafe.example.com", "uri": "/tea/x", "https": True, "body": bytes(body)})
    items.append({"host": "cafe.example.com", "uri": "/tea/x", "https": True, "body": b"aaaqzxjv"})
    reqs, arena = records.from_dicts(items)
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "alignment")
    assert (exp["n_hits"] == 1).sum() == len(items)


def test_waf_zone_boundaries(eng):
    """Patterns at the first and last byte of every zone, at both arena parities (the stride-2
    scan keys 4-byte patterns on windows that begin a byte before or end a byte after them, i.e.
    possibly in the neighbouring zone or request)."""
    rules = [sigs.Rule("lit", True, "uahb", b"/zq9"), sigs.Rule("lit", False, "ahb", b"kx7w"),
             sigs.Rule("re", False, "uahb", r"(k7fo|0ovr|gizw3)[a-z0-9]+--"),
             sigs.Rule("re", True, "ahb", r"qvxj\s*\(\d+\)"), sigs.Rule("lit", True, "ahb", b"jjqqz")]
    b = workloads.c4_blob(sigs.SigSet(rules))
    rng = np.random.Generator(np.random.PCG64(11))
    toks = [b"kx7w", b"k7foab--", b"QVXJ(12)", b"jjqqz", b"0ovr9--"]
    items = []
    for i in range(4000):
        t = toks[i % len(toks)]
        pad = b"a" * int(rng.integers(0, 7))
        where = (i // len(toks)) % 6
        it = {"host": "cafe.example.com", "uri": "/tea/zq9" + "b" * int(rng.integers(0, 5)), "https": True}
        if where == 0:
            it["args"] = (t + pad).decode()
        elif where == 1:
            it["args"] = (pad + t).decode()
        elif where == 2:
            it["headers"] = [(t.decode(), "v" + pad.decode())]
        elif where == 3:
            it["body"] = t + pad
            it["args"] = pad.decode()
        elif where == 4:
            it["body"] = pad + t
        else:
            it["uri"] = "/tea" + pad.decode() + "/zq9"
            it["args"] = (t + pad).decode()
        items.append(it)
    reqs, arena = records.from_dicts(items)
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "zone-boundaries")
    assert (exp["n_hits"] >= 2).sum() > 3000


def test_waf_prefix_regex_dfa_entry(eng):
    """Prefix-mode regexes (k_waf_exact starts their anchored DFA after the verified prefix
    literal, DLit.dfa_entry): case-insensitive prefixes, a case-sensitive regex whose prefix has
    letters (no skip: the literal matches any case), a letter-free case-sensitive prefix (skip), a
    regex that accepts right after its prefix, and `$` with the zone ending at, or one newline
    after, the match -- against the oracle's PCRE."""
    rules = [sigs.Rule("re", True, "ab", r"(abcd|efgh)\d+x"), sigs.Rule("re", False, "ab", r"Qwerty[0-9]{2}"),
             sigs.Rule("re", False, "ab", r"12345[a-z]+"), sigs.Rule("re", True, "ab", r"wxyz\d*"),
             sigs.Rule("re", False, "ab", r"mnopq\d+$"), sigs.Rule("re", True, "ab", r"zyxwv[^>]{0,4}on")]
    b = workloads.c4_blob(sigs.SigSet(rules))
    bodies = [b"ABCD12x", b"abcd12", b"..efgh9x", b"abcdx", b"qwerty12", b"Qwerty12", b"QWERTY12",
              b"12345abc", b"12345", b"x12345Z", b"WXYZ", b"wxyz", b"mnopq12", b"mnopq12\n", b"mnopq12x",
              b"mnopq12\n\n", b"ZYXWVabon", b"zyxwvabcdeon", b"zyxwv on", b"efgh", b"abcd9", b"abcd9X"]
    items = []
    for i, body in enumerate(bodies * 3):
        it = {"host": "cafe.example.com", "uri": "/tea/x", "https": True}
        pad = b"." * (i % 5)
        if i % 2:
            it["body"] = pad + body
        else:
            it["args"] = (pad + body).decode()
            it["body"] = b"-" * (i % 3)
        items.append(it)
    reqs, arena = records.from_dicts(items)
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "prefix-dfa-entry")
    assert (exp["n_hits"] > 0).sum() > 20


def test_e2e_kats_on_gpu(eng):
    adv = golden("advanced_routing.json")
    for case in adv["cases"]:
        vs = adv["virtual_servers"][case["vs"]]
        b = vs_blob([vs])
        eng.load(b, 1)
        reqs, arena = records.from_dicts([kat_request(adv["host"], adv["uri"], case["request"])])
        v, _ = eng.match_host(reqs, arena)
        ups = upstream_table(b)
        assert v[0]["action"] == 0
        assert ups[v[0]["upstream_id"]] == f"vs_default_{vs['metadata']['name']}_{case['expect_upstream']}", case


def test_match_values_on_gpu(eng):
    from test_oracle import _value_vs
    for case in golden("match_values.json")["cases"]:
        b = vs_blob([_value_vs(case["value"])])
        eng.load(b, 1)
        reqs, arena = records.from_dicts([{"host": "mv.example.com", "uri": "/x",
                                           "headers": [("X-V", case["subject"])]}])
        v, _ = eng.match_host(reqs, arena)
        ups = upstream_table(b)
        assert ups[v[0]["upstream_id"]] == ("vs_default_mv_m" if case["match"] else "vs_default_mv_d"), case


def test_location_semantics_on_gpu(eng):
    from test_oracle import test_location_lookup_semantics  # noqa: F401 (same config, GPU vs oracle)
    conf = """
    http {
      upstream u1 { server 1.1.1.1; }
      upstream u2 { server 1.1.1.2; }
      server {
        listen 80 default_server;
        server_name t.example.com *.wild.example.com .dot.example.com www.tail.*;
        if ($http_x_forwarded_proto = 'http') { return 301 https://$host$request_uri; }
        location = /exact { proxy_pass http://u1; }
        location /tea/ { proxy_pass http://u1; }
        location /img/ { return 403; }
        location ^~ /static { proxy_pass http://u2; }
        location ~ \\.php$ { proxy_pass http://u2; }
        location ~* \\.JPG$ { proxy_pass http://u1; }
        location / { proxy_pass http://u1; }
      }
      server { listen 80; server_name other.example.com a.wild.example.com; location / { return 404; } }
    }"""
    b = blob.make_blob(conf, {})
    uris = ["/exact", "/exact/", "/tea", "/tea/x", "/img", "/static/a.php", "/a.php", "/b.jpg", "/b.jpgx",
            "/img/x", "", "/t\x00"]
    hosts = ["t.example.com", "x.wild.example.com", "a.wild.example.com", "dot.example.com", "z.dot.example.com",
             "www.tail.org", "www.tail.", "other.example.com", "[::1]:80", "T.EXAMPLE.COM.", "x/y", ".lead.example.com"]
    items = [{"host": h, "uri": u} for h in hosts for u in uris]
    items += [{"host": "t.example.com", "uri": "/a", "headers": [("X-Forwarded-Proto", "http")]},
              {"host": "t.example.com", "uri": "/a", "headers": [("X-Forwarded-Proto", "HTTP")]}]
    reqs, arena = records.from_dicts(items)
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "locations")


def test_counters(eng):
    ss = workloads.c4_sigset(400, 100)
    reqs, arena = records.gen_c4(10_000, ss, plant_rate=0.1)
    b = workloads.c4_blob(ss, "monitoring")
    eng.load(b, 3)
    eng.counters_reset()
    got, gh = eng.match_host(reqs, arena)
    c = eng.counters()
    st = eng.stats()
    nl = st["n_locations"]
    loc = got["location_id"][got["location_id"] != 0xFFFFFFFF]
    assert np.array_equal(c[:nl], np.bincount(loc, minlength=nl))
    assert np.array_equal(c[nl:], np.bincount(gh, minlength=st["n_sigs"]))


def test_hit_cap_overflow_reported(eng):
    ss = workloads.c4_sigset(200, 50)
    reqs, arena = records.gen_c4(5_000, ss, plant_rate=0.5)
    eng.load(workloads.c4_blob(ss), 3)
    with pytest.raises(engine.GmError) as ei:
        eng.match_host(reqs, arena, hit_cap=10)
    assert ei.value.code == engine.GM_E_OVERFLOW


def test_empty_and_generation_swap(eng):
    eng.load(workloads.c1_blob(), 9)
    reqs, arena = records.from_dicts([])
    v, h = eng.match_host(reqs, arena)
    assert len(v) == 0
    reqs, arena = records.gen_c1(1000)
    v1, _ = eng.match_host(reqs, arena)
    assert (v1["gen"] == 9).all()
    with pytest.raises(engine.GmError):
        eng.load(b"GMB1\x00", 10)
    v2, _ = eng.match_host(reqs, arena)
    assert np.array_equal(v1, v2)


def test_c3_regex_locations_parity(eng):
    """C3: 1k regex locations, all in union-DFA slices (k_rloc_multi: the stats pin that path, no
    server is left to the factor prefilter; the X$ ones in reversed slices that run from the URI's
    end), URIs 32-256 B, 40 % crafted to hit; PCRE-only locations reached in order give
    GM_ACT_UNSUPPORTED on both sides."""
    regs = workloads.c3_regexes()
    reqs, arena = workloads.gen_c3(50_000, regs)
    got, gh, exp, eh = run_both(eng, workloads.c3_blob(regs), reqs, arena)
    st = eng.stats()
    assert st["n_rsl_slices"] > 0 and st["n_rk_prefilter"] == 0 and st["n_rsl_reversed"] > 0, st
    assert_verdicts_equal(got, exp, gh, eh, "c3")
    hit = np.isin(got["location_id"], np.arange(3, len(regs) + 3))
    assert 0.3 < hit.mean() < 0.99


def test_regex_location_prefilter_edges(eng):
    """More than RLOC_SEQ_MAX regex locations: > RK_K candidates sharing one key (rescan), the
    always list (no 4-byte factor) interleaved in config order, caseless, PCRE-only reached."""
    pats = [("~", f"^/api/v{i}/item$") for i in range(12)]          # 12 candidates on "/api"
    pats += [("~", r"^/x\d"), ("~*", r"\.PHP$"), ("~", r"^/api/(?=v)"), ("~", r"/api/v11/"),
             ("~", r"^/a"), ("~*", r"/API/Z")]
    locs = "".join(f'    location {op} "{p}" {{ return 2{i:02d}; }}\n' for i, (op, p) in enumerate(pats))
    conf = ("http {\n  server {\n    listen 80 default_server;\n    server_name e.example.com;\n"
            "    location / { return 404; }\n" + locs + "  }\n}\n")
    b = blob.make_blob(conf, {})
    uris = [f"/api/v{i}/item" for i in range(12)] + ["/api/v11/item/", "/api/v11/x", "/api/w", "/x7",
            "/y.php", "/y.PhP", "/a", "/b/api/z", "/b/API/z", "/api/v3/item/", "/", "", "/ap", "/API/v1/item"]
    reqs, arena = records.from_dicts([{"host": "e.example.com", "uri": u} for u in uris])
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "regex prefilter edges")


GRPC_CONF = """
http {
  upstream g1 { server 1.1.1.1; }
  upstream u1 { server 1.1.1.2; }
  server {
    listen 80 default_server;
    server_name g.example.com;
    location /grpc/ { grpc_pass grpc://g1; }
    location /grpcs { grpc_pass grpcs://g1; }
    location = /r304 { return 304; }
    location = /r307 { return 307; }
    location /nested { proxy_pass http://u1; if ($arg_x) { return 403; } }
    location / { proxy_pass http://u1; }
  }
  server {
    listen 80;
    server_name rw.example.com;
    if ($http_x_early = 'yes') { return 418; }
    rewrite ^/old/(.*)$ /new/$1 last;
    location / { proxy_pass http://u1; }
  }
}"""


def test_grpc_return_and_unsupported_constructs_on_gpu(eng):
    """grpc_pass proxies like proxy_pass (incl. auto_redirect, nginx.org/grpc-services,
    version1/nginx.ingress.tmpl:154-158); `return 304` is not a redirect; a nested `if` in a
    location and a server-level `rewrite` defer to nginx (GM_ACT_UNSUPPORTED), counted."""
    b = blob.make_blob(GRPC_CONF, {})
    items = [{"host": "g.example.com", "uri": u} for u in ("/grpc/x", "/grpc", "/grpcs/a", "/r304", "/r307",
                                                           "/nested/a", "/other")]
    items += [{"host": "rw.example.com", "uri": "/old/a"},
              {"host": "rw.example.com", "uri": "/x", "headers": [("X-Early", "yes")]}]
    reqs, arena = records.from_dicts(items)
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "grpc / return / unsupported")
    ups = upstream_table(b)
    assert got[0]["action"] == 0 and ups[got[0]["upstream_id"]] == "g1"
    assert got[1]["action"] == 3 and got[1]["status"] == 301          # auto_redirect for grpc_pass
    assert got[2]["action"] == 0 and ups[got[2]["upstream_id"]] == "g1"
    assert got[3]["action"] == 2 and got[3]["status"] == 304
    assert got[4]["action"] == 1 and got[4]["status"] == 307
    assert got[5]["action"] == 8 and got[6]["action"] == 0
    assert got[7]["action"] == 8                                       # server rewrite reached
    assert got[8]["action"] == 2 and got[8]["status"] == 418           # the `if` before it answers first
    eng.load(b, 2)
    assert eng.stats()["n_rejected_other"] == 2


def test_regex_locations_factor_prefilter_fallback(eng):
    """A server whose regex locations include one no union-DFA group can hold (2^12-state DFA,
    more rows than ALW_GROUP_BYTES) stays on the factor prefilter (k_rloc, gm_compile.cpp): the
    stats pin the path, and every verdict equals the oracle's -- the big regex, the ones before
    and after it in config order, and URIs that match none."""
    pats = [("~", f"^/r{i}/[0-9]+$") for i in range(10)] + [("~", "/[ab]*a[ab]{11}z")] + \
           [("~*", r"\.JPG$"), ("~", r"^/api/v[0-9]/"), ("~", "/abz")]
    locs = "".join(f'    location {op} "{p}" {{ return 2{i:02d}; }}\n' for i, (op, p) in enumerate(pats))
    conf = ("http {\n  server {\n    listen 80 default_server;\n    server_name f.example.com;\n"
            "    location / { return 404; }\n" + locs + "  }\n}\n")
    b = blob.make_blob(conf, {})
    rng = np.random.default_rng(17)
    uris = []
    for _ in range(20_000):
        k = rng.integers(0, 6)
        if k == 0:
            uris.append(f"/r{rng.integers(0, 12)}/{rng.integers(0, 99999)}")
        elif k == 1:
            tail = "".join(rng.choice(list("ab"), rng.integers(10, 24)))
            uris.append(f"/q/{tail}{'z' if rng.random() < 0.7 else 'y'}")
        elif k == 2:
            uris.append(f"/img/{rng.integers(0, 999)}.{'jpg' if rng.random() < 0.5 else 'JPG'}")
        elif k == 3:
            uris.append(f"/api/v{rng.integers(0, 12)}/x")
        elif k == 4:
            uris.append("/abz" if rng.random() < 0.5 else "/ab")
        else:
            uris.append("/" + "".join(rng.choice(list("abz/r0"), rng.integers(1, 40))))
    reqs, arena = records.from_dicts([{"host": "f.example.com", "uri": u} for u in uris])
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    st = eng.stats()
    assert st["n_rk_prefilter"] == 1 and st["n_rsl_slices"] == 0, st
    assert_verdicts_equal(got, exp, gh, eh, "regex locations, factor prefilter")
    assert len(np.unique(got["status"])) >= 8


def test_regex_locations_reversed_slices(eng):
    """X$ regex locations in reversed union-DFA slices (^(\\n)?rev(X) run from the URI's last byte
    backwards) beside forward anchored / unanchored ones, in config order: URIs ending in '\\n'
    ('$' before a final newline), empty URIs, matches of several patterns (the first in config
    order wins) -- every verdict equals the oracle's."""
    pats = [("~", r"\.php$"), ("~", "^/a/[0-9]+"), ("~*", r"/(img|css)/[a-z0-9]+\.(png|jpg)$"), ("~", "/b/c"),
            ("~", "x[0-9]{2,4}$"), ("~", "^/q$"), ("~", "(foo|bar)+baz$"), ("~", r"/v[0-9]/"),
            ("~", "[^/]+/z$"), ("~", "/a/1"), ("~*", "END$"), ("~", "a.b$")]
    locs = "".join(f'    location {op} "{p}" {{ return 2{i:02d}; }}\n' for i, (op, p) in enumerate(pats))
    conf = ("http {\n  server {\n    listen 80 default_server;\n    server_name r.example.com;\n"
            "    location / { return 404; }\n" + locs + "  }\n}\n")
    b = blob.make_blob(conf, {})
    rng = np.random.default_rng(23)
    parts = ["/a", "/b", "/c", "/img", "/css", "/q", "/v1", "/v22", "/foo", "/bar", "/z", "/x12", "/x1234",
             "/1", "/42", "baz", ".php", ".PNG", ".jpg", "END", "end", "a.b", "a_b", "foobarbaz"]
    uris = ["", "\n", "/q", "/q\n", "/q\n\n", "/x.php\n", "/a/1", "/end\n", "/a.b", "/a.b\n"]
    for _ in range(30_000):
        u = "".join(parts[int(k)] for k in rng.integers(0, len(parts), int(rng.integers(1, 7))))
        if rng.random() < 0.1:
            u += "\n"
        uris.append(u)
    reqs, arena = records.from_dicts([{"host": "r.example.com", "uri": u} for u in uris])
    got, gh, exp, eh = run_both(eng, b, reqs, arena)
    st = eng.stats()
    assert st["n_rsl_reversed"] > 0 and st["n_rk_prefilter"] == 0, st
    assert_verdicts_equal(got, exp, gh, eh, "reversed regex-location slices")
    assert len(np.unique(got["status"])) >= 10
