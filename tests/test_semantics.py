"""CPU: the verdict-affecting directives and the default-deny compile on the
oracle's known answers (tests/semantics_cases.py), and the compiler's counts and reject log on a
compile-only context.  The same cases run on the GPU against the oracle in test_gpu_semantics.py."""

import numpy as np
import pytest

import semantics_cases as SC
from gpumatch import engine, records
from oracle_py import Oracle


def _oracle(b, items, gen=3):
    reqs, arena = records.from_dicts(items)
    v, _ = Oracle(b, gen).match(reqs, arena)
    return v


@pytest.mark.parametrize("name", sorted(SC.ROUTE_CASES))
def test_route_kats_oracle(name):
    b, cases = SC.ROUTE_CASES[name]()
    v = _oracle(b, [c for c, _ in cases])
    for (it, want), r in zip(cases, v):
        assert r["action"] == want, (name, {k: it[k] for k in it if k != "body"}, len(it.get("body", b"")), r)
        if want == SC.TOO_LARGE:
            assert r["status"] == 413 and r["upstream_id"] == 0xFFFFFFFF and r["waf_mode"] == 0


@pytest.mark.parametrize("name", sorted(SC.MATCH_CASES))
def test_realip_kats_oracle(name):
    b, cases = SC.MATCH_CASES[name]()
    v = _oracle(b, [c for c, _ in cases])
    for (it, want), r in zip(cases, v):
        if want == SC.UNSUPPORTED:
            assert r["action"] == SC.UNSUPPORTED, (name, it, r)
        else:
            assert r["action"] == SC.PROXY and r["match_idx"] == want, (name, it, r)


def test_default_deny_oracle_and_compile():
    b, cases, rejects = SC.default_deny_case()
    v = _oracle(b, [c for c, _ in cases])
    for (it, want), r in zip(cases, v):
        assert r["action"] == want, (it["host"], it["uri"], r)
    e = engine.Engine(compile_only=True)
    e.load(b, 1)
    st = e.stats()
    got = e.rejects()
    for x in rejects:
        assert x in got, (x, got)
    assert st["n_rejected_other"] == len(got), (st["n_rejected_other"], got)


def test_http_unknown_counted_once():
    b, _ = SC.http_unknown_case()
    e = engine.Engine(compile_only=True)
    e.load(b, 1)
    assert e.stats()["n_rejected_other"] == 1 and e.rejects() == ["http: limit_req zone=one burst=5"]


def test_reference_templates_compile_clean():
    """Every directive the reference templates render (Ingress incl. gRPC / HSTS / realip / wallarm,
    VirtualServer incl. realip) is known to the compile: nothing rejected."""
    from gpumatch import blob, confgen
    p = confgen.default_config_params()
    p.update(SetRealIPFrom=["10.0.0.0/8"], RealIPHeader="X-Forwarded-For", RealIPRecursive=True,
             MainEnableWallarm=True, ClientMaxBodySize="2m", ProxyProtocol=True)
    ing = SC._ingress("cafe", "cafe.example.com", [("/tea", "tea"), ("/", "def")],
                      {"wallarm.com/mode": "block", "wallarm.com/parser-disable": "base64"})
    vs = SC._rules_vs("vs.example.com", {"header": "x-v"}, ["a"])
    files = confgen.ingress_files([ing], base=p)
    files.update(confgen.virtual_server_files([vs], base=p, pem_name=""))
    e = engine.Engine(compile_only=True)
    e.load(blob.make_blob(confgen.render_main(p), files), 1)
    st = e.stats()
    assert st["n_rejected_other"] == 0, e.rejects()
    assert st["n_realip"] == 2   # the cafe and the VS server (the default server has none)
