"""The reference's own configs and e2e known answers, classified on the GPU (libgpumatch.so) and
by the oracle on the same requests:

- the three whole-VirtualServer configs of virtualserver_test.go:163-731, each with a
  VirtualServerRoute -- the verdict's upstream must be the one the Go expected struct binds to the
  selected location (plain / split bucket / rules match);
- the mergeable master + minions of ingress_test.go:347-563;
- tests/suite/test_v_s_route.py:260-322 (VSR delegation, no endpoints -> 502, deleted VSR -> 404)
  and tests/suite/test_virtual_server.py:25-73 (host change -> old host 404, restore, 502).

A 502 is a normal verdict (proxy to the upstream whose only server is the 502 sentinel,
virtualserver.go:14,210-217); 404 is the default server's `location / { return 404; }`
(nginx.tmpl:81-102) or no matching location."""

import re

import numpy as np
import pytest

from gpumatch import blob, confgen, engine, records
from helpers import assert_verdicts_equal, golden, upstream_table
from oracle_py import Oracle

pytestmark = pytest.mark.gpu
G = golden("reference_configs.json")
E2E = golden("e2e_routes.json")


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    return engine.Engine(0)


def _run(eng, b, items, gen=7):
    reqs, arena = records.from_dicts(items)
    eng.load(b, gen)
    got, gh = eng.match_host(reqs, arena)
    exp, eh = Oracle(b, gen).match(reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "reference config")
    return got


def _servers_of(b):
    """upstream name -> its `server` addresses in the generation's config text"""
    out = {}
    for kind, _, data in blob.parse_blob(b):
        if kind == blob.ENTRY_SIGS:
            continue
        for m in re.finditer(rb"upstream\s+(\S+)\s*\{(.*?)\}", data, flags=re.S):
            out[m.group(1).decode()] = re.findall(rb"^\s*server\s+(\S+)", m.group(2), flags=re.M)
    return {k: [x.decode() for x in v] for k, v in out.items()}


def _vs_blob(vs, vsr_store, endpoints, params=None):
    p = confgen.default_config_params()
    p.update(params or {})
    files = confgen.virtual_server_files([vs], base=p, vsr_store=vsr_store, pem_name="",
                                         endpoints_of=lambda ns, svc, port: endpoints.get(f"{ns}/{svc}:{port}", []))
    return blob.make_blob(confgen.render_main(p), files)


def _rid(i):
    return bytes([(i * 37 + k * 11) & 0xFF for k in range(16)])


@pytest.mark.parametrize("name", ["basic", "splits", "rules"])
def test_reference_vs_configs_on_gpu(eng, name):
    case = G["vs_configs"][name]
    store = {"%s/%s" % (v["metadata"]["namespace"], v["metadata"]["name"]): v for v in case["vsrs"]}
    b = _vs_blob(case["vs"], store, case["endpoints"], case["params"])
    exp = case["expected"]
    loc_ups = {p: u.split("://", 1)[1] for p, u in exp["Server"]["Locations"]}
    irl = {x["Path"]: x["Destination"] for x in exp["Server"]["InternalRedirectLocations"]}
    host = "cafe.example.com"
    items = []
    for path in ("/tea", "/coffee", "/tea/x", "/coffee/y", "/other", "/"):
        for k in range(24):
            it = {"host": host, "uri": path, "rid": _rid(k + 100 * len(items))}
            if k % 3 == 1:
                it["headers"] = [("X-Version", "v2")]
            if k % 4 == 1:
                it["args"] = "version=v2"
            if k == 5:
                it["headers"] = [("X-Forwarded-Proto", "http")]
            items.append(it)
    v = _run(eng, b, items)
    ups = upstream_table(b)
    for it, r in zip(items, v):
        path = it["uri"]
        base = "/tea" if path.startswith("/tea") else "/coffee" if path.startswith("/coffee") else None
        if exp["Server"].get("RedirectToHTTPSBasedOnXForwarderProto") and ("X-Forwarded-Proto", "http") in it.get("headers", []):
            assert r["action"] == 1 and r["status"] == 301
            continue
        if base is None:
            assert r["status"] == 404, (it, r)     # no `location /` in the VS server
            continue
        assert r["action"] == 0, (it, r)
        if base in loc_ups:
            want = loc_ups[base]
        else:
            var = irl[base]                          # $vs_default_cafe_splits_<i> / _rules_<i>
            idx = var.rsplit("_", 1)[1]
            if "splits" in var:
                want = loc_ups[f"@splits_{idx}_split_{int(r['split_bucket'])}"]
            else:
                m = int(r["match_idx"])
                want = loc_ups[f"@rules_{idx}_default" if m == 0xFF else f"@rules_{idx}_match_{m}"]
        assert ups[r["upstream_id"]] == want, (it, r)
    if name == "splits":
        assert set(v["split_bucket"][v["route_kind"] == 2].tolist()) == {0, 1}
    if name == "rules":
        assert (v["match_idx"][v["route_kind"] == 3] == 0).any() and (v["match_idx"][v["route_kind"] == 3] == 0xFF).any()


def test_reference_mergeable_on_gpu(eng):
    k = G["mergeable"]
    cfg = confgen.generate_nginx_cfg_for_mergeable(
        {"Ingress": k["master"], "Endpoints": k["master_endpoints"]},
        [{"Ingress": m, "Endpoints": e} for m, e in k["minions"]], k["pems"], confgen.default_config_params())
    b = blob.make_blob(confgen.render_main(), {confgen.object_meta_to_file_name(k["master"]): confgen.render_ingress(cfg)})
    items = [{"host": "cafe.example.com", "uri": u, "https": h} for u in ("/coffee", "/tea/x", "/", "/teapot")
             for h in (True, False)]
    v = _run(eng, b, items)
    ups = upstream_table(b)
    want = {u[0] for u in k["expected"]["upstreams"]}
    for it, r in zip(items, v):
        if not it["https"]:
            assert r["action"] == 1 and r["status"] == 301      # SSLRedirect (nginx.ingress.tmpl:76-80)
        elif it["uri"] == "/":
            assert r["status"] == 404
        else:
            assert r["action"] == 0 and ups[r["upstream_id"]] in want


def _status(r, ups, servers):
    if r["action"] == 0:
        return 502 if servers[ups[r["upstream_id"]]] == [confgen.NGINX502_SERVER] else 200
    return int(r["status"])


def _normalize_on_gpu(eng, paths):
    """Raw request paths -> nginx $uri through gm_normalize_uris."""
    import torch
    dev = torch.device("cuda", 0)
    buf = b"".join(p.encode().ljust(64, b"\0") for p in paths)
    d_a = torch.from_numpy(np.frombuffer(buf, np.uint8).copy()).to(dev)
    d_off = torch.tensor([64 * i for i in range(len(paths))], dtype=torch.int64, device=dev)
    d_len = torch.tensor([len(p) for p in paths], dtype=torch.int32, device=dev)
    d_ol = torch.zeros(len(paths), dtype=torch.int32, device=dev)
    d_o = torch.zeros_like(d_a)
    eng.normalize_uris_ptr(d_a.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(paths), d_o.data_ptr(),
                           d_ol.data_ptr(), 0)
    eng.sync(0)
    o = d_o.cpu().numpy().tobytes()
    ol = d_ol.cpu().numpy().view(np.uint32)
    return [o[64 * i:64 * i + int(ol[i])].decode() for i in range(len(paths))]


def test_e2e_virtual_server_route_on_gpu(eng):
    """test_v_s_route.py: VSR delegation, backend port change -> 502, VSR deleted -> 404."""
    k = E2E["v_s_route"]
    vs = dict(k["vs"])
    vs["metadata"] = dict(vs["metadata"], namespace=k["vs_namespace"])
    vsrs = {}
    for ns, v in k["vsrs"]:
        v = dict(v)
        v["metadata"] = dict(v["metadata"], namespace=ns)
        vsrs[f"{ns}/{v['metadata']['name']}"] = v
    host = vs["spec"]["host"]
    for step in k["steps"]:
        store = {key: v for key, v in vsrs.items() if key not in step.get("deleted", [])}
        dead = set(step.get("no_endpoints", []))
        eps = {}
        for v in list(store.values()):
            for u in v["spec"]["upstreams"]:
                key = f"{v['metadata']['namespace']}/{u['service']}:{u['port']}"
                if key not in dead:
                    eps[key] = ["10.0.1.%d:80" % (len(eps) + 1)]
        b = _vs_blob(vs, store, eps)
        items = [{"host": host, "uri": p} for p, _ in step["paths"]]
        v = _run(eng, b, items)
        ups, servers = upstream_table(b), _servers_of(b)
        got = [_status(r, ups, servers) for r in v]
        assert got == [s for _, s in step["paths"]], step["step"]


def test_e2e_virtual_server_host_change_on_gpu(eng):
    """test_virtual_server.py:25-73: after a host change the old host answers 404 and the new one
    200; restoring swaps them back; a backend's port change gives 502.  The test's URLs carry a
    doubled slash ("//backend1"): the raw paths go through the GPU's $uri normalisation."""
    k = E2E["virtual_server"]
    ns = k["vs_namespace"]
    gen = 20
    for step in k["steps"]:
        vs = dict(k[step["config"]])
        vs["metadata"] = dict(vs["metadata"], namespace=ns)
        dead = set(step.get("no_endpoints", []))
        eps = {f"{ns}/{u['service']}:{u['port']}": ["10.0.2.1:80"] for u in vs["spec"]["upstreams"]
               if f"{ns}/{u['service']}:{u['port']}" not in dead}
        b = _vs_blob(vs, {}, eps)
        raw = [p for _, p, _ in step["requests"]]
        uris = _normalize_on_gpu(eng, raw)
        assert all(u == "/" + p.lstrip("/") for u, p in zip(uris, raw))
        items = [{"host": h, "uri": u, "ruri": p} for (h, p, _), u in zip(step["requests"], uris)]
        gen += 1
        v = _run(eng, b, items, gen)
        assert (v["gen"] == gen).all()
        ups, servers = upstream_table(b), _servers_of(b)
        assert [_status(r, ups, servers) for r in v] == [s for _, _, s in step["requests"]], step["step"]
