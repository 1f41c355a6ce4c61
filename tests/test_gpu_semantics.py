"""GPU parity for the verdict-affecting directives and the default-deny compile:
libgpumatch.so against the oracle, bit for bit, on tests/semantics_cases.py's known answers --

- client_max_body_size: a 1k location with Content-Length bodies around the limit, chunked bodies
  (checked only when proxied), the auto_redirect and default-server orders, and a VirtualServer
  whose `return 418` location (1m) and named locations (1k) disagree;
- realip: $remote_addr / $remote_port rules under X-Forwarded-For (recursive), X-Real-IP (the
  reference fixture's values), a named header and proxy_protocol (deferred when trusted); then
  20k requests of random forwarded-address lists through a rules route and `hash $remote_addr
  $remote_port consistent` / ip_hash balancers (the address text and bytes the device computes
  must equal the oracle's);
- default-deny: auth_basic / auth_request snippets and http-level unknown directives:
  GM_ACT_UNSUPPORTED, counted; the access module (allow / deny, the stock stub_status server);
- the wire parser's chunked flag (GM_REQ_CHUNKED) feeding the 413 decision."""

import numpy as np
import pytest

import semantics_cases as SC
from gpumatch import blob, confgen, engine, records, wire
from helpers import assert_verdicts_equal
from oracle_py import Balancer, Oracle, parse_requests

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    return engine.Engine(0)


def _both(e, b, items, gen=9):
    reqs, arena = records.from_dicts(items)
    e.load(b, gen)
    got, gh = e.match_host(reqs, arena)
    exp, eh = Oracle(b, gen).match(reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, "semantics")
    return got


@pytest.mark.parametrize("name", sorted(SC.ROUTE_CASES))
def test_route_kats_gpu(eng, name):
    b, cases = SC.ROUTE_CASES[name]()
    v = _both(eng, b, [c for c, _ in cases])
    assert v["action"].tolist() == [w for _, w in cases], name
    # every request counted at its location once, 413 included
    c = eng.counters()[:eng.stats()["n_locations"]]
    loc = v["location_id"][v["location_id"] != 0xFFFFFFFF]
    assert np.array_equal(c, np.bincount(loc, minlength=len(c)).astype(np.uint64))


@pytest.mark.parametrize("name", sorted(SC.MATCH_CASES))
def test_realip_kats_gpu(eng, name):
    b, cases = SC.MATCH_CASES[name]()
    v = _both(eng, b, [c for c, _ in cases])
    for (it, want), r in zip(cases, v):
        if want == SC.UNSUPPORTED:
            assert r["action"] == SC.UNSUPPORTED, (name, it, r)
        else:
            assert r["action"] == SC.PROXY and r["match_idx"] == want, (name, it, r)


def test_default_deny_gpu(eng):
    b, cases, rejects = SC.default_deny_case()
    v = _both(eng, b, [c for c, _ in cases])
    assert v["action"].tolist() == [w for _, w in cases]
    got = eng.rejects()
    assert all(x in got for x in rejects) and eng.stats()["n_rejected_other"] == len(got)


def test_reference_basic_fixture_realip_gpu(eng):
    """virtualserver_test.go:163-282 with its SetRealIPFrom 0.0.0.0/0 / X-Real-IP / recursive (the
    fields round 3's fixture had dropped): the config compiles with realip and nothing rejected."""
    from helpers import golden
    case = golden("reference_configs.json")["vs_configs"]["basic"]
    assert case["params"]["SetRealIPFrom"] == ["0.0.0.0/0"] and case["params"]["RealIPHeader"] == "X-Real-IP"
    p = confgen.default_config_params()
    p.update(case["params"])
    store = {"%s/%s" % (x["metadata"]["namespace"], x["metadata"]["name"]): x for x in case["vsrs"]}
    files = confgen.virtual_server_files([case["vs"]], base=p, vsr_store=store, pem_name="",
                                         endpoints_of=lambda ns, s, port: case["endpoints"].get(f"{ns}/{s}:{port}", []))
    b = blob.make_blob(confgen.render_main(p), files)
    items = [{"host": "cafe.example.com", "uri": u, "raddr": "8.8.8.8", "headers": [("X-Real-IP", "1.2.3.4")]}
             for u in ("/tea", "/coffee", "/x")]
    v = _both(eng, b, items)
    st = eng.stats()
    assert st["n_realip"] == 1 and st["n_rejected_other"] == 0, eng.rejects()
    assert v["action"].tolist() == [0, 0, 4]


# ---------------------------------------------------------------- random forwarded lists
def _rand_addr(rng):
    k = int(rng.integers(0, 14))
    if k < 4:
        return "%d.%d.%d.%d" % tuple(int(x) for x in rng.integers(0, 256, 4))
    if k == 4:
        return "10.1.%d.%d" % tuple(int(x) for x in rng.integers(0, 256, 2))     # trusted
    if k == 5:
        return "192.168.%d.%d:%d" % (int(rng.integers(0, 256)), int(rng.integers(0, 256)), int(rng.integers(0, 70000)))
    if k in (6, 7):
        g = [("%x" % int(x)) if rng.random() < 0.5 else "0" for x in rng.integers(0, 65536, 8)]
        s = ":".join(g)
        if rng.random() < 0.3:
            s = s.upper()
        return "[%s]:%d" % (s, int(rng.integers(1, 65536))) if k == 7 else s
    if k == 8:
        return "::ffff:%d.%d.%d.%d" % tuple(int(x) for x in rng.integers(0, 256, 4))
    if k == 9:
        z = int(rng.integers(1, 7))
        head = ":".join("%x" % int(x) for x in rng.integers(0, 65536, int(rng.integers(0, 8 - z))))
        tail = ":".join("%x" % int(x) for x in rng.integers(0, 65536, int(rng.integers(0, 8 - z))))
        return head + "::" + tail
    return ["unknown", "1.2.3", "1.2.3.4.5", "::1::", "[::1]", "1.2.3.4:0", "1..2.3", "255.255.255.255",
            "0.0.0.0", "::"][int(rng.integers(0, 10))]


def _rand_requests(n, host, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    items = []
    for i in range(n):
        hdrs = []
        for _ in range(int(rng.integers(0, 4))):
            lst = [_rand_addr(rng) for _ in range(int(rng.integers(1, 4)))]
            sep = [", ", ",", " ", " , "][int(rng.integers(0, 4))]
            hdrs.append(("X-Forwarded-For", sep.join(lst) + ("," if rng.random() < 0.1 else "")))
        if rng.random() < 0.5:
            hdrs.append(("X-Real-IP", _rand_addr(rng)))
        conn = ["192.168.0.7", "10.1.0.1", "172.16.5.5", "::ffff:192.168.1.2", "2001:db8::7", ""][int(rng.integers(0, 6))]
        items.append({"host": host, "uri": "/", "raddr": conn, "headers": hdrs,
                      "remote_port": int(rng.integers(1, 65536)), "rid": bytes(rng.integers(0, 256, 16, dtype=np.uint8))})
    return items


@pytest.mark.parametrize("header,rec", [("X-Forwarded-For", True), ("X-Forwarded-For", False), ("X-Real-IP", True)])
def test_realip_random_parity(eng, header, rec):
    vals = ["10.1.0.1", "192.168.0.7", "2001:db8::7"] + ["%d.%d.%d.%d" % (a, b, c, d) for a, b, c, d in
                                                           np.random.Generator(np.random.PCG64(3)).integers(0, 256, (6, 4))]
    vs = SC._rules_vs("r.example.com", {"variable": "$remote_addr"}, vals)
    b = SC._vs_blob(vs, SetRealIPFrom=["192.168.0.0/16", "10.1.0.0/16", "2001:db8::/32"], RealIPHeader=header,
                    RealIPRecursive=rec)
    v = _both(eng, b, _rand_requests(20_000, "r.example.com", 11 + rec))
    assert (v["match_idx"] != 0xFF).sum() > 500


def test_rules_route_many_chains(eng):
    """A VirtualServer rules route with more (match, condition) chains than a truth table holds
    (RULES_TABLE_MAX = 8): 9 matches x 2 conditions = 18 chains, the final map evaluated on the
    device as ngx_http_map_find does (exact keys, then regexes in order) over the chains' string."""
    rng = np.random.Generator(np.random.PCG64(17))
    addrs = ["192.168.0.7", "10.1.0.1", "172.16.5.5", "2001:db8::7"]
    matches = []
    for k in range(9):
        matches.append({"values": [addrs[k % 4] if k < 8 else "~^1", "~^(%d|%d)" % (k, k + 1)],
                        "upstream": f"u{k + 1}"})
    ups = [{"name": f"u{k}", "service": f"svc{k}", "port": 80} for k in range(10)]
    vs = {"metadata": {"name": "m", "namespace": "default"},
          "spec": {"host": "m.example.com", "upstreams": ups,
                   "routes": [{"path": "/", "rules": {"conditions": [{"variable": "$remote_addr"},
                                                                     {"header": "X-Pick"}],
                                                      "matches": matches, "defaultUpstream": "u0"}}]}}
    b = SC._vs_blob(vs)
    items = _rand_requests(20_000, "m.example.com", 29)
    for it in items:
        it["headers"] = it["headers"] + [("X-Pick", str(int(rng.integers(0, 12))))]
    v = _both(eng, b, items)
    st = eng.stats()
    assert st["n_routes_rules"] == 1 and st["n_rejected_other"] == 0, eng.rejects()
    assert len(set(v["match_idx"].tolist())) >= 6


def test_rules_header_cookie_arg_spans(eng):
    """rules_generic's header / cookie / argument spans (its one LF-first header walk for every
    header and cookie source of the route) against the oracle's walks: a header condition (name case
    and '-' / '_' variants, repeated lines -- the first wins --, spaces around values, CR-less and
    colon-less lines, a ':' inside a name of the wanted length), a cookie condition over 0-3 Cookie
    lines (look-alike names, a "Cook:e" line, ',' and ';' separators, spaces around '='), an
    argument condition; long blocks (300 lines, 5 KiB values, 20 Cookie lines)."""
    rng = np.random.Generator(np.random.PCG64(41))
    ups = [{"name": f"u{k}", "service": f"svc{k}", "port": 80} for k in range(5)]
    vs = {"metadata": {"name": "sp", "namespace": "default"},
          "spec": {"host": "sp.example.com", "upstreams": ups,
                   "routes": [{"path": "/", "rules": {
                       "conditions": [{"header": "X-Ab-C"}, {"cookie": "sess"}, {"argument": "q"}],
                       "matches": [{"values": ["v1", "v1", "v1"], "upstream": "u1"},
                                   {"values": ["~^v[0-9]$", "v2", "~2"], "upstream": "u2"},
                                   {"values": ["", "~^v", "v3"], "upstream": "u3"},
                                   {"values": ["v3", "", ""], "upstream": "u4"}],
                       "defaultUpstream": "u0"}}]}}
    b = SC._vs_blob(vs)
    vals = ["v1", "v2", "v3", "V1", "x", ""]
    names = ["X-Ab-C", "x-ab-c", "X_AB_C", "X-Ab-Cd", "X-Ab", "X:Ab-C"]
    ck_tok = ["sess=v1", "sess=v2", " sess = v3", "sess2=v1", "SESS=v2", "xsess=v1", "sess", "a=b", "sess=v3;x"]
    args = ["q=v1", "q=v2", "Q=v3", "aq=v1", "q=", "q", "x=1&q=v2", "q=v3&q=v1", "&q=v1"]
    items = []
    for i in range(6000):
        hdrs = [("Accept", "*/*"), ("User-Agent", "t" * int(rng.integers(0, 60)))]
        for _ in range(int(rng.integers(0, 3))):
            v = vals[int(rng.integers(0, len(vals)))]
            v = " " * int(rng.integers(0, 3)) + v + " " * int(rng.integers(0, 3))
            hdrs.insert(int(rng.integers(0, len(hdrs) + 1)), (names[int(rng.integers(0, len(names)))], v))
        for _ in range(int(rng.integers(0, 4))):
            toks = [ck_tok[int(t)] for t in rng.integers(0, len(ck_tok), int(rng.integers(1, 5)))]
            seps = ["; ", ";", ", ", " ; "]
            hdrs.append(("Cookie", seps[int(rng.integers(0, 4))].join(toks)))
        u = rng.random()
        if u < 0.05:
            hdrs.append(("X-Raw", "a\nNoColonLine"))          # a line without ':' (bare LF)
        elif u < 0.065:
            hdrs.insert(0, ("X-Raw", "a\nX-Ab-C\r"))          # the wanted name on a colon-less line
        elif u < 0.08:
            hdrs.insert(0, ("Cook:e", "sess=v2"))              # "cookie"'s length, a ':' inside
        elif u < 0.09:
            hdrs += [("X-H", "1")] * 300                      # 300 lines
        elif u < 0.10:
            hdrs.append(("X-Big", "b" * 5000))                 # a 5 KiB value
        elif u < 0.12:
            hdrs += [("Cookie", "k=v")] * 20                   # 20 Cookie lines
        a = "&".join(args[int(t)] for t in rng.integers(0, len(args), int(rng.integers(0, 3))))
        items.append({"host": "sp.example.com", "uri": "/", "args": a, "headers": hdrs})
    v = _both(eng, b, items)
    assert eng.stats()["n_rejected_other"] == 0, eng.rejects()
    got = set(v["match_idx"].tolist())
    assert {0, 1, 2, 3, 0xFF} <= got, got


def test_long_host_names(eng):
    """Hosts of 33..64 bytes take the route's 16-word SWAR path (round 6), longer ones the arena
    bytes: case, a port, a trailing dot, a ".." and a '/' in them, IPv6 literals, lengths 32 / 33 /
    64 / 65 around the boundaries, against the oracle."""
    long_host = "a" * 20 + ".virtual-server.example.com"        # 47 bytes
    edge64 = "b" * 48 + ".example.com.xy"                          # 63 bytes
    ups = [{"name": "u0", "service": "svc0", "port": 80}]
    vss = []
    for k, h in enumerate([long_host, edge64, "c" * 21 + ".example.com"]):   # (the last: 33 bytes)
        vss.append({"metadata": {"name": f"lh{k}", "namespace": "default"},
                    "spec": {"host": h, "upstreams": ups, "routes": [{"path": "/", "upstream": "u0"}]}})
    p = confgen.default_config_params()
    b = blob.make_blob(confgen.render_main(p), confgen.virtual_server_files(vss, base=p, pem_name=""))
    hosts = [long_host, long_host.upper(), long_host + ":8080", long_host + ".", long_host + "..",
             edge64, edge64 + "z", edge64 + "zz", edge64.upper() + ":1", "c" * 21 + ".example.com",
             "c" * 20 + ".example.com", "d" * 40 + "/x.example.com", "e" * 30 + "..example.com",
             "[2001:db8::1]:80" + "f" * 20, "[" + "1" * 40 + "]", "g" * 64, "h" * 65, "x" * 33, ""]
    items = [{"host": h, "uri": "/", "https": bool(i % 2)} for i in range(4) for h in hosts]
    v = _both(eng, b, items)
    assert (v["server_id"] != v["server_id"][-1]).any()


def _peer_pair(e, b, items, gen=4):
    import torch
    dev = torch.device("cuda", 0)
    reqs, arena = records.from_dicts(items)
    e.load(b, gen)
    n_peers = e.stats()["n_peers"]
    st = torch.zeros(max(n_peers, 1) * 16, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    e.peers_init_ptr(st.data_ptr(), n_peers, s)
    n = len(reqs)
    d_r = torch.from_numpy(reqs.view(np.uint8).reshape(-1).copy()).to(dev)
    d_a = torch.zeros(len(arena) + 1024, dtype=torch.uint8, device=dev)
    d_a[:len(arena)].copy_(torch.from_numpy(np.ascontiguousarray(arena)))
    d_o = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_h = torch.empty(4 * n + 1024, dtype=torch.int32, device=dev)
    d_p = torch.empty(n, dtype=torch.int32, device=dev)
    e.match_ptr(d_r.data_ptr(), d_a.data_ptr(), len(arena), n, d_o.data_ptr(), d_h.data_ptr(), 4 * n + 1024, s)
    e.select_peers_ptr(d_r.data_ptr(), d_a.data_ptr(), len(arena), n, d_o.data_ptr(), st.data_ptr(), n_peers,
                       d_p.data_ptr(), s)
    e.sync(s)
    got = d_p.cpu().numpy().view(np.uint32)
    o = Oracle(b, gen)
    ev, _ = o.match(reqs, arena)
    exp = Balancer(o).select(reqs, arena, ev)
    return got, exp


@pytest.mark.parametrize("method", ["ip_hash", "hash $remote_addr$remote_port consistent", "hash $remote_addr"])
def test_realip_balancer_keys_parity(eng, method):
    ing = SC._ingress("lb", "r.example.com", [("/", "svc")], {"nginx.org/lb-method": method})
    p = confgen.default_config_params()
    p.update(SetRealIPFrom=["192.168.0.0/16", "10.1.0.0/16", "2001:db8::/32"], RealIPHeader="X-Forwarded-For",
             RealIPRecursive=True)
    ex = {"Ingress": ing, "Endpoints": {"svc80": ["10.9.0.%d:80" % k for k in range(1, 12)]}}
    cfg = confgen.generate_nginx_cfg(ex, {}, False, p)
    b = blob.make_blob(confgen.render_main(p), {"default-lb": confgen.render_ingress(cfg)})
    got, exp = _peer_pair(eng, b, _rand_requests(20_000, "r.example.com", 5))
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, (method, len(bad), int(bad[0]))
    assert len(set(exp.tolist())) >= 8


def test_wire_chunked_body_limit_gpu(eng):
    """Raw requests through gm_parse_requests (chunked -> GM_REQ_CHUNKED) then gm_match_batch
    against the oracle's parse -> match: Content-Length vs chunked bodies around a 1k limit."""
    import torch
    dev = torch.device("cuda", 0)
    b, _ = SC.body_limit_case()
    msgs, conn = [], []
    for k, size in enumerate([0, 1, 1023, 1024, 1025, 3000]):
        for uri in ("/tea", "/coffee", "/nothing"):
            for ch in (False, True, [size // 2, size - size // 2] if size > 1 else False):
                msgs.append(wire.serialize({"method": "POST", "uri": uri, "host": "cafe.example.com",
                                            "body": b"p" * size, "chunked": ch}))
                conn.append({"https": False, "port": 80})
    W, M = wire.build(msgs, conn)
    eng.load(b, 5)
    n = len(M)
    cap = wire.arena_bound(M)
    d_w = torch.from_numpy(W).to(dev)
    d_m = torch.from_numpy(M.view(np.uint8).reshape(-1).copy()).to(dev)
    d_r = torch.zeros(n * 64 + 16, dtype=torch.uint8, device=dev)
    d_a = torch.zeros(cap + 64, dtype=torch.uint8, device=dev)
    d_len = torch.zeros(1, dtype=torch.int64, device=dev)
    eng.parse_ptr(d_w.data_ptr(), d_m.data_ptr(), n, d_r.data_ptr(), d_a.data_ptr(), cap, d_len.data_ptr(), 0)
    d_o = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_h = torch.empty(4 * n + 1024, dtype=torch.int32, device=dev)
    eng.match_ptr(d_r.data_ptr(), d_a.data_ptr(), cap, n, d_o.data_ptr(), d_h.data_ptr(), d_h.numel(), 0,
                  arena_len_dev=d_len.data_ptr())
    eng.sync(0)
    got = d_o.cpu().numpy().view(records.VERDICT_DTYPE)
    grec = d_r[:n * 64].cpu().numpy().view(records.REQ_DTYPE)
    reqs, arena = parse_requests(W, M)
    assert np.array_equal(grec["flags"], reqs["flags"])
    assert ((reqs["flags"] & records.REQ_CHUNKED) != 0).sum() > 10
    exp, _ = Oracle(b, 5).match(reqs, arena)
    assert_verdicts_equal(got, exp, None, None, "wire chunked")
    assert (exp["action"] == SC.TOO_LARGE).sum() > 5 and (exp["action"] == SC.PROXY).sum() > 5


def test_stock_main_config_gpu(eng):
    """the main config a stock controller renders (nginx.tmpl with its defaults:
    -nginx-status true, port 8080, allow 127.0.0.1, deny all) compiles with 0 rejects, and requests
    to every listener -- the status server's included, from allowed and denied IPv4 / IPv6 / mapped
    clients -- equal the oracle's verdicts on the GPU."""
    from gpumatch import workloads
    b = workloads.c1_blob()
    eng.load(b, 4)
    assert eng.stats()["n_rejected_other"] == 0, eng.rejects()
    rng = np.random.Generator(np.random.PCG64(8080))
    addrs = ["127.0.0.1", "127.0.0.2", "10.0.0.1", "::1", "::ffff:127.0.0.1", "2001:db8::1", "192.168.1.1"]
    items = []
    for i in range(6000):
        k = int(rng.integers(0, 4))
        it = {"raddr": addrs[int(rng.integers(0, len(addrs)))]}
        if k == 0:
            it.update(host="localhost", uri=["/stub_status", "/stub_status/x", "/", "/other"][int(rng.integers(0, 4))],
                      port=8080)
        elif k == 1:
            it.update(host="cafe.example.com", uri=["/tea", "/coffee", "/", "/tea/x"][int(rng.integers(0, 4))],
                      https=bool(rng.random() < 0.5))
        else:
            it.update(host=["nope.example.com", "cafe.example.com"][int(rng.integers(0, 2))], uri="/")
        items.append(it)
    v = _both(eng, b, items, gen=4)
    st = v[[it.get("port") == 8080 for it in items]]
    assert (st["action"] == SC.FORBIDDEN).sum() > 100 and (st["status"] == 200).sum() > 50
