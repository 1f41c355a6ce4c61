"""HTTP/1.x wire parser on the GPU (gm_parse_requests) against the oracle's
restatement of nginx's intake (oracle/gm_oracle.c orc_parse_one): the same records (status,
flags, lengths, connection fields) and the same field bytes; then the whole data-plane chain
raw bytes -> gm_parse_requests -> gm_match_batch (arena length handed over on the device, no
host round trip) against oracle parse -> oracle match.  Parity unpinned (nginx's parser is not in
the reference); the known answers are tests/test_wire.py's."""

import numpy as np
import pytest

from gpumatch import engine, records, wire, workloads
from helpers import assert_verdicts_equal
from oracle_py import Oracle, parse_requests

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    return torch, torch.device("cuda", 0), engine.Engine(0)


def _gpu_parse(torch, dev, e, W, M, stream=0, cap=None):
    n = len(M)
    cap = wire.arena_bound(M) if cap is None else cap
    d_w = torch.from_numpy(W).to(dev)
    d_m = torch.from_numpy(M.view(np.uint8).reshape(-1).copy()).to(dev)
    d_r = torch.zeros(n * 64 + 16, dtype=torch.uint8, device=dev)
    d_a = torch.full((cap + 64,), 0xAB, dtype=torch.uint8, device=dev)   # garbage: the parser zero-fills slack
    d_len = torch.zeros(1, dtype=torch.int64, device=dev)
    e.parse_ptr(d_w.data_ptr(), d_m.data_ptr(), n, d_r.data_ptr(), d_a.data_ptr(), cap, d_len.data_ptr(), stream)
    return d_w, d_m, d_r, d_a, d_len, cap


def test_gpu_parse_arena_overflow(env):
    """An arena smaller than the records need: gm_sync reports GM_E_OVERFLOW, nothing is written
    past the capacity, and every record stays inside it (the void batch's layout is legal)."""
    torch, dev, e = env
    msgs, conn = wire.synthetic(3_000, seed=7)
    W, M = wire.build(msgs, conn)
    full = wire.arena_bound(M)
    cap = (full // 3) & ~15
    d_w, d_m, d_r, d_a, d_len, cap = _gpu_parse(torch, dev, e, W, M, cap=cap)
    with pytest.raises(engine.GmError) as ei:
        e.sync(0)
    assert ei.value.code == engine.GM_E_OVERFLOW
    a = d_a.cpu().numpy()
    assert (a[cap:] == 0xAB).all()
    got = d_r[:len(M) * 64].cpu().numpy().view(records.REQ_DTYPE)
    assert int(d_len.item()) <= cap
    assert (got["base"].astype(np.int64) <= cap).all()


def _fields(reqs, arena):
    out = {}
    for f in records.WIRE_FIELDS:
        out[f] = b"".join(records.field_bytes(reqs, arena, i, f) for i in range(len(reqs)))
    return out


def test_gpu_parse_matches_oracle(env):
    torch, dev, e = env
    msgs, conn = wire.synthetic(12_000, seed=99)
    msgs = list(wire._EDGE) + msgs
    conn = [{"https": False, "port": 80}] * len(wire._EDGE) + conn
    W, M = wire.build(msgs, conn)
    d_w, d_m, d_r, d_a, d_len, cap = _gpu_parse(torch, dev, e, W, M)
    e.sync(0)
    n = len(M)
    got = d_r[:n * 64].cpu().numpy().view(records.REQ_DTYPE)
    alen = int(d_len.item())
    ga = d_a[:alen].cpu().numpy()
    exp, ea = parse_requests(W, M)
    for f in ("flags", "pad0", "pad1", "uri_len", "args_len", "hdr_len", "body_len", "host_len", "method_len",
              "ruri_len", "raddr_len", "port", "remote_port", "rid"):
        bad = np.nonzero((got[f] != exp[f]).reshape(n, -1).any(axis=1))[0]
        assert len(bad) == 0, (f, int(bad[0]), msgs[int(bad[0])][:120], got[int(bad[0])], exp[int(bad[0])])
    assert (got["base"] % 16 == 0).all() and (np.diff(got["base"].astype(np.int64)) >= 0).all()
    gf, ef = _fields(got, ga), _fields(exp, ea)
    for f in records.WIRE_FIELDS:
        assert gf[f] == ef[f], f
    # the arena between and after the records is zero (slack is cleared: the WAF scan reads it all)
    used = np.zeros(alen, bool)
    for r in got:
        tot = sum(records.field_len(r, f) for f in records.WIRE_FIELDS)
        used[int(r["base"]):int(r["base"]) + tot] = True
    assert not ga[~used].any()
    assert (got["flags"] & records.REQ_INVALID).sum() > 100


@pytest.mark.parametrize("cfg", ["c2", "c4"])
def test_parse_then_match_chain(env, cfg):
    """raw bytes -> parse -> match on one stream (arena length on the device) == oracle chain."""
    torch, dev, e = env
    msgs, conn = wire.synthetic(20_000, seed=123)
    if cfg == "c4":
        ss = workloads.c4_sigset(800, 200)
        blob = workloads.c4_blob(ss, "block")
        # plant signatures into some bodies so the WAF layer has hits
        rng = np.random.Generator(np.random.PCG64(5))
        ex = [r.example for r in ss.rules if r.example is not None and r.kind == "lit" and "b" in r.zones]
        for i in range(0, len(msgs), 7):
            body = ex[int(rng.integers(0, len(ex)))]
            msgs[i] = wire.serialize({"method": "POST", "uri": "/tea/x", "host": "cafe.example.com", "body": body,
                                      "chunked": bool(i % 2)})
    else:
        blob = workloads.c2_blob()
    W, M = wire.build(msgs, conn)
    e.load(blob, 3)
    s = torch.cuda.Stream(device=dev)
    d_w, d_m, d_r, d_a, d_len, cap = _gpu_parse(torch, dev, e, W, M, s.cuda_stream)
    n = len(M)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_h = torch.empty(4 * n + 1024, dtype=torch.int32, device=dev)
    e.match_ptr(d_r.data_ptr(), d_a.data_ptr(), cap, n, d_out.data_ptr(), d_h.data_ptr(), d_h.numel(), s.cuda_stream,
                arena_len_dev=d_len.data_ptr())
    e.sync(s.cuda_stream)
    total = e.stats()["last_hits"]
    got = d_out.cpu().numpy().view(records.VERDICT_DTYPE)
    gh = d_h[:total].cpu().numpy().view(np.uint32)
    reqs, arena = parse_requests(W, M)
    exp, eh = Oracle(blob, 3).match(reqs, arena)
    assert_verdicts_equal(got, exp, gh, eh, f"wire chain {cfg}")
    assert (exp["action"] == 5).sum() > 100                       # rejected requests: BAD_REQUEST + status
    assert {400, 501, 505} <= set(exp["status"][exp["action"] == 5].tolist())
    if cfg == "c4":
        assert (exp["action"] == 6).sum() > 1000
    else:
        assert (exp["route_kind"] == 3).any() and (exp["match_idx"] != 0xFF).any()


def _proxy_blob():
    """the reference's `basic` VirtualServer with examples/proxy-protocol's ConfigMap (below)"""
    from helpers import golden
    from gpumatch import blob, confgen
    from semantics_cases import ADDRS, _rules_vs
    case = golden("reference_configs.json")["vs_configs"]["basic"]
    p = confgen.default_config_params()
    p.update(case["params"])
    p = confgen.configmap_params({"proxy-protocol": "True", "real-ip-header": "proxy_protocol",
                                  "set-real-ip-from": "192.168.192.168"}, p)
    store = {"%s/%s" % (x["metadata"]["namespace"], x["metadata"]["name"]): x for x in case["vsrs"]}
    files = confgen.virtual_server_files([case["vs"], _rules_vs("pp.example.com", {"variable": "$remote_addr"}, ADDRS)],
                                         base=p, vsr_store=store, pem_name="",
                                         endpoints_of=lambda ns, s_, port: case["endpoints"].get(f"{ns}/{s_}:{port}", []))
    return blob.make_blob(confgen.render_main(p), files)


def test_gpu_parse_fits_the_documented_bound(env):
    """gm_parse_requests' documented arena bound (include/gpumatch.h) is the sum over
    requests of align16(2 * len + raddr_len + 46) -- a record also carries $proxy_protocol_addr (up
    to 46 B) after raddr.  Keep-alive requests of PROXY connections (GM_WIRE_PROXY_DONE) with the
    longest raddr and an IPv6 paddr, in an arena of exactly that size: no overflow, the oracle's
    records."""
    torch, dev, e = env
    b = _proxy_blob()
    e.load(b, 9)
    orc = Oracle(b, 9)
    raddr = "2001:0db8:85a3:0000:0000:8a2e:0370:7334"   # 39 B (the field holds up to 40)
    msgs, conn = [], []
    for i in range(3000):
        msgs.append(b"GET / HTTP/1.0\r\n\r\n" if i % 3 else b"GET /tea HTTP/1.0\r\n\r\n")
        conn.append({"proxy_done": True, "paddr": "2001:db8:ffff:ffff:ffff:ffff:ffff:%04x" % i, "proxy_port": 4000 + i,
                     "raddr": raddr + "0", "port": 80})
    W, M = wire.build(msgs, conn, seed=3)
    bound = int((((2 * M["len"].astype(np.int64) + M["raddr_len"] + 46) + 15) & ~15).sum())
    d_w, d_m, d_r, d_a, d_len, cap = _gpu_parse(torch, dev, e, W, M, cap=bound)
    e.sync(0)   # no GM_E_OVERFLOW
    n = len(M)
    got = d_r[:n * 64].cpu().numpy().view(records.REQ_DTYPE)
    assert int(d_len.item()) <= bound
    exp, ea = parse_requests(W, M, proxy_ports=orc.proxy_ports())
    ga = d_a[:int(d_len.item())].cpu().numpy()
    gf, ef = _fields(got, ga), _fields(exp, ea)
    for f in records.WIRE_FIELDS:
        assert gf[f] == ef[f], f
    assert (got["pad0"][:, 0] >= 38).all() and (got["raddr_len"] == 40).all()


def test_gpu_proxy_protocol_parity(env):
    """PROXY protocol on the GPU: the reference's `basic` VirtualServer fixture
    (virtualserver_test.go:163-282, ProxyProtocol true) with examples/proxy-protocol's ConfigMap
    (proxy-protocol True, real-ip-header proxy_protocol, set-real-ip-from 192.168.192.168), plus a
    rules route on $remote_addr.  gm_parse_requests on PROXY v1 / v2 / broken / keep-alive
    messages equals the oracle's parse (records, $proxy_protocol_addr bytes), and parse -> match
    equals the oracle's chain: realip takes the PROXY source address on the trusted balancer's
    connections only.  Parity unpinned (no nginx in the reference)."""
    import torch
    from helpers import golden
    from gpumatch import blob, confgen
    from semantics_cases import ADDRS, _rules_vs
    torch_, dev, e = env
    case = golden("reference_configs.json")["vs_configs"]["basic"]
    p = confgen.default_config_params()
    p.update(case["params"])
    p = confgen.configmap_params({"proxy-protocol": "True", "real-ip-header": "proxy_protocol",
                                  "set-real-ip-from": "192.168.192.168"}, p)
    store = {"%s/%s" % (x["metadata"]["namespace"], x["metadata"]["name"]): x for x in case["vsrs"]}
    files = confgen.virtual_server_files([case["vs"], _rules_vs("pp.example.com", {"variable": "$remote_addr"}, ADDRS)],
                                         base=p, vsr_store=store, pem_name="",
                                         endpoints_of=lambda ns, s_, port: case["endpoints"].get(f"{ns}/{s_}:{port}", []))
    b = blob.make_blob(confgen.render_main(p), files)
    orc = Oracle(b, 9)
    assert sorted(orc.proxy_ports()) == [80, 443]
    e.load(b, 9)
    assert e.stats()["n_rejected_other"] == 0, e.rejects()
    # the KAT messages, then a seeded mix: v1 / v2 headers with ADDRS and random sources, trusted
    # (the balancer 192.168.192.168) and untrusted peers, keep-alive requests, TLS and plain
    cases = wire.proxy_cases()
    msgs, conn = [c[0] for c in cases], [c[1] for c in cases]
    rng = np.random.Generator(np.random.PCG64(515))
    for i in range(4000):
        src = ADDRS[i % 4] if rng.random() < 0.5 else "%d.%d.%d.%d" % tuple(int(x) for x in rng.integers(0, 256, 4))
        sport = int(rng.integers(0, 65536))
        host = ["pp.example.com", "cafe.example.com"][int(rng.integers(0, 2))]
        req = wire.serialize({"uri": ["/", "/tea", "/coffee", "/x"][int(rng.integers(0, 4))], "host": host})
        https = bool(rng.random() < 0.5)
        peer = "192.168.192.168" if rng.random() < 0.7 else "10.1.2.3"
        k = int(rng.integers(0, 10))
        if k < 4:
            m = wire.proxy_v1(src, "10.0.0.1", sport, 443 if https else 80) + req
            c = {}
        elif k < 8:
            m = wire.proxy_v2(src, "10.0.0.1", sport, 443 if https else 80) + req
            c = {}
        elif k == 8:
            m = req
            c = {"proxy_done": True, "paddr": src, "proxy_port": sport}
        else:
            m = bytes(wire.proxy_v1(src, "10.0.0.1", sport))[:int(rng.integers(1, 30))] + req   # broken
            c = {}
        c.update({"https": https, "port": 443 if https else 80, "raddr": peer})
        msgs.append(m)
        conn.append(c)
    W, M = wire.build(msgs, conn, seed=7)
    d_w, d_m, d_r, d_a, d_len, cap = _gpu_parse(torch_, dev, e, W, M)
    n = len(M)
    d_v = torch_.zeros(n * 32, dtype=torch_.uint8, device=dev)
    d_h = torch_.zeros(4 * n + 1024, dtype=torch_.int32, device=dev)
    e.match_ptr(d_r.data_ptr(), d_a.data_ptr(), cap, n, d_v.data_ptr(), d_h.data_ptr(), d_h.numel(), 0,
                arena_len_dev=d_len.data_ptr())
    e.sync(0)
    got = d_r[:n * 64].cpu().numpy().view(records.REQ_DTYPE)
    alen = int(d_len.item())
    ga = d_a[:alen].cpu().numpy()
    exp, ea = parse_requests(W, M, proxy_ports=orc.proxy_ports())
    for f in ("flags", "pad0", "pad1", "uri_len", "args_len", "hdr_len", "body_len", "host_len", "method_len",
              "ruri_len", "raddr_len", "port", "remote_port"):
        bad = np.nonzero((got[f] != exp[f]).reshape(n, -1).any(axis=1))[0]
        assert len(bad) == 0, (f, int(bad[0]), msgs[int(bad[0])][:120], got[int(bad[0])], exp[int(bad[0])])
    gf, ef = _fields(got, ga), _fields(exp, ea)
    for f in records.WIRE_FIELDS:
        assert gf[f] == ef[f], f
    st = (got["flags"] & records.REQ_INVALID) != 0
    assert (got["pad0"][:, 0] > 0).sum() > 2000 and st.sum() > 300
    ev, eh = orc.match(exp, ea)
    gv = d_v.cpu().numpy().view(records.VERDICT_DTYPE)
    assert_verdicts_equal(gv, ev, None, None, "PROXY protocol parse -> match")
    # realip took effect: trusted connections route on the PROXY source
    pp_rules = (gv["route_kind"] == 3) & (gv["match_idx"] != 0xFF)
    assert pp_rules.sum() > 100   # (227 on the seeded mix)
