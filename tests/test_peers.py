"""Upstream peer selection on the CPU: the LBMethod parsing the reference tests
(parsing_helpers_test.go:269-360), the compiler's upstream tables, and the oracle's balancers
against an independent Python restatement (zlib CRC-32, ipaddress) of nginx's ip_hash / hash /
hash consistent / random choices.  The balancers themselves are nginx 1.17.3 behaviour restated
from its published algorithms -- nginx is not in the reference, so the choice is "parity
unpinned" beyond these restatement cross-checks."""

import bisect
import ipaddress
import zlib

import numpy as np
import pytest

from gpumatch import blob, confgen, engine, peers, records
from oracle_py import Balancer, Oracle, crc32

# parsing_helpers_test.go:269-313 (TestParseLBMethod) and :315-360 (TestParseLBMethodForPlus)
LB_VALID = [("least_conn", "least_conn"), ("round_robin", ""), ("ip_hash", "ip_hash"), ("random", "random"),
            ("random two", "random two"), ("random two least_conn", "random two least_conn"),
            ("hash $request_id", "hash $request_id"), ("hash $request_id consistent", "hash $request_id consistent")]
LB_INVALID = ["", "blabla", "least_time header", "hash123", "hash $request_id conwrongspelling", "random one",
              "random two least_time=header", "random two least_time=last_byte", "random two ip_hash"]
LB_VALID_PLUS = [("least_conn", "least_conn"), ("round_robin", ""), ("ip_hash", "ip_hash"), ("random", "random"),
                 ("random two", "random two"), ("random two least_conn", "random two least_conn"),
                 ("random two least_time=header", "random two least_time=header"),
                 ("random two least_time=last_byte", "random two least_time=last_byte"),
                 ("hash $request_id", "hash $request_id"), ("least_time header", "least_time header"),
                 ("least_time last_byte", "least_time last_byte"),
                 ("least_time header inflight", "least_time header inflight"),
                 ("least_time last_byte inflight", "least_time last_byte inflight")]
LB_INVALID_PLUS = ["", "blabla", "hash123", "least_time", "last_byte", "least_time inflight header", "random one",
                   "random two ip_hash", "random two least_time"]


@pytest.mark.parametrize("inp,exp", LB_VALID)
def test_parse_lb_method_valid(inp, exp):
    assert confgen.parse_lb_method(inp) == exp


@pytest.mark.parametrize("inp", LB_INVALID)
def test_parse_lb_method_invalid(inp):
    with pytest.raises(ValueError):
        confgen.parse_lb_method(inp)


@pytest.mark.parametrize("inp,exp", LB_VALID_PLUS)
def test_parse_lb_method_plus_valid(inp, exp):
    assert confgen.parse_lb_method(inp, plus=True) == exp


@pytest.mark.parametrize("inp", LB_INVALID_PLUS)
def test_parse_lb_method_plus_invalid(inp):
    with pytest.raises(ValueError):
        confgen.parse_lb_method(inp, plus=True)


def test_lb_annotations_render_upstream():
    """nginx.org/lb-method, max-fails, fail-timeout and keepalive reach the upstream block
    (annotations.go:60-74,275-293; version1/nginx.ingress.tmpl:2-8); an invalid method keeps the
    ConfigMap's (logged, annotations.go:68-70)."""
    ing = {"metadata": {"name": "cafe", "namespace": "default",
                        "annotations": {"nginx.org/lb-method": "hash $request_uri consistent",
                                        "nginx.org/max-fails": "3", "nginx.org/fail-timeout": "30s",
                                        "nginx.org/keepalive": "16"}},
           "spec": {"rules": [{"host": "cafe.example.com", "http": {"paths": [
               {"path": "/tea", "backend": {"serviceName": "tea-svc", "servicePort": 80}}]}}]}}
    ex = {"Ingress": ing, "Endpoints": {"tea-svc80": ["10.0.0.1:8080", "10.0.0.2:8080"]}}
    cfg = confgen.generate_nginx_cfg(ex, {}, False, confgen.default_config_params())
    text = confgen.render_ingress(cfg)
    assert "hash $request_uri consistent;" in text
    assert "server 10.0.0.1:8080 max_fails=3 fail_timeout=30s;" in text
    assert "keepalive 16;" in text
    ing["metadata"]["annotations"] = {"nginx.org/lb-method": "random one", "nginx.org/max-fails": "x"}
    cfg = confgen.generate_nginx_cfg(ex, {}, False, confgen.default_config_params())
    text = confgen.render_ingress(cfg)
    assert "random two least_conn;" in text and "max_fails=1 " in text


def test_crc32_kat():
    assert crc32(b"123456789") == 0xCBF43926 == zlib.crc32(b"123456789")
    assert crc32(b"") == 0


@pytest.fixture(scope="module")
def pblob():
    return peers.peers_blob()


def test_compiler_peer_tables(pblob):
    e = engine.Engine(compile_only=True)
    e.load(pblob, 3)
    st = e.stats()
    o = Oracle(pblob, 3)
    n_peers = sum(k for _, k in peers.UPSTREAMS) + 2
    assert st["n_peers"] == Balancer(o).n_peers == n_peers
    assert st["n_upstreams"] == len(peers.UPSTREAMS) + 1
    # hash $host, least_time, weight=2
    assert st["n_upstreams_deferred"] == 3
    names = sorted(f"default-peers-u{u:02d}-svc-80" for u in range(len(peers.UPSTREAMS) + 1))
    base = 0
    for uid, name in enumerate(names):
        u = int(name.split("-u")[1][:2])
        k = peers.UPSTREAMS[u][1] if u < len(peers.UPSTREAMS) else 2
        for j in range(k):
            addr, up = e.peer_address(base + j)
            assert up == uid
            if u < len(peers.UPSTREAMS):
                assert addr == peers._addr(u, j)
        base += k
    with pytest.raises(engine.GmError):
        e.peer_address(base)


def _tiny_blob(method, k, down=()):
    servers = "".join(f"\tserver 10.0.0.{j + 1}:80{' down' if j in down else ''};\n" for j in range(k))
    m = f"\t{method};\n" if method else ""
    conf = (f"upstream u {{\n{m}{servers}}}\nserver {{\n\tlisten 80;\n\tserver_name a.example.com;\n"
            f"\tlocation / {{\n\t\tproxy_pass http://u;\n\t}}\n}}\n")
    return blob.make_blob(None, {"t": conf})


def _picks(b, items, batches=1):
    o = Oracle(b, 1)
    bal = Balancer(o)
    out = []
    for _ in range(batches):
        reqs, arena = records.from_dicts(items)
        v, _ = o.match(reqs, arena, nthreads=1)
        out.append(bal.select(reqs, arena, v))
    return np.concatenate(out), bal


def test_round_robin_sequence():
    """Smooth weighted round robin with equal weights: config order, cyclic; down peers skipped."""
    items = [{"host": "a.example.com", "uri": "/"}] * 9
    p, bal = _picks(_tiny_blob("", 3), items)
    assert list(p) == [0, 1, 2] * 3
    assert list(bal.state["conns"]) == [3, 3, 3]
    p, _ = _picks(_tiny_blob("", 4, down={1}), items)
    assert list(p) == [0, 2, 3] * 3


def test_least_conn_sequence():
    """least_conn from an idle upstream: fewest connections, ties broken by the smooth WRR over the
    tied peers (nginx keeps their current_weight): 0 1 2, then 2 1 0, period two rounds."""
    items = [{"host": "a.example.com", "uri": "/"}] * 12
    p, bal = _picks(_tiny_blob("least_conn", 3), items)
    assert list(p) == [0, 1, 2, 2, 1, 0, 0, 1, 2, 2, 1, 0]
    assert list(bal.state["current_weight"]) == [0, 0, 0]
    # a loaded peer is avoided until the others catch up
    o = Oracle(_tiny_blob("least_conn", 3), 1)
    bal = Balancer(o)
    bal.state["conns"][:] = [0, 5, 1]
    reqs, arena = records.from_dicts(items[:7])
    v, _ = o.match(reqs, arena, nthreads=1)
    got = list(bal.select(reqs, arena, v))
    assert got[0] == 0 and got.count(1) == 0 and sorted(got[:3]) == [0, 0, 2]
    assert list(bal.state["conns"]) == [4, 5, 4]


def _py_ip_hash(raddr, n, live):
    try:
        a = ipaddress.ip_address(raddr)
        b, alen = a.packed, (3 if a.version == 4 else 16)
    except ValueError:
        b, alen = bytes(3), 3
    h = 89
    for _ in range(21):
        for i in range(alen):
            h = (h * 113 + b[i]) % 6271
        if live[h % n]:
            return h % n
    return None


def _py_hash(key, n, live):
    acc = 0
    for t in range(21):
        acc += (zlib.crc32((str(t).encode() if t else b"") + key) >> 16) & 0x7FFF
        if live[acc % n]:
            return acc % n
    return None


def _py_ring(addrs):
    pts = []
    for j, a in enumerate(addrs):
        host, port = a, ""
        if a[:5].lower() == "unix:":
            host = a[5:]
        else:
            for q in range(len(a) - 1, -1, -1):
                if a[q] == ":":
                    host, port = a[:q], a[q + 1:]
                    break
                if not a[q].isdigit():
                    break
        base = host.encode() + b"\0" + port.encode()
        prev = 0
        for _ in range(160):
            h = zlib.crc32(base + prev.to_bytes(4, "little"))
            pts.append((h, j))
            prev = h
    pts.sort()
    ring = []
    for h, j in pts:
        if not ring or ring[-1][0] != h:
            ring.append((h, j))
    return ring


def _py_chash(key, ring, live):
    i = bisect.bisect_left([h for h, _ in ring], zlib.crc32(key))
    for t in range(21):
        j = ring[(i + t) % len(ring)][1]
        if live[j]:
            return j
    return None


def _py_draw(rid, j):
    M = (1 << 64) - 1
    lo = int.from_bytes(rid[:8], "little")
    hi = int.from_bytes(rid[8:], "little")
    x = lo ^ ((hi * 0x9E3779B97F4A7C15) & M) ^ (((j + 1) * 0xD1B54A32D192ED03) & M)
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & M
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & M
    x ^= x >> 31
    return x >> 32


def test_stateless_methods_match_python_restatement(pblob):
    """The oracle's ip_hash / hash / hash consistent / random picks over the peers workload equal an
    independent Python restatement (round-robin fallbacks excluded)."""
    reqs, arena = peers.gen_requests(6000, seed=records.SEED_BASE + 41)
    o = Oracle(pblob, 1)
    bal = Balancer(o)
    v, _ = o.match(reqs, arena, nthreads=4)
    got = bal.select(reqs, arena, v)
    names = sorted(f"default-peers-u{u:02d}-svc-80" for u in range(len(peers.UPSTREAMS) + 1))
    first, base = {}, 0
    for name in names:
        u = int(name.split("-u")[1][:2])
        first[u] = base
        base += peers.UPSTREAMS[u][1] if u < len(peers.UPSTREAMS) else 2
    rings = {}
    checked = {m: 0 for m in ("ip_hash", "hash", "chash", "random")}
    for i in range(len(reqs)):
        if v["action"][i] != 0:
            continue
        u = int(records.field_bytes(reqs, arena, i, "host").split(b".")[0][1:])
        if u >= len(peers.UPSTREAMS):
            assert got[i] == engine.GM_PEER_DEFER
            continue
        m, k = peers.UPSTREAMS[u]
        live = [(u, j) not in peers.DOWN for j in range(k)]
        args = records.field_bytes(reqs, arena, i, "args").decode()
        hdrs = records.field_bytes(reqs, arena, i, "hdrs").decode()
        raddr = records.field_bytes(reqs, arena, i, "raddr").decode()
        exp = "skip"
        if k == 1:
            continue
        if m == "ip_hash":
            try:
                ipaddress.ip_address(raddr)
            except ValueError:
                continue   # inet_pton vs ipaddress corner forms: covered by the GPU parity test
            exp, kind = _py_ip_hash(raddr, k, live), "ip_hash"
        elif m == "hash $request_uri":
            ruri = records.field_bytes(reqs, arena, i, "uri") + (b"?" + args.encode() if args else b"")
            exp, kind = _py_hash(ruri, k, live), "hash"
        elif m == "hash $arg_user consistent":
            user = dict(kv.split("=", 1) for kv in args.split("&") if "=" in kv).get("user", "")
            if not user:
                continue
            ring = rings.setdefault(u, _py_ring([peers._addr(u, j) for j in range(k)]))
            exp, kind = _py_chash(user.encode(), ring, live), "chash"
        elif m == "random":
            rid = bytes(reqs["rid"][i])
            for t in range(21):
                x = _py_draw(rid, t) % k
                if live[x]:
                    exp = x
                    break
            kind = "random"
        if exp == "skip" or exp is None:
            continue
        assert got[i] == first[u] + exp, (i, m, raddr, args, hdrs)
        checked[kind] += 1
    assert all(c > 50 for c in checked.values()), checked


def test_oracle_state_accounting(pblob):
    """conns grow by the batch's picks; released connections come off; state carries over."""
    reqs, arena = peers.gen_requests(3000, seed=records.SEED_BASE + 42)
    o = Oracle(pblob, 1)
    bal = Balancer(o)
    v, _ = o.match(reqs, arena, nthreads=4)
    p1 = bal.select(reqs, arena, v)
    real = p1[p1 < bal.n_peers]
    assert int(bal.state["conns"].sum()) == len(real)
    assert np.array_equal(np.bincount(real, minlength=bal.n_peers), bal.state["conns"])
    bal.release(real[:1000])
    assert int(bal.state["conns"].sum()) == len(real) - 1000
    down = bal.state["flags"] & engine.GM_PEER_DOWN
    assert not np.any(np.isin(real, np.nonzero(down)[0]))


# ---------------------------------------------------------------- NGINX Plus endpoint updates
# Configurator.UpdateEndpoints* push servers through Manager.UpdateServersInPlus with no reload
# (configurator.go:442,467,489; manager.go:257-284): gm_update_upstream patches the live tables'
# upstream section.  Its peer tables must equal a fresh compile of the config a reload with the
# new server lines would have rendered, in NGINX Plus's order (peers.plus_order: kept servers first).
def _addresses(e):
    st = e.stats()
    return [e.peer_address(p) for p in range(st["n_peers"])]


@pytest.mark.parametrize("u,servers", [
    (1, [peers._addr(1, j) for j in range(5, 55)] + [f"10.77.0.{j}:9000" for j in range(1, 21)]),   # RR 70 -> 70
    (9, [peers._addr(9, j) for j in (6, 0, 2)] + ["10.9.9.9:80"]),                                 # chash 7 -> 4
    (9, ["10.9.9.9:80", "10.9.9.9:80"]),                       # chash naming one address twice: deferred
    (4, [f"10.4.1.{j}:8080" for j in range(1, 1100)]),          # least_conn past SEQ_PEERS_MAX: deferred
    (2, []),                                                     # every server removed
])
def test_update_upstream_equals_fresh_compile(pblob, u, servers):
    e = engine.Engine(compile_only=True)
    e.load(pblob, 4)
    e.update_upstream(peers.upstream_name(u), servers)
    f = engine.Engine(compile_only=True)
    f.load(peers.peers_blob(servers={u: peers.plus_order(peers.server_addrs(u), servers)}), 4)
    se, sf = e.stats(), f.stats()
    for k in ("gen", "n_peers", "n_upstreams", "n_upstreams_deferred", "n_counters", "n_locations"):
        assert se[k] == sf[k], k
    assert _addresses(e) == _addresses(f)


def test_plus_order():
    assert peers.plus_order(["a", "b", "c"], ["d", "c", "a"]) == ["a", "c", "d"]
    assert peers.plus_order(["a", "b"], ["b", "b", "e"]) == ["b", "b", "e"]
    assert peers.plus_order(["a"], []) == []


def test_update_upstream_unknown_name(pblob):
    e = engine.Engine(compile_only=True)
    e.load(pblob, 4)
    n0 = e.stats()["n_peers"]
    with pytest.raises(engine.GmError):
        e.update_upstream("no-such-upstream", ["10.0.0.1:80"])
    assert e.stats()["n_peers"] == n0   # the live tables stay


def test_update_upstream_racing_a_load_is_refused(pblob):
    """a gm_load_generation that publishes between gm_update_upstream's read of the live
    tables and its publish must not be undone -- the update fails GM_E_STALE (the reference's
    verifyConfigVersion refusal, manager.go:258) and the loaded generation stays live."""
    import ctypes
    e = engine.Engine(compile_only=True)
    e.load(pblob, 4)
    other = peers.peers_blob(servers={1: ["10.55.0.1:80", "10.55.0.2:80"]})
    L = engine.lib()
    calls = []

    @ctypes.CFUNCTYPE(None, ctypes.c_void_p)
    def hook(_arg):
        if not calls:
            calls.append(1)
            e.load(other, 5)
    L.gm_debug_update_hook.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.gm_debug_update_hook(ctypes.cast(hook, ctypes.c_void_p), None)
    try:
        with pytest.raises(engine.GmError) as ei:
            e.update_upstream(peers.upstream_name(9), ["10.9.9.9:80"])
        assert ei.value.code == engine.GM_E_STALE
        f = engine.Engine(compile_only=True)
        f.load(other, 5)
        assert e.stats()["gen"] == 5
        assert _addresses(e) == _addresses(f)   # the reload's tables, not the stale update's
        # re-issued against the new generation, the update goes through
        e.update_upstream(peers.upstream_name(9), ["10.9.9.9:80"])
        assert e.stats()["gen"] == 5
        assert [a for a, _ in _addresses(e)].count("10.9.9.9:80") == 1
    finally:
        L.gm_debug_update_hook(None, None)


def test_parse_sticky_service_kats():
    """annotations_test.go:44-62 (parseStickyService): a valid and an invalid declaration."""
    from gpumatch import confgen
    assert confgen.parse_sticky_service("serviceName=coffee-svc srv_id expires=1h domain=.example.com path=/") == \
        ("coffee-svc", "srv_id expires=1h domain=.example.com path=/")
    with pytest.raises(ValueError):
        confgen.parse_sticky_service("serviceNamecoffee-svc srv_id expires=1h domain=.example.com path=/")


def test_sticky_cookie_compiles_and_oracle_picks():
    """NGINX Plus `sticky cookie` (nginx-plus.ingress.tmpl:9-11): the compiler keeps the upstreams
    (none deferred), and the oracle sends a request whose cookie is the hex MD5 (hashlib) of a live
    peer's address to that peer; a down peer, a stale / uppercase / short value or another
    upstream's cookie leaves the request to the balancing method.  Parity unpinned (no Plus)."""
    import hashlib
    from gpumatch import confgen
    b = peers.sticky_blob()
    ings, _ = peers.sticky_ingresses()
    txt = confgen.ingress_files(ings[:1], endpoints={"svc-080": peers.sticky_endpoints(0)}, is_plus=True)
    assert "sticky cookie srv_0 expires=1h path=/;" in "".join(txt.values())
    e = engine.Engine(compile_only=True)
    e.load(b, 1)
    st = e.stats()
    assert st["n_upstreams_deferred"] == 0 and st["n_rejected_other"] == 0, e.rejects()
    o = Oracle(b, 1)
    bal = Balancer(o)
    reqs, arena = peers.sticky_requests(3000)
    v, _ = o.match(reqs, arena)
    state = bal.state
    down = {int(x) for x in np.nonzero(np.arange(len(state)) % 7 == 3)[0]}
    state["flags"][sorted(down)] = 1
    picks = bal.select(reqs, arena, v)
    names = [e.peer_address(j)[0] for j in range(len(state))]
    hits = 0
    for i in range(len(reqs)):
        hd = records.field_bytes(reqs, arena, i, "hdrs").decode()
        host = records.field_bytes(reqs, arena, i, "host").decode()
        k = int(host[1])
        uri = records.field_bytes(reqs, arena, i, "uri").decode()
        ck = [c.split("=", 1)[1] for c in hd.replace("Cookie: ", "").replace("\r\n", "").split("; ")
              if c.startswith(f"srv_{k}=")]
        if uri != "/" or not ck:
            continue
        want = [j for j in range(len(state)) if names[j] in peers.sticky_endpoints(k) and
                hashlib.md5(names[j].encode()).hexdigest() == ck[0] and j not in down]
        if want:
            assert picks[i] == want[0], (i, hd, picks[i], want)
            hits += 1
    assert hits > 400
