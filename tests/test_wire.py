"""HTTP/1.x wire parser -- the CPU side: the oracle's restatement of nginx's
request intake (oracle/gm_oracle.c orc_parse_one) on known answers, and the serialise -> parse
round trip of the synthetic request mix.  Parity unpinned: no reference test fixes these bytes
(nginx's source is not in /root/reference); the known answers restate nginx 1.17.3's documented
behaviour, listed at orc_parse_one.  The GPU parity test is tests/test_gpu_wire.py."""

import numpy as np
import pytest

from gpumatch import records, wire
from oracle_py import parse_requests

# (message index in wire._EDGE, expected status or the expected fields)
EDGE_KATS = {
    0: 400, 1: 505, 2: 400, 3: 400,
    4: {"method": b"GET", "uri": b"/", "host": b"", "ruri": b"/", "flags": records.REQ_HTTP10},
    5: {"uri": b"/tea", "args": b"x=1", "host": b"Cafe.Example.com", "ruri": b"/tea?x=1", "hdrs": b"Host: other\r\n"},
    6: {"uri": b"/", "host": b"cafe.example.com", "ruri": b"/"},
    7: 400, 8: 400, 9: 400, 10: 400, 11: 501, 12: 400,
    13: {"body": b"ok"},
    14: {"body": b"abcd", "hdrs": b"Host: a\r\nTransfer-Encoding: Chunked\r\nContent-Length: 99\r\n"},
    15: 400, 16: 400,
    17: {"hdrs": b"Host: a\r\nGood-One: v\r\nNoColon: \r\n"},
    18: 400, 19: 400, 20: 400,
    21: {"uri": b"/a/c", "args": b"q=1#f", "ruri": b"//a/./b/%2e%2E/c?q=1#f"},
    22: {"uri": b"/lead", "method": b"GET"},
    23: 400,
    24: {"hdrs": b"Host: a\r\nCookie: u=1\r\nCookie: v=2\r\nX-V: \tt\t\r\n"},
    25: 400, 26: 400, 27: 400, 28: 400,
    29: {"args": b"a=1&b=%zz"},
    30: 414, 31: 400, 32: 400,
    # IP-literal hosts in the absolute form (nginx sw_host_ip_literal)
    44: {"uri": b"/v6", "args": b"x=1", "host": b"[::1]", "ruri": b"/v6?x=1"},
    45: {"uri": b"/", "host": b"[v1.fe80::a+en1]", "ruri": b"/"},
    46: 400, 47: 400, 48: 400,
}


def _status(r):
    return int(r["pad0"][1]) | int(r["pad0"][2]) << 8 if r["flags"] & records.REQ_INVALID else 0


def test_oracle_wire_known_answers():
    W, M = wire.build(wire._EDGE, [{"https": False, "port": 80}] * len(wire._EDGE))
    reqs, arena = parse_requests(W, M)
    for i, exp in EDGE_KATS.items():
        r = reqs[i]
        if isinstance(exp, int):
            assert _status(r) == exp, (i, wire._EDGE[i][:60], _status(r))
            assert r["uri_len"] == 0 and r["hdr_len"] == 0 and records.field_bytes(reqs, arena, i, "raddr")
            continue
        assert _status(r) == 0, (i, _status(r))
        for f, v in exp.items():
            if f == "flags":
                assert r["flags"] & v, i
            else:
                assert records.field_bytes(reqs, arena, i, f) == v, (i, f, records.field_bytes(reqs, arena, i, f))
    assert reqs[33]["hdr_len"] == len(b"Host: a\r\n") + 200 * len(b"X-H: 1\r\n")


def test_serialise_parse_round_trip():
    """records.gen_c2 requests -> HTTP/1.1 bytes -> the oracle's parser: the same fields."""
    reqs, arena = records.gen_c2(3000, seed=5)
    items = []
    for i in range(len(reqs)):
        f = {k: records.field_bytes(reqs, arena, i, k) for k in ("uri", "args", "hdrs", "host", "method")}
        hl = [ln.split(b": ", 1) for ln in f["hdrs"].split(b"\r\n") if ln]
        items.append(wire.serialize({"method": f["method"], "uri": f["uri"], "args": f["args"], "host": f["host"],
                                     "headers": [(k, v) for k, v in hl]}))
    W, M = wire.build(items)
    got, ga = parse_requests(W, M)
    assert not (got["flags"] & records.REQ_INVALID).any()
    for i in range(len(reqs)):
        for f in ("uri", "args", "method", "host"):
            assert records.field_bytes(got, ga, i, f) == records.field_bytes(reqs, arena, i, f), (i, f)
        assert records.field_bytes(got, ga, i, "hdrs") == b"Host: " + records.field_bytes(reqs, arena, i, "host") + \
            b"\r\n" + records.field_bytes(reqs, arena, i, "hdrs")


def test_synthetic_mix_statuses():
    msgs, conn = wire.synthetic(4000)
    W, M = wire.build(msgs, conn)
    reqs, arena = parse_requests(W, M)
    st = np.array([_status(r) for r in reqs])
    assert 0.05 < (st != 0).mean() < 0.3
    assert {400, 501, 505, 414} <= set(st.tolist())
    assert (reqs["body_len"] > 0).sum() > 500
    assert (np.diff(reqs["base"].astype(np.int64)) >= 0).all() and (reqs["base"] % 16 == 0).all()


def test_oracle_proxy_protocol_known_answers():
    """PROXY protocol intake (ngx_proxy_protocol_read, nginx 1.17.3; parity unpinned: nginx is not
    in the reference) on a listener with proxy_protocol (ports 80, 443; 8080 without): the source
    address and port of v1 / v2 headers, UNKNOWN / LOCAL / other transports without an address,
    broken or missing headers closing the connection (444), keep-alive requests carrying the
    connection's address."""
    cases = wire.proxy_cases()
    W, M = wire.build([c[0] for c in cases], [c[1] for c in cases])
    reqs, arena = parse_requests(W, M, proxy_ports=(80, 443))
    for i, (_, _, want) in enumerate(cases):
        r = reqs[i]
        if isinstance(want, int):
            assert _status(r) == want, (i, _status(r))
            assert records.field_bytes(reqs, arena, i, "paddr") == b""
            continue
        assert _status(r) == 0, (i, _status(r))
        assert records.field_bytes(reqs, arena, i, "paddr") == want[0], (i, records.field_bytes(reqs, arena, i, "paddr"))
        if want[0]:
            assert records.proxy_port(r) == want[1], (i, records.proxy_port(r))
        assert records.field_bytes(reqs, arena, i, "uri") == want[2]
        assert records.field_bytes(reqs, arena, i, "raddr") == bytes(M[i]["raddr"][:M[i]["raddr_len"]])
