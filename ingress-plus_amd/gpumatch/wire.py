"""HTTP/1.x wire bytes for the parser: ``gm_wire_msg`` descriptors and raw
request bytes, from request dicts (the same keys as ``records.from_dicts``) or from a seeded
synthetic mix that exercises nginx's intake rules (oracle/gm_oracle.c orc_parse_one).

Host tooling: tests and benches build inputs with it; the device parses them
(``Engine.parse_ptr`` -> gm_parse_requests)."""

from __future__ import annotations

import numpy as np

from . import records

WIRE_MSG_DTYPE = np.dtype([
    ("off", "<u8"), ("len", "<u4"), ("port", "<u2"), ("remote_port", "<u2"), ("flags", "u1"),
    ("raddr_len", "u1"), ("paddr_len", "u1"), ("pad", "u1"), ("rid", "u1", (16,)), ("raddr", "u1", (40,)),
    ("proxy_port", "<u2"), ("pad2", "u1", (2,)), ("paddr", "u1", (46,)), ("pad3", "u1", (2,)),
])
assert WIRE_MSG_DTYPE.itemsize == 128
WIRE_PROXY_DONE = 0x40   # a keep-alive request of a proxy_protocol connection (gpumatch.h)


def proxy_v1(src: str, dst: str = "10.0.0.1", sport: int = 51234, dport: int = 443, fam: str | None = None) -> bytes:
    """A PROXY protocol v1 header line ("PROXY TCP4 src dst sport dport\\r\\n")."""
    fam = fam or ("TCP6" if ":" in src else "TCP4")
    return f"PROXY {fam} {src} {dst} {sport} {dport}\r\n".encode()


def proxy_v2(src: str, dst: str = "10.0.0.1", sport: int = 51234, dport: int = 443, command: int = 1,
             transport: int = 1, tlv: bytes = b"") -> bytes:
    """A PROXY protocol v2 header (binary): signature, version 2 | command, family | transport, length,
    the addresses and ports, then optional TLV bytes."""
    import ipaddress
    a, d = ipaddress.ip_address(src), ipaddress.ip_address(dst)
    fam = 1 if a.version == 4 else 2
    body = a.packed + d.packed + sport.to_bytes(2, "big") + dport.to_bytes(2, "big") + tlv
    return (b"\r\n\r\n\x00\r\nQUIT\n" + bytes([0x20 | command, fam << 4 | transport]) +
            len(body).to_bytes(2, "big") + body)


def _b(x):
    return x.encode() if isinstance(x, str) else bytes(x)


def serialize(it: dict) -> bytes:
    """One request dict -> HTTP/1.1 bytes.  Keys: method, uri, args, headers, body, host (None:
    no Host line), version ("1.1"), chunked (list of chunk sizes or True), target (raw request
    target, overrides uri/args), raw (the whole message, overrides everything)."""
    if "raw" in it:
        return _b(it["raw"])
    target = _b(it["target"]) if "target" in it else _b(it.get("uri", "/")) + (
        b"?" + _b(it["args"]) if it.get("args") else b"")
    ver = it.get("version", "1.1")
    lines = [_b(it.get("method", "GET")) + b" " + target + (b" HTTP/" + _b(ver) if ver else b"")]
    host = it.get("host", "cafe.example.com")
    if host is not None:
        lines.append(b"Host: " + _b(host))
    for k, v in it.get("headers", []):
        lines.append(_b(k) + b": " + _b(v))
    body = _b(it.get("body", b""))
    ch = it.get("chunked")
    if ch:
        lines.append(b"Transfer-Encoding: chunked")
        sizes = ch if isinstance(ch, list) else [len(body)] if body else []
        out, pos = b"", 0
        for s in sizes:
            out += b"%x\r\n" % s + body[pos:pos + s] + b"\r\n"
            pos += s
        body = out + b"0\r\n\r\n"
    elif body or it.get("content_length") is not None:
        lines.append(b"Content-Length: " + _b(str(it.get("content_length", len(body)))))
    return b"\r\n".join(lines) + b"\r\n\r\n" + body


def build(messages, conn=None, seed=0, align=1):
    """Raw messages -> (wire bytes as a uint8 array, WIRE_MSG_DTYPE descriptors).  ``conn``: per
    message dicts with port / https / raddr / remote_port / rid; defaults: port 443 + TLS."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n = len(messages)
    msgs = np.zeros(n, dtype=WIRE_MSG_DTYPE)
    parts, off = [], 0
    for i, m in enumerate(messages):
        m = _b(m)
        pad = (-off) % align
        if pad:
            parts.append(b"\0" * pad)
            off += pad
        msgs[i]["off"] = off
        msgs[i]["len"] = len(m)
        parts.append(m)
        off += len(m)
        c = (conn[i] if conn is not None else None) or {}
        https = c.get("https", True)
        msgs[i]["port"] = c.get("port", 443 if https else 80)
        msgs[i]["flags"] = records.REQ_HTTPS if https else 0
        msgs[i]["remote_port"] = c.get("remote_port", 40000 + i % 20000)
        ra = _b(c.get("raddr", "10.0.%d.%d" % ((i >> 8) & 255, i & 255)))[:40]
        msgs[i]["raddr_len"] = len(ra)
        msgs[i]["raddr"][:len(ra)] = np.frombuffer(ra, np.uint8)
        rid = c.get("rid")
        msgs[i]["rid"] = np.frombuffer(rid, np.uint8) if rid is not None else rng.integers(0, 256, 16, dtype=np.uint8)
        if c.get("proxy_done"):   # a keep-alive request: the connection's PROXY address, from the caller
            msgs[i]["flags"] |= WIRE_PROXY_DONE
            pa = _b(c.get("paddr", b""))[:46]
            msgs[i]["paddr_len"] = len(pa)
            msgs[i]["paddr"][:len(pa)] = np.frombuffer(pa, np.uint8)
            msgs[i]["proxy_port"] = c.get("proxy_port", 0)
    wire = np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8).copy()
    return wire, msgs


def arena_bound(msgs) -> int:
    """The arena capacity gm_parse_requests always fits in: sum of align16(2 * len + raddr_len + 46)."""
    return int((((2 * msgs["len"].astype(np.int64) + msgs["raddr_len"] + 46) + 15) & ~15).sum()) + 16


# ---------------------------------------------------------------- synthetic mix
_EDGE = [
    b"get / HTTP/1.1\r\nHost: a\r\n\r\n",                                 # lowercase method: 400
    b"GET / HTTP/2.0\r\nHost: a\r\n\r\n",                                 # 505
    b"GET /\r\n\r\n",                                                       # HTTP/0.9: 400 (divergence)
    b"GET / HTTP/1.1\r\n\r\n",                                              # 1.1 without Host: 400
    b"GET / HTTP/1.0\r\n\r\n",                                              # 1.0 without Host: ok
    b"GET http://Cafe.Example.com:8080/tea?x=1 HTTP/1.1\r\nHost: other\r\n\r\n",   # absolute-form
    b"GET http://cafe.example.com HTTP/1.0\r\n\r\n",                        # absolute, no path
    b"GET / HTTP/1.1\r\nHost: a\r\nHost: b\r\n\r\n",                        # duplicate Host: 400
    b"POST /x HTTP/1.1\r\nHost: a\r\nContent-Length: 3\r\nContent-Length: 3\r\n\r\nabc",   # dup CL
    b"POST /x HTTP/1.1\r\nHost: a\r\nContent-Length: 3x\r\n\r\nabc",       # bad CL: 400
    b"POST /x HTTP/1.1\r\nHost: a\r\nContent-Length: 10\r\n\r\nabc",       # short body: 400
    b"POST /x HTTP/1.1\r\nHost: a\r\nTransfer-Encoding: gzip\r\n\r\n",      # 501
    b"POST /x HTTP/1.1\r\nHost: a\r\nTransfer-Encoding: gzip\r\nHost: b\r\n\r\n",   # 400 before 501
    b"POST /x HTTP/1.1\r\nHost: a\r\nTransfer-Encoding: identity\r\nContent-Length: 2\r\n\r\nok",
    b"POST /x HTTP/1.1\r\nHost: a\r\nTransfer-Encoding: Chunked\r\nContent-Length: 99\r\n\r\n"
    b"3;ext=1\r\nabc\r\n1\nd\r\n0\r\nX-Trailer: 1\r\n\r\n",                 # chunked wins over CL
    b"POST /x HTTP/1.1\r\nHost: a\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n",   # bad chunk: 400
    b"POST /x HTTP/1.1\r\nHost: a\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nab\r\n",   # short chunk
    b"GET /a HTTP/1.1\r\nHost: a\r\nX_Under: 1\r\nGood-One:  v  \r\n folded\r\n: empty\r\nNoColon\r\n\r\n",
    b"GET /a HTTP/1.1\r\nHost: a\r\nX-Nul: a\0b\r\n\r\n",                  # NUL in a header: 400
    b"GET /a%2 HTTP/1.1\r\nHost: a\r\nTransfer-Encoding: gzip\r\n\r\n",     # bad URI: 400 before 501
    b"GET /../x HTTP/1.1\r\nHost: a\r\n\r\n",                               # above the root: 400
    b"GET //a/./b/%2e%2E/c?q=1#f HTTP/1.1\nHost: a\n\n",                    # bare LF, complex URI
    b"\r\n\r\nGET  /lead   HTTP/1.1  \r\nHost: a\r\n\r\n",                  # leading CRLF, spaces
    b"GET /x HTTP/1.1\r\nHost: a\r\n",                                      # no empty line: 400
    b"GET /x HTTP/1.1\r\nHost:a\r\nCookie: u=1\r\nCookie: v=2\r\nX-V:\tt\t\r\n\r\n",
    b"G@T / HTTP/1.1\r\nHost: a\r\n\r\n",                                   # bad method char
    b"GET / HTTP/1.x\r\nHost: a\r\n\r\n",                                   # bad version
    b"GET ftp:/x HTTP/1.1\r\nHost: a\r\n\r\n",                              # bad absolute form
    b"OPTIONS * HTTP/1.1\r\nHost: a\r\n\r\n",                               # '*' target: 400
    b"GET /q?a=1&b=%zz HTTP/1.1\r\nHost: a\r\n\r\n",                        # args are raw
    b"GET /" + b"p" * 9000 + b" HTTP/1.1\r\nHost: a\r\n\r\n",               # request line > 8 KiB: 414
    b"GET / HTTP/1.1\r\nHost: a\r\nX-Long: " + b"v" * 9000 + b"\r\n\r\n",   # header line > 8 KiB: 400
    b"GET / HTTP/1.1\r\nHost: a\r\n" + b"X-H: 1\r\n" * 300 + b"\r\n",       # > 254 header lines: 400
    b"GET / HTTP/1.1\r\nHost: a\r\n" + b"X-H: 1\r\n" * 200 + b"\r\n",       # 201 lines: ok
    b"GET /a/. HTTP/1.1\r\nHost: a\r\n\r\n",                                # trailing "/."
    b"GET /a/.b#f HTTP/1.1\r\nHost: a\r\n\r\n",                             # "/." not a segment
    b"GET /a\0b HTTP/1.1\r\nHost: a\r\n\r\n",                               # NUL in the target: 400
    b"GET /a\0b?q HTTP/1.1\r\nHost: a\r\n\r\n",
    b"GET /" + b"s" * 1500 + b"?" + b"q" * 900 + b" HTTP/1.1\r\nHost: a\r\n\r\n",      # long, simple
    b"GET /" + b"s" * 1500 + b"//x%41 HTTP/1.1\r\nHost: a\r\n\r\n",         # long, complex late
    b"GET http://h:8/x/../y HTTP/1.1\r\nHost: a\r\n\r\n",                    # absolute, dot segment
    b"GET / HTTP/1.1\r\nHost: a\r\nX: v \nY: w\r\n\r\n",                    # trailing SP, bare LF
    b"GET / HTTP/1.1\r\nHost: a\r\nX: v\r\r\nY: \r\nZ:\r\n\r\n",             # CR in a value, empties
    b"GET / HTTP/1.1\r\nHost: a\r\nX:  v\r\nY:v\r\n\r\n",                    # two spaces, none
    b"GET http://[::1]:8080/v6?x=1 HTTP/1.1\r\nHost: other\r\n\r\n",            # IP-literal host
    b"GET http://[v1.fe80::a+en1]/ HTTP/1.1\r\nHost: x\r\n\r\n",              # literal with sub-delims
    b"GET http://[::1 HTTP/1.1\r\nHost: a\r\n\r\n",                            # unterminated literal: 400
    b"GET http://[::1]x/ HTTP/1.1\r\nHost: a\r\n\r\n",                         # junk after ']': 400
    b"GET http://[a/b]/ HTTP/1.1\r\nHost: a\r\n\r\n",                          # '/' inside: 400
]


def synthetic(n: int, seed: int = 0xC0FFEE + 7, edge_rate: float = 0.15):
    """n raw messages: the C2-like request mix of records.gen_c2 serialised (with random
    Content-Length or chunked bodies), plus ``edge_rate`` of hand-made edge cases."""
    rng = np.random.Generator(np.random.PCG64(seed))
    reqs, arena = records.gen_c2(n, seed=seed)
    out = []
    for i in range(n):
        if rng.random() < edge_rate:
            out.append(_EDGE[int(rng.integers(0, len(_EDGE)))])
            continue
        f = {k: records.field_bytes(reqs, arena, i, k) for k in ("uri", "args", "hdrs", "host", "method")}
        body = bytes(rng.integers(32, 127, int(rng.integers(0, 300)), dtype=np.uint8)) if rng.random() < 0.4 else b""
        hdr_lines = [ln.split(b": ", 1) for ln in f["hdrs"].split(b"\r\n") if ln]
        it = {"method": f["method"], "uri": f["uri"], "args": f["args"], "host": f["host"] or None,
              "headers": [(k, v) for k, v in hdr_lines], "body": body,
              "version": "1.0" if rng.random() < 0.05 else "1.1"}
        if it["host"] is None and it["version"] == "1.1":
            it["host"] = "cafe.example.com"
        if body and rng.random() < 0.3:
            cuts = sorted(set(int(x) for x in rng.integers(1, len(body), int(rng.integers(0, 4))))) if len(body) > 1 else []
            edges = [0] + cuts + [len(body)]
            it["chunked"] = [edges[k + 1] - edges[k] for k in range(len(edges) - 1)]
        out.append(serialize(it))
    conn = [{"https": bool(rng.random() < 0.5), "rid": bytes(reqs[i]["rid"])} for i in range(n)]
    return out, conn


# ---------------------------------------------------------------- PROXY protocol cases
def proxy_cases():
    """Messages on a proxy_protocol listener (port 80 plain, 443 TLS) and what nginx 1.17.3's
    ngx_proxy_protocol_read makes of them: (message bytes, conn dict, expected) with expected
    either 444 (no response: a broken / missing header, or no request after it) or the record's
    (paddr, proxy_port, uri).  The KATs of tests/test_wire.py and the GPU parity test use them."""
    req = serialize({"uri": "/tea", "host": "cafe.example.com"})
    v6 = proxy_v2("2001:db8:0:0:0:0:0:1", "2001:db8::2", 443, 8443)
    C = {"https": False, "port": 80}
    cases = [
        (proxy_v1("192.168.0.1", "192.168.0.11", 56324, 80) + req, C, (b"192.168.0.1", 56324, b"/tea")),
        (proxy_v1("2001:DB8::1", "2001:db8::2", 1, 80) + req, C, (b"2001:DB8::1", 1, b"/tea")),   # v1: as sent
        (b"PROXY UNKNOWN\r\n" + req, C, (b"", 0, b"/tea")),
        (b"PROXY UNKNOWN ffff:f...f:ffff ffff:f...f:ffff 65535 65535\r\n" + req, C, (b"", 0, b"/tea")),
        (proxy_v1("10.0.0.5:99", "10.0.0.1", 7, 80) + req, C, (b"10.0.0.5:99", 7, b"/tea")),   # chars only
        (proxy_v1("1.2.3.4", "5.6.7.8", 0, 0) + req, C, (b"1.2.3.4", 0, b"/tea")),
        (b"PROXY TCP4 1.2.3.4 5.6.7.8 080 80\r\n" + req, C, (b"1.2.3.4", 80, b"/tea")),   # ngx_atoi
        (proxy_v2("203.0.113.7", "10.0.0.1", 40001, 80) + req, C, (b"203.0.113.7", 40001, b"/tea")),
        (v6 + req, {"https": True, "port": 443}, (b"2001:db8::1", 443, b"/tea")),          # ngx_sock_ntop
        (proxy_v2("203.0.113.7", "10.0.0.1", 40001, 80, tlv=b"\x04\x00\x01x") + req, C,
         (b"203.0.113.7", 40001, b"/tea")),                                                 # TLVs skipped
        (proxy_v2("203.0.113.7", "10.0.0.1", 1, 80, command=0) + req, C, (b"", 0, b"/tea")),    # LOCAL
        (proxy_v2("203.0.113.7", "10.0.0.1", 1, 80, transport=2) + req, C, (b"", 0, b"/tea")),  # DGRAM
        (proxy_v2("::ffff:1.2.3.4", "::1", 9, 80) + req, C, (b"::ffff:1.2.3.4", 9, b"/tea")),
        # broken or missing: nginx closes the connection
        (req, C, 444),
        (b"PROXY TCP4 1.2.3.4 5.6.7.8 99999 80\r\n" + req, C, 444),
        (b"PROXY TCP4 1.2.3.4 5.6.7.8 -1 80\r\n" + req, C, 444),
        (b"PROXY TCP4 1.2.3.4 5.6.7.8  80\r\n" + req, C, 444),                  # empty port
        (b"PROXY TCP5 1.2.3.4 5.6.7.8 1 80\r\n" + req, C, 444),
        (b"PROXY TCP4 1.2.3.g 5.6.7.8 1 80\r\n" + req, C, 444),
        (b"PROXY TCP4 1.2.3.4\r\n" + req, C, 444),
        (b"proxy TCP4 1.2.3.4 5.6.7.8 1 80\r\n" + req, C, 444),
        (b"PROXY TCP4 1.2.3.4 5.6.7.8 1 80", C, 444),                           # no CRLF at all
        (proxy_v1("1.2.3.4"), C, 444),                                          # no request after it
        (b"\r\n\r\n\x00\r\nQUIT\n\x11\x11\x00\x0c" + bytes(12) + req, C, 444),   # v2, version 1
        (b"\r\n\r\n\x00\r\nQUIT\n\x21\x11\x01\x00" + bytes(12), C, 444),         # length past the end
        (b"\r\n\r\n\x00\r\nQUIT\n\x21\x11\x00\x08" + bytes(8) + req, C, 444),    # INET, too short
        (b"PROXY TCP4 " + b"1" * 60 + b" 5.6.7.8 1 80\r\n" + req, C, (b"", 1, b"/tea")),   # too long to be an address
        # keep-alive: the caller's copy of the connection's address, no header read
        (req, {"https": False, "port": 80, "proxy_done": True, "paddr": "198.51.100.9", "proxy_port": 333},
         (b"198.51.100.9", 333, b"/tea")),
        # not a proxy_protocol port: a PROXY line is a (bad) request line
        (proxy_v1("1.2.3.4") + req, {"https": False, "port": 8080}, 400),
        (req, {"https": False, "port": 8080}, (b"", 0, b"/tea")),
    ]
    return cases
