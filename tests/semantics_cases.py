"""Verdict-affecting directives every rendered config carries, and the default-deny compile
(VERDICT r3 item 1): known-answer cases shared by the CPU oracle tests (tests/test_semantics.py)
and the GPU parity tests (tests/test_gpu_semantics.py).

- client_max_body_size (version1/nginx.ingress.tmpl:175, version2/nginx.virtualserver.tmpl:93; set
  by nginx.org/client-max-body-size, annotations.go:172, and the ConfigMap, configmaps.go:70):
  nginx answers 413 in its find-config phase when Content-Length exceeds the limit of the location
  found (the server's when none; 1m by default, config_params.go:112) -- before a location
  `return`, an auto_redirect or an internal redirect, and before the Wallarm access phase.  A
  chunked body is checked only when it is read, i.e. by the location that proxies it.
- realip (nginx.ingress.tmpl:46-49, nginx.virtualserver.tmpl:64-72, configmaps.go:153-169): under
  set_real_ip_from, $remote_addr (a whitelisted VS condition variable, validation.go:357) and the
  ip_hash key come from X-Real-IP / X-Forwarded-For / a named header.  The reference's own
  virtualserver_test.go:225-263 carries SetRealIPFrom 0.0.0.0/0, X-Real-IP, recursive.
- default-deny: snippet directives the engine does not model (auth_basic, auth_request, ...) make
  the requests reaching them GM_ACT_UNSUPPORTED, counted in n_rejected_other.
- the access module (allow / deny, round 6): the main template's stub_status server
  (nginx.tmpl:104-115, -nginx-status-allow-cidrs), snippet rules at server and location level,
  IPv4 / IPv6 / IPv4-mapped clients, the address after realip, `return` before the access phase.

The expected answers are nginx 1.17.3 behaviour written out by hand (parity unpinned: no
reference test pins them beyond the fixture's fields); the engine and the oracle must also agree
on every other verdict field."""

from __future__ import annotations

from gpumatch import blob, confgen

PROXY, REDIRECT, RETURN, AUTO_301, NOT_FOUND, UNSUPPORTED, TOO_LARGE, FORBIDDEN = 0, 1, 2, 3, 4, 8, 10, 11
ANY = None   # oracle parity only


def _ingress(name, host, paths, ann=None):
    return {"metadata": {"name": name, "namespace": "default", "annotations": dict(ann or {})},
            "spec": {"rules": [{"host": host, "http": {"paths": [
                {"path": p, "backend": {"serviceName": s, "servicePort": 80}} for p, s in paths]}}]}}


def body_limit_case():
    """An Ingress whose locations carry client_max_body_size 1k; the main config's default server."""
    ing = _ingress("cafe", "cafe.example.com", [("/tea", "tea-svc"), ("/coffee/", "coffee-svc")],
                   {"nginx.org/client-max-body-size": "1k"})
    b = blob.make_blob(confgen.render_main(), confgen.ingress_files([ing]))
    h = "cafe.example.com"
    big = 1024 * 1024 + 1   # past the default 1m
    cases = [
        ({"host": h, "uri": "/tea", "body": b"x" * 1023}, PROXY),
        ({"host": h, "uri": "/tea", "body": b"x" * 1024}, PROXY),            # "1k" = 1024: not above it
        ({"host": h, "uri": "/tea", "body": b"x" * 1025}, TOO_LARGE),
        ({"host": h, "uri": "/tea/cup", "body": b"y" * 4000}, TOO_LARGE),
        ({"host": h, "uri": "/tea", "body": b"x" * 1025, "chunked": True}, TOO_LARGE),   # read by proxy_pass
        ({"host": h, "uri": "/tea", "body": b"x" * 1024, "chunked": True}, PROXY),
        ({"host": h, "uri": "/tea", "body": b""}, PROXY),
        ({"host": h, "uri": "/coffee", "body": b"z" * 2000}, TOO_LARGE),     # before the auto_redirect
        ({"host": h, "uri": "/coffee", "body": b"z" * 2000, "chunked": True}, AUTO_301),   # never read
        ({"host": h, "uri": "/coffee", "body": b"z" * 10}, AUTO_301),
        ({"host": h, "uri": "/coffee/beans", "body": b"z" * 1500}, TOO_LARGE),
        ({"host": h, "uri": "/nothing", "body": b"n" * 2000}, NOT_FOUND),    # the server's limit: 1m
        ({"host": h, "uri": "/nothing", "body": b"n" * big}, TOO_LARGE),
        ({"host": "other.example.com", "uri": "/", "body": b"d" * 9}, RETURN),           # default server's 404
        ({"host": "other.example.com", "uri": "/", "body": b"d" * big}, TOO_LARGE),      # before `return 404`
        ({"host": "other.example.com", "uri": "/", "body": b"d" * big, "chunked": True}, RETURN),
        # HTTP/2 DATA frames without a content-length header: nginx's content_length_n is -1, so
        # only a location that reads the body checks it -- the caller marks such a record
        # GM_REQ_CHUNKED (gpumatch.h); parity-unpinned (no reference fixture covers HTTP/2 bodies)
        ({"host": h, "uri": "/coffee", "body": b"z" * 2000, "chunked": True, "http2": True}, AUTO_301),
        ({"host": "other.example.com", "uri": "/", "body": b"d" * big, "chunked": True, "http2": True}, RETURN),
        ({"host": h, "uri": "/tea", "body": b"x" * 1025, "chunked": True, "http2": True}, TOO_LARGE),
        ({"host": h, "uri": "/tea", "body": b"x" * 1025, "http2": True}, TOO_LARGE),   # with content-length
    ]
    return b, cases


def vs_body_case():
    """A VirtualServer rules route under client_max_body_size 1k: the `return 418` location has no
    limit of its own (1m), the named @rules locations carry 1k -- so a Content-Length body of 2000
    passes (checked at the 418 location) and a chunked one gets 413 (read by @rules_*)."""
    vs = {"metadata": {"name": "cafe", "namespace": "default"},
          "spec": {"host": "cafe.example.com",
                   "upstreams": [{"name": "tea-v1", "service": "tea-svc-v1", "port": 80},
                                 {"name": "tea-v2", "service": "tea-svc-v2", "port": 80}],
                   "routes": [{"path": "/tea", "rules": {"conditions": [{"header": "x-version"}],
                                                         "matches": [{"values": ["v2"], "upstream": "tea-v2"}],
                                                         "defaultUpstream": "tea-v1"}},
                              {"path": "/coffee", "upstream": "tea-v1"}]}}
    p = confgen.default_config_params()
    p["ClientMaxBodySize"] = "1k"
    b = blob.make_blob(confgen.render_main(p), confgen.virtual_server_files([vs], base=p, pem_name=""))
    h = "cafe.example.com"
    cases = [
        ({"host": h, "uri": "/tea", "body": b"b" * 2000}, PROXY),
        ({"host": h, "uri": "/tea", "body": b"b" * 2000, "headers": [("X-Version", "v2")]}, PROXY),
        ({"host": h, "uri": "/tea", "body": b"b" * 2000, "chunked": True}, TOO_LARGE),
        ({"host": h, "uri": "/tea", "body": b"b" * 2000, "chunked": True, "headers": [("X-Version", "v2")]}, TOO_LARGE),
        ({"host": h, "uri": "/tea", "body": b"b" * 900, "chunked": True}, PROXY),
        ({"host": h, "uri": "/tea", "body": b"b" * (1024 * 1024 + 1)}, TOO_LARGE),   # the 418 location's 1m
        ({"host": h, "uri": "/coffee", "body": b"c" * 2000}, TOO_LARGE),             # a plain location: 1k
        ({"host": h, "uri": "/coffee", "body": b"c" * 2000, "chunked": True}, TOO_LARGE),
    ]
    return b, cases


def _rules_vs(host, cond, values):
    ups = [{"name": f"u{k}", "service": f"svc{k}", "port": 80} for k in range(len(values) + 1)]
    return {"metadata": {"name": host.split(".")[0], "namespace": "default"},
            "spec": {"host": host, "upstreams": ups,
                     "routes": [{"path": "/", "rules": {"conditions": [cond],
                                                        "matches": [{"values": [v], "upstream": f"u{k + 1}"}
                                                                    for k, v in enumerate(values)],
                                                        "defaultUpstream": "u0"}}]}}


def _vs_blob(vs, **params):
    p = confgen.default_config_params()
    p.update(params)
    return blob.make_blob(confgen.render_main(p), confgen.virtual_server_files([vs], base=p, pem_name=""))


# match index per request: 0.. = matches[k], 0xFF = default (u0)
ADDRS = ["10.0.0.5", "2001:db8::1", "::ffff:1.2.3.4", "1.2.3.4"]


def realip_xff_case():
    """real_ip_header X-Forwarded-For, recursive, trusted 192.168.0.0/16 and 10.1.0.0/16: a rules
    route on $remote_addr (matches ADDRS) and one on $remote_port."""
    vs = _rules_vs("xff.example.com", {"variable": "$remote_addr"}, ADDRS)
    b = _vs_blob(vs, SetRealIPFrom=["192.168.0.0/16", "10.1.0.0/16"], RealIPHeader="X-Forwarded-For",
                 RealIPRecursive=True)
    h = "xff.example.com"

    def r(raddr, *xff):
        return {"host": h, "uri": "/", "raddr": raddr, "headers": [("X-Forwarded-For", x) for x in xff]}
    cases = [
        (r("192.168.1.1", "10.0.0.5"), 0),
        (r("172.16.0.1", "10.0.0.5"), 0xFF),                      # connection not trusted
        (r("192.168.1.1", "10.0.0.5, 10.1.2.3"), 0),              # recursive past the trusted 10.1.2.3
        (r("192.168.1.1", "10.0.0.5, 172.16.9.9"), 0xFF),         # 172.16.9.9 is not trusted: it stays
        (r("192.168.1.1", "10.0.0.5", "10.1.0.1"), 0),            # the last header first, then the one before
        (r("192.168.1.1", "10.0.0.5", "1.2.3.4"), 3),
        (r("192.168.1.1", "2001:DB8:0:0:0:0:0:1"), 1),            # ngx_inet6_ntop text
        (r("192.168.1.1", "[2001:db8::1]:8080"), 1),
        (r("192.168.1.1", "::ffff:1.2.3.4"), 2),
        (r("192.168.1.1", "garbage"), 0xFF),
        (r("192.168.1.1", ""), 0xFF),
        (r("192.168.1.1", "1.2.3.4:99999"), 0xFF),               # port out of range: not an address
        (r("192.168.1.1", "1.2.3.4:80"), 3),
        (r("192.168.1.1", " 1.2.3.4 ,"), 3),                     # trailing separators trimmed
        (r("192.168.1.1", ",1.2.3.4"), 0xFF),                    # byte 0 is never a separator: ",1.2.3.4"
        (r("::ffff:192.168.1.1", "10.0.0.5"), 0),                 # an IPv4-mapped connection matches as IPv4
        (r("192.168.1.1", "1..2.3"), 0xFF),                       # ngx_inet_addr: empty octets are 0 -> 1.0.2.3
        (r("192.168.1.1"), 0xFF),                                 # no header
        (r("192.168.1.1", "10.1.0.9, 10.1.0.8"), 0xFF),           # all trusted: the leftmost is taken (10.1.0.9)
        (r("10.1.3.3", "1.2.3.4"), 3),
        (r("", "1.2.3.4"), 0xFF),                                 # a record without a connection address
    ]
    return b, cases


def realip_xrealip_case():
    """The reference's own fixture values (virtualserver_test.go:230-232): set_real_ip_from 0.0.0.0/0,
    real_ip_header X-Real-IP, real_ip_recursive on -- X-Real-IP is one header, the first."""
    vs = _rules_vs("xri.example.com", {"variable": "$remote_addr"}, ADDRS)
    b = _vs_blob(vs, SetRealIPFrom=["0.0.0.0/0"], RealIPHeader="X-Real-IP", RealIPRecursive=True)
    h = "xri.example.com"

    def r(raddr, *hdrs):
        return {"host": h, "uri": "/", "raddr": raddr, "headers": list(hdrs)}
    cases = [
        (r("8.8.8.8", ("X-Real-IP", "10.0.0.5")), 0),
        (r("8.8.8.8", ("x-real-ip", "1.2.3.4"), ("X-Real-IP", "10.0.0.5")), 3),   # the first one
        # recursive with 0.0.0.0/0: every IPv4 address is trusted, so the walk goes on to the list's
        # first address
        (r("8.8.8.8", ("X-Real-IP", "10.0.0.5, 1.2.3.4")), 0),
        (r("8.8.8.8", ("X-Real-IP", "1.2.3.4, 10.0.0.5")), 3),
        (r("2001:db8::9", ("X-Real-IP", "10.0.0.5")), 0xFF),      # IPv6 connection: 0.0.0.0/0 does not hold it
        (r("8.8.8.8", ("X-Forwarded-For", "10.0.0.5")), 0xFF),
        (r("8.8.8.8"), 0xFF),
    ]
    return b, cases


def realip_header_port_case():
    """A named header (real_ip_header CF-Connecting-IP), not recursive, and $remote_port."""
    vs = _rules_vs("hdr.example.com", {"variable": "$remote_port"}, ["8080", "40000"])
    b = _vs_blob(vs, SetRealIPFrom=["127.0.0.1", "::1"], RealIPHeader="CF-Connecting-IP")
    h = "hdr.example.com"

    def r(raddr, *hdrs, rport=40000):
        return {"host": h, "uri": "/", "raddr": raddr, "headers": list(hdrs), "remote_port": rport}
    cases = [
        (r("127.0.0.1", ("CF-Connecting-IP", "1.2.3.4:8080")), 0),
        (r("127.0.0.1", ("cf-connecting-ip", "1.2.3.4")), 0xFF),   # no port: $remote_port is ""
        (r("127.0.0.2", ("CF-Connecting-IP", "1.2.3.4:8080")), 1),  # untrusted: the connection's port
        (r("::1", ("CF-Connecting-IP", "[::2]:8080")), 0),
        (r("127.0.0.1", ("CF-Connecting-IP", "1.2.3.4:8080, 5.6.7.8")), 0xFF),   # not recursive: the last
        (r("127.0.0.1"), 1),
    ]
    return b, cases


def realip_proxy_protocol_case():
    """real_ip_header proxy_protocol (examples/proxy-protocol/README.md): a trusted connection's
    $remote_addr is its PROXY header's source address (the record's paddr, gm_parse_requests); no
    PROXY address (a record without one, "PROXY UNKNOWN") or an untrusted peer keeps the peer's;
    a PROXY address that is no address is declined too."""
    vs = _rules_vs("pp.example.com", {"variable": "$remote_addr"}, ADDRS)
    b = _vs_blob(vs, SetRealIPFrom=["10.0.0.0/8"], RealIPHeader="proxy_protocol", ProxyProtocol=True)
    h = "pp.example.com"
    cases = [
        ({"host": h, "uri": "/", "raddr": "10.9.9.9"}, 0xFF),                                   # no PROXY address
        ({"host": h, "uri": "/", "raddr": "1.2.3.4"}, 3),
        ({"host": h, "uri": "/", "raddr": "10.0.0.5"}, 0),
        ({"host": h, "uri": "/", "raddr": "10.9.9.9", "paddr": "1.2.3.4", "proxy_port": 5555}, 3),
        ({"host": h, "uri": "/", "raddr": "10.9.9.9", "paddr": "2001:db8::1", "proxy_port": 1}, 1),
        ({"host": h, "uri": "/", "raddr": "10.9.9.9", "paddr": "2001:DB8:0::1", "proxy_port": 1}, 1),   # ntop
        ({"host": h, "uri": "/", "raddr": "8.8.8.8", "paddr": "1.2.3.4", "proxy_port": 5555}, 0xFF),  # untrusted
        ({"host": h, "uri": "/", "raddr": "10.9.9.9", "paddr": "1.2.3", "proxy_port": 5555}, 0xFF),   # no address
        ({"host": h, "uri": "/", "raddr": "10.9.9.9", "paddr": "10.0.0.5:99", "proxy_port": 7}, 0),   # addr:port
    ]
    return b, cases


def proxy_port_case():
    """real_ip_header proxy_protocol: $remote_port becomes the PROXY header's source port."""
    vs = _rules_vs("pport.example.com", {"variable": "$remote_port"}, ["5555", "40000"])
    b = _vs_blob(vs, SetRealIPFrom=["0.0.0.0/0"], RealIPHeader="proxy_protocol", ProxyProtocol=True)
    h = "pport.example.com"
    cases = [
        ({"host": h, "uri": "/", "raddr": "10.9.9.9", "paddr": "1.2.3.4", "proxy_port": 5555}, 0),
        ({"host": h, "uri": "/", "raddr": "10.9.9.9"}, 1),                    # no PROXY address: the peer's
        ({"host": h, "uri": "/", "raddr": "10.9.9.9", "paddr": "1.2.3.4", "proxy_port": 40000}, 1),
        ({"host": h, "uri": "/", "raddr": "10.9.9.9", "paddr": "zz", "proxy_port": 5555}, 1),   # declined
    ]
    return b, cases


def default_deny_case():
    """Snippets the engine does not model: `deny all;` in one Ingress's locations, an access rule in
    another's server, an `if` doing more than `return` -- and neutral snippets that stay compiled."""
    a = _ingress("denied", "denied.example.com", [("/", "a-svc"), ("/x", "a-svc")],
                 {"nginx.org/location-snippets": "auth_basic closed;"})
    bsrv = _ingress("acl", "acl.example.com", [("/", "b-svc")],
                    {"nginx.org/server-snippets": "auth_request /auth;\nallow unknown.example;",
                     "nginx.org/redirect-to-https": "true"})
    c = _ingress("neutral", "neutral.example.com", [("/", "c-svc")],
                 {"nginx.org/location-snippets": "add_header X-Frame-Options DENY;\nproxy_set_header X-A b;",
                  "nginx.org/server-snippets": "if ($http_x_debug) { set $dbg 1; }"})
    d = _ingress("ok", "ok.example.com", [("/", "d-svc")],
                 {"nginx.org/location-snippets": "proxy_read_timeout 5s;\n# a comment"})
    b = blob.make_blob(confgen.render_main(), confgen.ingress_files([a, bsrv, c, d]))
    cases = [
        ({"host": "denied.example.com", "uri": "/"}, UNSUPPORTED),
        ({"host": "denied.example.com", "uri": "/x/y"}, UNSUPPORTED),
        ({"host": "denied.example.com", "uri": "/", "body": b"q" * 2000000}, TOO_LARGE),   # 413 comes first
        ({"host": "acl.example.com", "uri": "/"}, UNSUPPORTED),
        ({"host": "acl.example.com", "uri": "/", "headers": [("X-Forwarded-Proto", "http")]}, REDIRECT),
        ({"host": "neutral.example.com", "uri": "/"}, UNSUPPORTED),      # the `if` sets a variable
        ({"host": "ok.example.com", "uri": "/"}, PROXY),
        ({"host": "ok.example.com", "uri": "/z"}, PROXY),
    ]
    # rejected constructs gm_rejects lists (each once)
    rejects = ["location /: auth_basic closed", "location /x: auth_basic closed", "server: auth_request /auth",
               "server: allow unknown.example", "server: if ($http_x_debug)"]
    return b, cases, rejects


def access_case():
    """ngx_http_access_module (nginx 1.17.3, satisfy all): the stock main config's stub_status server
    (port 8080, allow 127.0.0.1, deny all) and a status server with more CIDRs; snippet rules in a
    server (inherited by its locations) and in a location (replacing the server's); IPv6 and
    IPv4-mapped clients; a `return` location (rewrite phase: before the access phase); a realip
    server whose rules see the X-Real-IP address."""
    p = confgen.default_config_params()
    p["NginxStatusAllowCIDRs"] = ["127.0.0.1", "10.8.0.0/16", "2001:db8::/32"]
    srv = _ingress("acl", "acl.example.com", [("/", "b-svc"), ("/open", "c-svc")],
                   {"nginx.org/server-snippets": "deny 10.1.2.3;\nallow 10.0.0.0/8;\nallow ::1;\ndeny all;",
                    })
    loc = _ingress("loc", "loc.example.com", [("/", "d-svc")],
                   {"nginx.org/location-snippets": "allow 192.168.0.0/16;\ndeny all;"})
    ret = _ingress("ret", "ret.example.com", [("/", "e-svc")],
                   {"nginx.org/server-snippets": "deny all;", "nginx.org/redirect-to-https": "true"})
    rip = _ingress("rip", "rip.example.com", [("/", "f-svc")],
                   {"nginx.org/server-snippets": "set_real_ip_from 10.0.0.0/8;\nallow 1.2.3.0/24;\ndeny all;"})
    b = blob.make_blob(confgen.render_main(p), confgen.ingress_files([srv, loc, ret, rip]))

    def st(raddr, uri="/stub_status"):
        return {"host": "x", "uri": uri, "raddr": raddr, "port": 8080, "https": False}
    a, lo, rt, rp = "acl.example.com", "loc.example.com", "ret.example.com", "rip.example.com"
    cases = [
        (st("127.0.0.1"), RETURN), (st("127.0.0.2"), FORBIDDEN), (st("10.8.3.4"), RETURN),
        (st("2001:db8:1::5"), RETURN), (st("2001:db9::5"), FORBIDDEN), (st("::ffff:127.0.0.1"), RETURN),
        (st("::ffff:10.9.0.1"), FORBIDDEN), (st("::1"), FORBIDDEN),
        (st("10.8.3.4", "/other"), NOT_FOUND), (st("9.9.9.9", "/other"), FORBIDDEN),   # the server level's rules
        ({"host": a, "uri": "/", "raddr": "10.1.2.3"}, FORBIDDEN),      # the first matching rule decides
        ({"host": a, "uri": "/", "raddr": "10.1.2.4"}, PROXY),
        ({"host": a, "uri": "/open", "raddr": "11.0.0.1"}, FORBIDDEN),
        ({"host": a, "uri": "/", "raddr": "::1"}, PROXY),
        ({"host": a, "uri": "/", "raddr": "::ffff:10.0.0.9"}, PROXY),   # mapped: the IPv4 rules
        ({"host": a, "uri": "/", "raddr": "2001:db8::7"}, FORBIDDEN),
        ({"host": lo, "uri": "/", "raddr": "192.168.7.7"}, PROXY),
        ({"host": lo, "uri": "/", "raddr": "10.0.0.1"}, FORBIDDEN),
        ({"host": rt, "uri": "/", "raddr": "10.0.0.1"}, FORBIDDEN),
        ({"host": rt, "uri": "/", "raddr": "10.0.0.1", "headers": [("X-Forwarded-Proto", "http")]}, REDIRECT),
        ({"host": rp, "uri": "/", "raddr": "10.0.0.1", "headers": [("X-Real-IP", "1.2.3.9")]}, PROXY),
        ({"host": rp, "uri": "/", "raddr": "10.0.0.1", "headers": [("X-Real-IP", "1.2.4.9")]}, FORBIDDEN),
        ({"host": rp, "uri": "/", "raddr": "1.2.3.1", "headers": [("X-Real-IP", "8.8.8.8")]}, PROXY),   # untrusted
        ({"host": rp, "uri": "/", "raddr": "not-an-address"}, UNSUPPORTED),
    ]
    return b, cases


def http_unknown_case():
    """An http-level directive outside the known set (http snippets): every server's requests defer
    once past their server rewrite phase (redirects still answered)."""
    main = confgen.render_main().replace("http {\n", "http {\n    limit_req zone=one burst=5;\n", 1)
    ing = _ingress("cafe", "cafe.example.com", [("/", "s")], {"nginx.org/redirect-to-https": "true"})
    b = blob.make_blob(main, confgen.ingress_files([ing]))
    cases = [
        ({"host": "cafe.example.com", "uri": "/"}, UNSUPPORTED),
        ({"host": "cafe.example.com", "uri": "/", "headers": [("X-Forwarded-Proto", "http")]}, REDIRECT),
        ({"host": "nope.example.com", "uri": "/"}, UNSUPPORTED),
    ]
    return b, cases


ROUTE_CASES = {"body_limit": body_limit_case, "vs_body": vs_body_case, "http_unknown": http_unknown_case,
               "access": access_case}
# expected: the rules route's match index (0xFF default), or UNSUPPORTED for a deferred verdict
MATCH_CASES = {"realip_xff": realip_xff_case, "realip_xrealip": realip_xrealip_case,
               "realip_header_port": realip_header_port_case, "realip_proxy_protocol": realip_proxy_protocol_case,
               "realip_proxy_port": proxy_port_case}
