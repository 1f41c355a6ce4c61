"""nginx.org/rewrites: the URI a proxied request is sent upstream with.

Pinned by the reference: parseRewrites' unit tests (annotations_test.go:9-41) and the rewrites
example's stated mappings (examples/rewrites/README.md:37-45: /tea/ -> /, /tea/abc -> /abc,
/coffee/ -> /beans/, /coffee/abc -> /beans/abc, /tea -> redirect to /tea/).  The %-escaping of
the $uri tail is nginx's ngx_http_proxy_create_request behaviour restated (parity unpinned).
CPU: confgen + the oracle; the GPU chain (gm_parse_requests -> gm_match_batch ->
gm_upstream_uris) is in test_gpu_rewrites.py."""

import pytest

from gpumatch import blob, confgen, wire
from oracle_py import Oracle, parse_requests, upstream_uris, uri_list


def test_parse_rewrites_kats():
    # annotations_test.go:9-41
    assert confgen.parse_rewrites("serviceName=coffee-svc rewrite=/beans/") == ("coffee-svc", "/beans/")
    assert confgen.parse_rewrites("\t\n serviceName=coffee-svc rewrite=/beans/ \t\n") == ("coffee-svc", "/beans/")
    with pytest.raises(ValueError):
        confgen.parse_rewrites("serviceNamecoffee-svc rewrite=/")
    # getRewrites: ';'-separated, invalid entries skipped (annotations.go:347-361)
    ing = {"metadata": {"annotations": {"nginx.org/rewrites":
                                        "serviceName=tea-svc rewrite=/;bad;serviceName=coffee-svc rewrite=/beans/"}}}
    assert confgen.get_rewrites(ing) == {"tea-svc": "/", "coffee-svc": "/beans/"}


def cafe_rewrites_blob():
    """examples/rewrites/README.md's cafe-ingress (+ a path without a rewrite)."""
    ing = {"metadata": {"name": "cafe-ingress", "namespace": "default",
                        "annotations": {"nginx.org/rewrites":
                                        "serviceName=tea-svc rewrite=/;serviceName=coffee-svc rewrite=/beans/"}},
           "spec": {"rules": [{"host": "cafe.example.com", "http": {"paths": [
               {"path": "/tea/", "backend": {"serviceName": "tea-svc", "servicePort": 80}},
               {"path": "/coffee/", "backend": {"serviceName": "coffee-svc", "servicePort": 80}},
               {"path": "/juice", "backend": {"serviceName": "juice-svc", "servicePort": 80}}]}}]}}
    return blob.make_blob(confgen.render_main(), confgen.ingress_files([ing]))


def test_rewrite_renders_proxy_pass_uri():
    text = blob.parse_blob(cafe_rewrites_blob())
    conf = b"".join(d for k, _, d in text if k == blob.ENTRY_CONFD)
    assert b"proxy_pass http://default-cafe-ingress-cafe.example.com-tea-svc-80/;" in conf
    assert b"proxy_pass http://default-cafe-ingress-cafe.example.com-coffee-svc-80/beans/;" in conf
    assert b"proxy_pass http://default-cafe-ingress-cafe.example.com-juice-svc-80;" in conf


# (raw request target, expected upstream URI; None = not proxied)
KATS = [
    ("/tea/", b"/"), ("/tea/abc", b"/abc"), ("/coffee/", b"/beans/"), ("/coffee/abc", b"/beans/abc"),  # README
    ("/tea", None),                                   # README: /tea is redirected to /tea/ (auto_redirect)
    ("/coffee/abc?x=1&y=%20", b"/beans/abc?x=1&y=%20"),  # args appended raw
    ("/coffee/a%20b", b"/beans/a%20b"),               # quoted: the decoded tail is re-escaped
    ("/coffee/caf%C3%A9?q", b"/beans/caf%C3%A9?q"),   # bytes >= 0x80 escaped upper-case
    ("/coffee/%3F%23%25", b"/beans/%3F%23%25"),       # '?', '#', '%' in the decoded tail
    ("/coffee//a%20b", b"/beans/a b"),                # "//" before the '%': not quoted, tail raw
    ("/coffee/./a%41", b"/beans/aA"),                 # "/." first: not quoted
    ("/coffee/x%41/../y", b"/beans/y"),               # quoted and normalised
    ("/juice/x?y", b"/juice/x?y"),                    # no URI part: $request_uri unchanged
    ("/juice//a/../b%20c", b"/juice//a/../b%20c"),
    ("/other", None),                                 # default location: 404
    ("http://cafe.example.com/coffee/z?k", b"/beans/z?k"),   # absolute-form
]


def oracle_chain(b, targets):
    msgs = [f"GET {t} HTTP/1.1\r\nHost: cafe.example.com\r\n\r\n".encode() for t in targets]
    w, m = wire.build(msgs, [{"https": False, "port": 80}] * len(msgs))
    reqs, arena = parse_requests(w, m)
    o = Oracle(b, 1)
    v, _ = o.match(reqs, arena, nthreads=1)
    out, off, ln = upstream_uris(o, reqs, arena, v)
    return (w, m), v, uri_list(out, off, ln)


def test_rewrite_kats_oracle():
    _, v, got = oracle_chain(cafe_rewrites_blob(), [t for t, _ in KATS])
    for (t, exp), g, vv in zip(KATS, got, v):
        assert g == exp, (t, g, exp, vv)
    assert v["status"][4] == 301
