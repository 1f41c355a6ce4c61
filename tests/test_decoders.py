"""Request parsers before the WAF stages (Wallarm's parser_disable decoders):
the oracle's decoded views (percent, urlenc, json_doc, base64) and wallarm_parser_disable at
server and location level (annotations.go:320-329 -> nginx.ingress.tmpl:26,111).  The Wallarm
parsers themselves are not in the reference (proprietary package), so the views are the
engine's stated contract (include/gpumatch.h GM_DEC_*, gm_decode.inc) -- parity unpinned beyond
the oracle, which restates them independently; the GPU side is test_gpu_decoders.py."""

import base64

import numpy as np

from gpumatch import blob, confgen, engine, records, sigs
from oracle_py import Oracle

CONF = """http {
    wallarm_mode block;
    upstream u { server 10.0.0.1:80; }
    server {
        listen 80;
        server_name a.example.com;
        location / { proxy_pass http://u; }
        location /nopct/ { wallarm_parser_disable percent; proxy_pass http://u; }
        location /off/ { wallarm_mode off; proxy_pass http://u; }
    }
    server {
        listen 80;
        server_name b.example.com;
        wallarm_parser_disable base64;
        wallarm_parser_disable json_doc;
        location / { proxy_pass http://u; }
        location /all/ { wallarm_parser_disable urlenc; proxy_pass http://u; }
    }
}
"""

RULES = [sigs.Rule("lit", True, "ab", b"union select"), sigs.Rule("lit", True, "ab", b"<script>"),
         sigs.Rule("re", False, "ab", r"etc/pass(wd|wd2)"), sigs.Rule("lit", False, "b", b"/bin/sh"),
         sigs.Rule("re", True, "ab", r"[0-9]{3}zq"), sigs.Rule("lit", True, "u", b"/nothing")]
DECODERS = ("percent", "urlenc", "json_doc", "base64")


def decoder_blob(decoders=DECODERS):
    return blob.make_blob(CONF, {}, sigs.SigSet(RULES, decoders).to_text())


B64 = base64.b64encode(b"cat /etc/passwd now").decode()
JSON = ("Content-Type", "application/json; charset=utf-8")
FORM = ("Content-Type", "application/x-www-form-urlencoded")
# (host, uri, args, headers, body, expected hit count with every decoder on)
KATS = [
    ("a", "/", "q=union%20select", [], b"", 1),            # percent
    ("a", "/", "q=union+select", [], b"", 1),              # urlenc
    ("a", "/", "q=union select", [], b"", 1),              # raw
    ("a", "/nopct/", "q=union%20select", [], b"", 0),      # percent off in the location
    ("a", "/nopct/", "q=union+select", [], b"", 1),        # urlenc still on
    ("b", "/all/", "q=union+select", [], b"", 0),          # urlenc off (location)
    ("b", "/all/", "q=union%20select", [], b"", 1),        # its percent is the server's
    ("a", "/", "", [JSON], b'{"q": "\\u003cscript>"}', 1),   # json_doc
    ("b", "/", "", [JSON], b'{"q": "\\u003cscript>"}', 0),   # json_doc off (server)
    ("a", "/", "", [], b'{"q": "\\u003cscript>"}', 0),       # no json Content-Type
    ("a", "/", "x=" + B64, [], b"", 1),                    # base64 in $args
    ("b", "/", "x=" + B64, [], b"", 0),                    # base64 off (server)
    ("a", "/", "", [FORM], b"a=union+select&b=%2Fbin%2Fsh", 2),   # form body: both rules, body zone
    ("a", "/", "", [], b"a=union+select&b=%2Fbin%2Fsh", 0),       # not a form body
    ("a", "/", "", [], B64.encode(), 1),                   # base64 in the body
    ("a", "/off/", "q=union%20select", [], b"", 0),        # WAF off
    ("a", "/", "q=%31%32%33zq&r=un%69on%20select", [], b"", 2),   # decoded regex + literal
    ("a", "/", "q=%zz%2", [], b"", 0),                     # bad escapes stay
    ("a", "/", "", [JSON], b'"\\ud83d\\ude00 \\ud800x \\/bin\\/sh \\q"', 1),   # pairs, lone, \/ , unknown
]


def kat_items():
    return [{"host": f"{h}.example.com", "uri": u, "args": a, "headers": hd, "body": b, "port": 80}
            for h, u, a, hd, b, _ in KATS]


def test_decoders_directive_and_stats():
    e = engine.Engine(compile_only=True)
    e.load(decoder_blob(), 1)
    assert e.stats()["decoders"] == 0xF
    e.load(decoder_blob(("base64", "bogus")), 2)
    assert e.stats()["decoders"] == 0x8
    assert sigs.SigSet.from_text(sigs.SigSet(RULES, DECODERS).to_text()).decoders == list(DECODERS)


def test_decoded_views_oracle():
    reqs, arena = records.from_dicts(kat_items())
    v, h = Oracle(decoder_blob(), 1).match(reqs, arena, nthreads=1)
    assert [int(x) for x in v["n_hits"]] == [k[5] for k in KATS]
    # without decoders only the raw match remains
    v0, _ = Oracle(decoder_blob(()), 1).match(reqs, arena, nthreads=1)
    assert [int(x) for x in v0["n_hits"]] == [1 if k[2] == "q=union select" else 0 for k in KATS]
    assert all(v["action"][i] == (6 if KATS[i][5] else 0) for i in range(len(KATS)))


def test_parser_disable_annotation_renders():
    """wallarm.com/parser-disable -> wallarm_parser_disable lines (annotations.go:320-329,
    nginx.ingress.tmpl:26)."""
    base = confgen.default_config_params()
    base["MainEnableWallarm"] = True
    ing = {"metadata": {"name": "cafe", "namespace": "default",
                        "annotations": {"wallarm.com/mode": "block",
                                        "wallarm.com/parser-disable": "base64, json_doc"}},
           "spec": {"rules": [{"host": "cafe.example.com", "http": {"paths": [
               {"path": "/tea", "backend": {"serviceName": "tea-svc", "servicePort": 80}}]}}]}}
    files = confgen.ingress_files([ing], base=base)
    text = "".join(files.values())
    assert "wallarm_parser_disable base64;" in text and "wallarm_parser_disable json_doc;" in text
    b = blob.make_blob(confgen.render_main(base), files, sigs.SigSet(RULES, DECODERS).to_text())
    items = [{"host": "cafe.example.com", "uri": "/tea", "args": "x=" + B64, "port": 80},
             {"host": "cafe.example.com", "uri": "/tea", "args": "q=union%20select", "port": 80}]
    reqs, arena = records.from_dicts(items)
    v, _ = Oracle(b, 1).match(reqs, arena, nthreads=1)
    assert list(v["n_hits"]) == [0, 1]
