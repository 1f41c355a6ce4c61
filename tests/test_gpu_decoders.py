"""Request parsers before the WAF stages (§8 f4) on the GPU: gm_match_batch's decoded-view pass
(gm_decode.inc: shadow records, the WAF stages again, one dedupe set) against the oracle's
decoded views -- the decoder KATs, and 20k requests of the 10k-rule C4 set with its signature
examples planted percent-, plus-, JSON- and base64-encoded, under each parser_disable shape."""

import base64
import json

import numpy as np
import pytest

from gpumatch import engine, records, sigs, workloads
from helpers import assert_verdicts_equal
from oracle_py import Oracle
from test_decoders import KATS, decoder_blob, kat_items

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    return engine.Engine(0)


def _both(eng, b, items):
    reqs, arena = records.from_dicts(items)
    eng.load(b, 5)
    got, gh = eng.match_host(reqs, arena)
    exp, eh = Oracle(b, 5).match(reqs, arena, nthreads=16)
    assert_verdicts_equal(got, exp, gh, eh, "decoders")
    return got


def test_decoder_kats_on_gpu(eng):
    got = _both(eng, decoder_blob(), kat_items())
    assert [int(x) for x in got["n_hits"]] == [k[5] for k in KATS]


def _encoded_items(ss, n, seed):
    rng = np.random.default_rng(seed)
    ex = [r.example for r in ss.rules if r.example]
    items = []
    for i in range(n):
        e = ex[int(rng.integers(0, len(ex)))]
        k = int(rng.integers(0, 6))
        item = {"host": "cafe.example.com", "uri": "/tea/x", "https": True}
        if k == 0:      # percent in $args
            item["args"] = "q=" + "".join("%%%02X" % c if rng.random() < 0.6 else chr(c) if 32 < c < 127 and c not in b"%+&#" else "%%%02x" % c for c in e)
        elif k == 1:    # urlenc
            item["args"] = "q=" + e.decode("latin-1").replace(" ", "+").replace("&", "%26")
        elif k == 2:    # json body
            item["headers"] = [("Content-Type", "application/json")]
            item["body"] = json.dumps({"v": e.decode("latin-1"), "pad": "x" * int(rng.integers(0, 300))}, ensure_ascii=True).encode()
        elif k == 3:    # base64 in args or body
            enc = base64.b64encode(e + b" padding-bytes").decode()
            if rng.random() < 0.5:
                item["args"] = "t=" + enc
            else:
                item["body"] = b"data=" + enc.encode()
        elif k == 4:    # form body
            item["headers"] = [("Content-Type", "application/x-www-form-urlencoded")]
            item["body"] = b"f=" + e.replace(b" ", b"+").replace(b"&", b"%26")
        else:           # benign with escapes
            item["args"] = "a=%41%42+c&b=" + "QUJDREVGR0hJSktMTU5PUA=="
        items.append(item)
    return items


@pytest.mark.parametrize("disable", ["", "base64, json_doc", "percent, urlenc"])
def test_c4_encoded_plants_parity(eng, disable):
    ss = workloads.c4_sigset()
    ss = sigs.SigSet(ss.rules, ("percent", "urlenc", "json_doc", "base64"))
    b = workloads.c4_blob(ss, "monitoring", parser_disable=disable)
    got = _both(eng, b, _encoded_items(ss, 20_000, 91 + len(disable)))
    assert int((got["n_hits"] > 0).sum()) > 5000
