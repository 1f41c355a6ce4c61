"""The upstream request URI (§8 f1, nginx.org/rewrites) on the GPU: raw HTTP/1.x bytes ->
gm_parse_requests -> gm_match_batch -> gm_upstream_uris, every step on the device, against the
oracle's chain (orc_parse_requests -> orc_match -> orc_upstream_uris) on the same bytes: the
README KATs of examples/rewrites plus 100k random paths (%-escapes, dot segments, '//', '?',
'#', NUL) under the rewritten and the plain locations."""

import numpy as np
import pytest

from gpumatch import engine, records, wire
from oracle_py import Oracle, parse_requests, upstream_uris, uri_list
from test_rewrites import KATS, cafe_rewrites_blob
from test_uri import random_paths

pytestmark = pytest.mark.gpu


def _targets(n, seed):
    rng = np.random.default_rng(seed)
    pre = [b"/tea", b"/coffee", b"/juice", b"/coffee/", b"/tea/", b""]
    out = []
    for p in random_paths(n, seed):
        out.append(pre[int(rng.integers(0, len(pre)))] + p)
    return out


def test_gpu_upstream_uris_parity():
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    dev = torch.device("cuda", 0)
    b = cafe_rewrites_blob()
    targets = [t.encode() for t, _ in KATS] + _targets(100_000, 31)
    msgs = [b"GET " + t + b" HTTP/1.1\r\nHost: cafe.example.com\r\n\r\n" for t in targets]
    w, m = wire.build(msgs, [{"https": False, "port": 80}] * len(msgs))
    n = len(m)
    # oracle chain
    oreqs, oarena = parse_requests(w, m)
    o = Oracle(b, 1)
    ov, _ = o.match(oreqs, oarena, nthreads=16)
    oout, ooff, oln = upstream_uris(o, oreqs, oarena, ov)
    exp = uri_list(oout, ooff, oln)
    # device chain
    e = engine.Engine(0)
    e.load(b, 1)
    s = torch.cuda.current_stream().cuda_stream
    d_w = torch.from_numpy(w).to(dev)
    d_m = torch.from_numpy(m.view(np.uint8).reshape(-1)).to(dev)
    cap = wire.arena_bound(m)
    d_reqs = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    d_arena = torch.empty(cap + 1024, dtype=torch.uint8, device=dev)
    d_alen = torch.zeros(1, dtype=torch.int64, device=dev)
    d_v = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_hits = torch.empty(1 << 16, dtype=torch.int32, device=dev)
    ucap = 4 * cap + 64 * n
    d_u = torch.empty(ucap, dtype=torch.uint8, device=dev)
    d_uoff = torch.empty(n, dtype=torch.int64, device=dev)
    d_ulen = torch.empty(n, dtype=torch.int32, device=dev)
    e.parse_ptr(d_w.data_ptr(), d_m.data_ptr(), n, d_reqs.data_ptr(), d_arena.data_ptr(), cap, d_alen.data_ptr(), s)
    e.match_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), cap, n, d_v.data_ptr(), d_hits.data_ptr(), 1 << 16, s,
                arena_len_dev=d_alen.data_ptr())
    e.upstream_uris_ptr(d_reqs.data_ptr(), d_arena.data_ptr(), cap, n, d_v.data_ptr(), d_u.data_ptr(), ucap,
                        d_uoff.data_ptr(), d_ulen.data_ptr(), s)
    e.sync(s)
    gv = d_v.cpu().numpy().view(records.VERDICT_DTYPE)
    assert np.array_equal(gv["action"], ov["action"]) and np.array_equal(gv["location_id"], ov["location_id"])
    got = uri_list(d_u.cpu().numpy(), d_uoff.cpu().numpy().view(np.uint64), d_ulen.cpu().numpy().view(np.uint32))
    for i in range(len(KATS)):
        assert got[i] == KATS[i][1], (KATS[i], got[i])
    bad = [i for i in range(n) if got[i] != exp[i]]
    assert not bad, f"{len(bad)} upstream URIs differ; first {targets[bad[0]]!r}: {got[bad[0]]!r} vs {exp[bad[0]]!r}"
    kinds = {"none": sum(x is None for x in got), "uri": sum(isinstance(x, bytes) for x in got)}
    assert kinds["none"] > 1000 and kinds["uri"] > 30_000, kinds
