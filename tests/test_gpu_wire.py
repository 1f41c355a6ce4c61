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
    for f in records.FIELDS:
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
    for f in ("flags", "pad0", "uri_len", "args_len", "hdr_len", "body_len", "host_len", "method_len", "ruri_len",
              "raddr_len", "port", "remote_port", "rid"):
        bad = np.nonzero((got[f] != exp[f]).reshape(n, -1).any(axis=1))[0]
        assert len(bad) == 0, (f, int(bad[0]), msgs[int(bad[0])][:120], got[int(bad[0])], exp[int(bad[0])])
    assert (got["base"] % 16 == 0).all() and (np.diff(got["base"].astype(np.int64)) >= 0).all()
    gf, ef = _fields(got, ga), _fields(exp, ea)
    for f in records.FIELDS:
        assert gf[f] == ef[f], f
    # the arena between and after the records is zero (slack is cleared: the WAF scan reads it all)
    used = np.zeros(alen, bool)
    for r in got:
        tot = sum(int(r[records.LEN_FIELD[f]]) for f in records.FIELDS)
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
