"""The N > 1 path with libgpumatch doing the classification (SURVEY.md §8 e): two ranks, each its
own process and gm_ctx, shard BASELINE's C5 stream with gpumatch.shard (the code bench.py
--config c5 runs), classify their slices on the GPU in batches and reduce the cumulative
per-location counters out of place after every step.  The single GPU of a test box hosts both
ranks, so the reduction runs over gloo (RCCL needs a device per rank; its one-rank all-reduce is
tested in test_gpu_pipeline.py).  The merged verdicts and the reduced counters must equal the
oracle's over the whole stream."""

import os
import socket

import numpy as np
import pytest

from gpumatch import engine, records, shard, workloads
from oracle_py import Oracle

pytestmark = pytest.mark.gpu

STREAM, POOL, BATCH, STEPS, N_LOCS = 60_000, 7_000, 9_000, 2, 4096


def _pool():
    return workloads.c5_blob(n_hosts=120), workloads.gen_c5(POOL, n_hosts=120)


def _rank(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    blob, (preqs, parena) = _pool()
    e = engine.Engine(0)
    e.load(blob, 1)
    lo, hi = shard.shard_bounds(STREAM, world, rank)
    reqs, plen, first, ncopies, alen = shard.stream_records(preqs, len(parena), lo, hi)
    d_pool = torch.from_numpy(np.ascontiguousarray(parena)).to(dev)
    d_arena = torch.zeros(ncopies * plen + 1024, dtype=torch.uint8, device=dev)
    for k in range(ncopies):
        d_arena[k * plen:k * plen + len(parena)].copy_(d_pool)
    d_reqs = torch.from_numpy(reqs.view(np.uint8).reshape(-1)).to(dev)
    n = hi - lo
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_hits = torch.empty(1024, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def reduce(x):
        t = torch.from_numpy(x)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.numpy()
    ctr = shard.StreamCounters(N_LOCS, reduce)

    def classify(b0, b1):
        e.match_ptr(d_reqs.data_ptr() + 64 * b0, d_arena.data_ptr(), alen, b1 - b0, d_out.data_ptr() + 32 * b0,
                    d_hits.data_ptr(), 1024, s)

    def after_step(step):
        e.sync(s)
        c = e.counters()                  # gm_counters: this rank's cumulative location counters
        ctr.local[:] = 0
        ctr.add(np.pad(c[:N_LOCS].astype(np.int64), (0, max(0, N_LOCS - len(c))))[:N_LOCS])
        tot = ctr.reduce()
        if rank == 0:
            np.save(os.path.join(out_dir, f"counters_{step}.npy"), tot)
    shard.run_stream(classify, 0, n, BATCH, after_step, steps=STEPS)
    v = d_out.cpu().numpy().view(records.VERDICT_DTYPE)
    gathered = [None] * world
    dist.all_gather_object(gathered, v.tobytes())
    if rank == 0:
        np.save(os.path.join(out_dir, "verdicts.npy"),
                np.concatenate([np.frombuffer(b, dtype=records.VERDICT_DTYPE) for b in gathered]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def test_two_ranks_one_gpu_c5_stream(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_rank, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    blob, (preqs, parena) = _pool()
    reqs, plen, _, ncopies, _ = shard.stream_records(preqs, len(parena), 0, STREAM)
    arena = np.zeros(ncopies * plen, dtype=np.uint8)
    for k in range(ncopies):
        arena[k * plen:k * plen + len(parena)] = parena
    exp, _ = Oracle(blob, 1).match(reqs, arena, nthreads=8)
    got = np.load(tmp_path / "verdicts.npy")
    bad = np.nonzero(got.view(np.uint8).reshape(-1, 32).any(axis=1) & (got != exp))[0]
    assert got.tobytes() == exp.tobytes(), f"{len(bad)} verdicts differ, first {bad[:4]}"
    loc = exp["location_id"][exp["location_id"] != 0xFFFFFFFF].astype(np.int64)
    one = np.bincount(loc, minlength=N_LOCS)
    for step in range(1, STEPS + 1):
        assert np.array_equal(np.load(tmp_path / f"counters_{step}.npy"), step * one)
