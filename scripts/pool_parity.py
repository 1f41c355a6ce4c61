"""Full-pool parity check (GPU box): the bench's C4 request pool through the HIP path and through
the CPU oracle, compared verdict by verdict and hit list by hit list.  Prints the first
mismatching requests with both hit lists.

    python scripts/pool_parity.py [--pool 1000000] [--oracle-n N]
"""

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ingress-plus_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def split_hits(v, hits):
    return [hits[int(o):int(o) + int(k)].tolist() for o, k in zip(v["first_hit_off"], v["n_hits"])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pool", type=int, default=1_000_000)
    ap.add_argument("--oracle-n", type=int, default=0)
    args = ap.parse_args()
    from gpumatch import engine, records, workloads
    from oracle_py import Oracle

    ss = workloads.c4_sigset()
    blob = workloads.c4_blob(ss, "block", sample=workloads.c4_sample(ss))   # as bench.py
    reqs, arena = records.gen_c4(args.pool, ss, seed=records.SEED_BASE + 3)
    m = args.oracle_n or len(reqs)
    e = engine.Engine(0)
    e.load(blob, 1)
    t = time.time()
    got, gh = e.match_host(reqs[:m], arena, hit_cap=8 * m + 1024)
    print(f"gpu {m} requests in {time.time() - t:.1f}s, {len(gh)} hits", flush=True)
    t = time.time()
    exp, eh = Oracle(blob, 1).match(reqs[:m], arena, nthreads=16, hit_cap=8 * m + 1024)
    print(f"oracle {m} requests in {time.time() - t:.1f}s, {len(eh)} hits", flush=True)
    bad = np.nonzero(got != exp)[0]
    print(f"verdict mismatches: {len(bad)}")
    gs, es = split_hits(got, gh), split_hits(exp, eh)
    hb = [i for i in range(m) if gs[i] != es[i]]
    print(f"hit-list mismatches: {len(hb)}")
    for i in list(bad[:5]) + hb[:10]:
        r = reqs[i]
        print(f"req {i}: gpu {got[i]} hits {gs[i]}\n        exp {exp[i]} hits {es[i]}")
        for z, f in enumerate(("uri_len", "args_len", "hdr_len", "body_len")):
            o = int(r["base"]) + sum(int(r[g]) for g in ("uri_len", "args_len", "hdr_len", "body_len")[:z])
            print(f"   zone {z} [{o}, {o + int(r[f])})")
        for rid in set(gs[i]) ^ set(es[i]):
            rl = ss.rules[rid]
            print(f"   rule {rid}: {rl.kind} nocase={rl.nocase} zones={rl.zones} pattern={rl.pattern!r}")
    sys.exit(0 if len(bad) == 0 and not hb else 1)


if __name__ == "__main__":
    main()
