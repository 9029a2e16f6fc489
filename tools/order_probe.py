#!/usr/bin/env python3
"""Pose order inside an agent vs the SpMM passes: the C5 grid as generated (snake order: a 64-pose tile is 2.5 lattice
rows) against the same graph relabelled so every agent's poses run in 4 x 4 x 4 lattice blocks (a tile is one block:
most neighbour gathers and record visits stay inside the tile).  Interleaved rounds in one process: the standalone
X.Q (MODE_XQ), the Riemannian HVP (MODE_HESS) and full colour-schedule steps in the CG regime.  A/B probe only."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def snake_coords(k):
    n = k ** 3
    i = np.arange(n)
    z = i // (k * k)
    idx = i % (k * k)
    idx = np.where(z & 1, k * k - 1 - idx, idx)
    y = idx // k
    x = idx % k
    x = np.where(y & 1, k - 1 - x, x)
    return x, y, z


def blocked_labels(k, A, blk):
    """new id of every pose: agents in id order, inside an agent lexicographic over (block z, y, x) then (z, y, x)."""
    x, y, z = snake_coords(k)
    s = k // A
    agent = (x // s) + A * ((y // s) + A * (z // s))
    lx, ly, lz = x % s, y % s, z % s
    key = np.lexsort((lx % blk, ly % blk, lz % blk, lx // blk, ly // blk, lz // blk, agent))
    new = np.empty(k ** 3, np.int64)
    new[key] = np.arange(k ** 3)
    return new


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--blk", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--burnin", type=int, default=200)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from dpgo_amd import hip as H
    g0 = H.Graph.grid3d(args.k, seed=0)
    a = g0.arrays()
    new = blocked_labels(args.k, 4, args.blk)
    g1 = H.Graph.from_arrays(3, g0.n, new[a["p1"]], new[a["p2"]], a["R"], a["t"], a["kappa"], a["tau"])
    aop0 = g0.grid_partition(4)
    aop1 = np.empty_like(aop0)
    aop1[new] = aop0
    YL = H.lifting_matrix(3, 5)
    engs = {}
    for name, g, aop in (("snake", g0, aop0), ("blocked", g1, aop1)):
        e = H.Rbcd(g, aop, np.zeros(64, np.int32), 0, 1, H.rbcd_params(r=5, acceleration=1))
        X0, _, _ = g.distributed_init(aop, 5, YL, gpu=True, rtol=1e-12, max_iters=50000, dev_layout=True)
        e.set_X(X0)
        for it in range(args.burnin):
            e.pre_exchange(it % 2)
            e.update(it % 2, None)
        torch.cuda.synchronize()
        engs[name] = e
    res = {n: {"xq": [], "hvp": [], "step": []} for n in engs}
    for rnd in range(args.rounds):
        for n, e in engs.items():
            _, ms = e.bench_spmm(0, args.reps)
            res[n]["xq"].append(ms)
            res[n]["hvp"].append(e.bench_hvp(0, args.reps))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for it in range(args.steps):
                e.pre_exchange(it % 2)
                e.update(it % 2, None)
            torch.cuda.synchronize()
            res[n]["step"].append(1e3 * (time.perf_counter() - t0) / (args.steps / 2))
    out = {n: {k: float(np.median(v)) for k, v in d.items()} for n, d in res.items()}
    for n, e in engs.items():
        st = e.stats()
        out[n]["tcg_iters_per_update"] = float(st[:, 3].sum() / max(st[:, 0].sum(), 1))
    print(json.dumps({"what": "median ms: xq / hvp per colour-0 launch, step = both colours", "k": args.k,
                      "blk": args.blk, "res": out}), flush=True)


if __name__ == "__main__":
    main()
