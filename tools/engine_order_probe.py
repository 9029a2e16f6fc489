#!/usr/bin/env python3
"""Probe: do identical RBCD engines built one after another in a process step at the same rate?  Builds --engines
engines of the bench workload (1M-pose grid, 64 agents, block-Jacobi), burns each in from the same distributed
initialisation, then times --steps steps per engine in alternating rounds (optionally measuring the engines in
reverse order) and prints per-engine medians of ms/step, the HVP and the standalone X.Q.  Probe only."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engines", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--burnin", type=int, default=300)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--reverse", type=int, default=0)
    a = ap.parse_args()
    import torch
    from dpgo_amd import hip as H
    dev = torch.device("cuda", 0)
    g = H.Graph.grid3d(a.k, seed=0)
    aop = g.grid_partition(4)
    X0, _, _ = g.distributed_init(aop, 5, H.lifting_matrix(3, 5), gpu=True, rtol=1e-12, max_iters=50000,
                                  dev_layout=True)
    s = torch.cuda.Stream(dev)
    engs = []
    for _ in range(a.engines):
        e = H.Rbcd(g, aop, np.zeros(64, np.int32), 0, 1, H.rbcd_params(r=5, acceleration=1))
        e.set_stream(s.cuda_stream)
        e.set_X(X0)
        engs.append(e)

    def step(e):
        for c in range(e.num_colors):
            e.pre_exchange(c)
            e.update(c, None)

    res = {i: {"ms": [], "hvp": [], "xq": []} for i in range(a.engines)}
    with torch.cuda.stream(s):
        Xb = []
        for e in engs:
            for _ in range(a.burnin):
                step(e)
            x = np.zeros(X0.size)
            e.get_X_into(x)
            Xb.append(x)
        order = list(range(a.engines))
        if a.reverse:
            order.reverse()
        for _ in range(a.rounds):
            for i in order:
                e = engs[i]
                e.set_X(Xb[i])
                step(e)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    step(e)
                torch.cuda.synchronize()
                res[i]["ms"].append(1e3 * (time.perf_counter() - t0) / a.steps)
                res[i]["hvp"].append(e.bench_hvp(0, 20))
                res[i]["xq"].append(e.bench_spmm(0, 20)[1])
    print(json.dumps({"engines": a.engines, "reverse": a.reverse,
                      "median": {i: {k: float(np.median(v)) for k, v in d.items()} for i, d in res.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
