#!/usr/bin/env python3
"""Exact-preconditioner step probe (C4 by default): per-step wall times after a short burn-in, and one
standalone application of the preconditioner over colour 0 timed alone (HIP events)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=48)
    ap.add_argument("--burnin", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from dpgo_amd import hip as H
    g = H.Graph.grid3d(a.k, seed=0)
    aop = g.grid_partition(4)
    eng = H.Rbcd(g, aop, np.zeros(64, np.int32), 0, 1, H.rbcd_params(r=5, acceleration=1, precon=H.PRECON_EXACT))
    s = torch.cuda.Stream()
    eng.set_stream(s.cuda_stream)
    X0, _, _ = g.distributed_init(aop, 5, H.lifting_matrix(3, 5), gpu=True, rtol=1e-12, max_iters=50000,
                                  dev_layout=True)
    eng.set_X(X0)

    def step():
        for c in range(eng.num_colors):
            eng.pre_exchange(c)
            eng.update(c, None)

    out = {}
    with torch.cuda.stream(s):
        t0 = time.time()
        step()
        torch.cuda.synchronize()
        out["first_step_s"] = time.time() - t0  # includes both colours' factorisations
        for _ in range(a.burnin):
            step()
        torch.cuda.synchronize()
        st0 = eng.stats().copy()
        per = []
        for _ in range(a.steps):
            t0 = time.perf_counter()
            step()
            torch.cuda.synchronize()
            per.append(1e3 * (time.perf_counter() - t0))
        st = (eng.stats() - st0).sum(axis=0)
    out["ms_per_step"] = per
    out["tcg_iters_per_update"] = float(st[3]) / max(float(st[0]), 1.0)
    out["runs_per_update"] = float(st[2]) / max(float(st[0]), 1.0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
