#!/usr/bin/env python3
"""A/B timing of a tuning key over the bench workload in the CG regime (1M-pose grid, 64 agents,
distributed init + burn-in): alternating rounds of `--steps` RBCD steps per value, plus the standalone
Riemannian HVP over colour 0.  Prints one JSON line per round and a summary (median ms/step per value).

  python tools/step_ab.py --key 2 --values 0 1 [--rounds 3 --steps 20 --burnin 300]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", type=int, required=True)
    ap.add_argument("--values", type=int, nargs="+", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--burnin", type=int, default=300)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--agents-per-axis", type=int, default=4)
    ap.add_argument("--precon", default="block_jacobi", choices=["block_jacobi", "exact"])
    ap.add_argument("--kernel-timing", type=int, default=0, help="sample every k-th in-step SpMM launch per mode")
    a = ap.parse_args()
    import torch
    from dpgo_amd import hip as H
    dev = torch.device("cuda", 0)
    g = H.Graph.grid3d(a.k, seed=0)
    A = a.agents_per_axis
    aop = g.grid_partition(A)
    eng = H.Rbcd(g, aop, np.zeros(A ** 3, np.int32), 0, 1, H.rbcd_params(
        r=5, acceleration=1, precon=H.PRECON_EXACT if a.precon == "exact" else H.PRECON_BLOCK_JACOBI))
    s = torch.cuda.Stream(dev)
    eng.set_stream(s.cuda_stream)
    X0, _, _ = g.distributed_init(aop, 5, H.lifting_matrix(3, 5), gpu=True, rtol=1e-12, max_iters=50000,
                                  dev_layout=True)
    eng.set_X(X0)

    def step():
        for c in range(eng.num_colors):
            eng.pre_exchange(c)
            eng.update(c, None)

    if a.kernel_timing:
        eng.set_kernel_timing(a.kernel_timing)
    kt = {v: {} for v in a.values}
    with torch.cuda.stream(s):
        for _ in range(a.burnin):
            step()
        Xb = np.zeros(X0.size)
        eng.get_X_into(Xb)
        res = {v: [] for v in a.values}
        hvp = {v: [] for v in a.values}
        xqs = {}
        fin = {}
        for rnd in range(a.rounds):
            for v in a.values:
                eng.set_tuning(a.key, v)
                eng.set_X(Xb)
                step()
                torch.cuda.synchronize()
                if a.kernel_timing:
                    eng.kernel_times()  # drop the warm-up step's samples
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    step()
                torch.cuda.synchronize()
                ms = 1e3 * (time.perf_counter() - t0) / a.steps
                if a.kernel_timing:
                    for m, (tot, cnt) in eng.kernel_times().items():
                        kt[v].setdefault(m, []).append(1e3 * tot / max(cnt, 1))
                f, _ = eng.central_eval()
                hv = eng.bench_hvp(0, 20)
                _, xq = eng.bench_spmm(0, 20)
                res[v].append(ms)
                hvp[v].append(hv)
                xqs.setdefault(v, []).append(xq)
                fin.setdefault(v, f)
                print(json.dumps({"round": rnd, "value": v, "ms_per_step": ms, "hvp_ms": hv, "f": f}), flush=True)
    print(json.dumps({"key": a.key, "median_ms_per_step": {v: float(np.median(res[v])) for v in a.values},
                      "median_hvp_ms": {v: float(np.median(hvp[v])) for v in a.values},
                      "median_xq_ms": {v: float(np.median(xqs[v])) for v in a.values},
                      "f_after": fin,
                      "median_kernel_us": {v: {m: float(np.median(x)) for m, x in kt[v].items()} for v in a.values}}),
          flush=True)


if __name__ == "__main__":
    main()
