#!/usr/bin/env python3
"""A/B the X.Q SpMM variants (edge-stream or BSR Q) in ONE process, interleaved rounds (cdna_hip_programming.md 5.4 rule 24).
Workload: one colour class of the C5 problem (grid3d k=100, 64 agents -> 32 agents, 500k poses)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--qfmt", default="edges", choices=["edges", "bsr"])
    args = ap.parse_args()
    from dpgo_amd import hip as H
    g = H.Graph.grid3d(args.k, seed=0)
    aop = g.grid_partition(4)
    qf = H.QFMT_EDGES if args.qfmt == "edges" else H.QFMT_BSR
    key = 1 if args.qfmt == "edges" else 0
    eng = H.Rbcd(g, aop, np.zeros(64, np.int32), 0, 1, H.rbcd_params(r=5, acceleration=1, q_format=qf))
    eng.set_X(g.chain_init_dev_layout(5, H.lifting_matrix(3, 5)))
    variants = [int(v) for v in args.variants.split(",")]
    res = {v: [] for v in variants}
    for rnd in range(args.rounds):
        for v in variants:
            eng.set_tuning(key, v)
            b, ms = eng.bench_spmm(0, args.reps)
            res[v].append(ms)
    eng.set_tuning(key, -1 if key == 1 else 0)
    out = {}
    for v in variants:
        t = np.array(res[v])
        out[v] = dict(median_us=1e3 * float(np.median(t)), min_us=1e3 * float(t.min()),
                      GBps=b / (np.median(t) * 1e-3) / 1e9)
    # achievable-bandwidth calibration: device-to-device copy of the same byte count (read + write)
    import torch
    n = int(b // 16)
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    x.fill_(1.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        y.copy_(x)
    e0.record()
    for _ in range(20):
        y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    copy_gbs = 2 * n * 8 / (e0.elapsed_time(e1) / 20 * 1e-3) / 1e9
    bsr_b, fmt_b = eng.spmm_bytes(0)
    print(json.dumps({"qfmt": args.qfmt, "bytes": b, "bsr_bytes": bsr_b, "format_bytes": fmt_b, "variants": out,
                      "d2d_copy_GBps": copy_gbs}))


if __name__ == "__main__":
    main()
