"""Histogram of per-agent RTR statistics (tCG status, inner iterations, Runs) over the bench
workload's RBCD steps: which tCG exits dominate decides which passes are worth fusing."""
import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--steps", type=int, default=12)
    args = ap.parse_args()
    import torch
    from dpgo_amd import hip as H
    torch.cuda.set_device(0)
    g = H.Graph.grid3d(args.k, seed=0)
    aop = g.grid_partition(4)
    eng = H.Rbcd(g, aop, [0] * 64, 0, 1, H.rbcd_params(r=5, acceleration=1, robust_cost=H.ROBUST["L2"]))
    eng.set_X(g.chain_init_dev_layout(5, H.lifting_matrix(3, 5)))
    hist = collections.Counter()
    per_step = []
    for s in range(args.steps):
        step = collections.Counter()
        for c in range(eng.num_colors):
            eng.pre_exchange(c)
            for r in eng.update(c, None, want_results=True):
                key = (r["tCGStatus"], r["inner_iters"], r["runs"])
                hist[key] += 1
                step[key] += 1
        per_step.append({str(k): v for k, v in sorted(step.items())})
    print(json.dumps({"key": "(tCGStatus, inner_iters, runs)",
                      "total": {str(k): v for k, v in sorted(hist.items())}, "per_step": per_step}, indent=1))


if __name__ == "__main__":
    main()
