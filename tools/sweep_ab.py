#!/usr/bin/env python3
"""A/B of the exact preconditioner's sweeps under an environment switch read when the factor is built (SWEEP_ENV
names it, SWEEP_ORDERS="a,b" its values; unset: one engine, no switch): one engine per value on the same grid, standalone full applications over colour 0 alternated between them
(dpgo_rbcd_bench_precond, HIP events).  Prints one JSON line.  A/B probe only."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from dpgo_amd import hip as H
    g = H.Graph.grid3d(a.k, seed=0)
    aop = g.grid_partition(4)
    X0 = g.chain_init_dev_layout(5, H.lifting_matrix(3, 5))
    engs = {}
    dummy = None
    if os.environ.get("SWEEP_DUMMY_K"):  # a small engine built (and kept) first: tells a first-engine effect apart
        gd = H.Graph.grid3d(int(os.environ["SWEEP_DUMMY_K"]), seed=0)
        ad = gd.grid_partition(2)
        dummy = H.Rbcd(gd, ad, np.zeros(8, np.int32), 0, 1, H.rbcd_params(r=5, acceleration=1, precon=H.PRECON_EXACT))
        dummy.set_X(gd.chain_init_dev_layout(5, H.lifting_matrix(3, 5)))
        dummy.pre_exchange(0)
        dummy.update(0, None)
    for idx, order in enumerate(os.environ.get("SWEEP_ORDERS", "default").split(",")):
        if os.environ.get("SWEEP_ENV"):
            os.environ[os.environ["SWEEP_ENV"]] = order
        e = H.Rbcd(g, aop, np.zeros(64, np.int32), 0, 1, H.rbcd_params(r=5, acceleration=1, precon=H.PRECON_EXACT))
        e.set_X(X0)
        e.pre_exchange(0)
        e.update(0, None)  # builds colour 0's factor with this order
        engs[f"{order}#{idx}"] = e  # a value may repeat (engine-order checks)
    res = {o: {"fwd": [], "bwd": []} for o in engs}
    pb = 0.0
    for _ in range(a.rounds):
        items = list(engs.items())
        if os.environ.get("SWEEP_REVERSE"):  # measure the engines last-built first (order-effect checks)
            items.reverse()
        for o, e in items:
            f, b, pb = e.bench_precond(0, a.reps)
            res[o]["fwd"].append(f)
            res[o]["bwd"].append(b)
    out = {o: {k: float(np.median(v)) for k, v in d.items()} for o, d in res.items()}
    for o in out:
        out[o]["fwd_GBps"] = pb / (out[o]["fwd"] * 1e-3) / 1e9
        out[o]["bwd_GBps"] = pb / (out[o]["bwd"] * 1e-3) / 1e9
    print(json.dumps({"k": a.k, "panel_bytes": pb, "ms": out}), flush=True)


if __name__ == "__main__":
    main()
