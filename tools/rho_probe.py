#!/usr/bin/env python3
"""Diagnostic: per-Run RTR trace (rho, f1 - f2, model decrease) of a few engine agents on the
synthetic grid from a chosen initialisation (GPU).  Usage: python tools/rho_probe.py --k 100 --init chordal"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--A", type=int, default=4)
    ap.add_argument("--init", default="chordal")
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--accel", type=int, default=1)
    ap.add_argument("--agents", default="0,21,42")
    a = ap.parse_args()
    from dpgo_amd import hip as H
    g = H.Graph.grid3d(a.k, seed=0)
    aop = g.grid_partition(a.A)
    YL = H.lifting_matrix(3, 5)
    X0 = g.chordal_init_gpu(5, YL, rtol=1e-10, max_iters=50000, dev_layout=True)[0] if a.init == "chordal" \
        else g.chain_init_dev_layout(5, YL)
    e = H.Rbcd(g, aop, np.zeros(a.A ** 3, np.int32), 0, 1, H.rbcd_params(r=5, acceleration=a.accel))
    e.set_X(X0)
    e.set_trace(512)
    for it in range(a.iters):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
    out = {}
    for ag in [int(x) for x in a.agents.split(",")]:
        recs = e.get_trace(ag)
        out[ag] = [{k: r[k] for k in ("op", "run", "j", "f1", "f2", "rho", "Delta", "d_Hd", "tau", "status", "accepted")}
                   for r in recs if r["op"] == 5][:40]
    print(json.dumps({"stats": e.stats().sum(axis=0).tolist(), "f": e.central_eval()[0], "runs": out}))


if __name__ == "__main__":
    main()
