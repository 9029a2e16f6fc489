#!/usr/bin/env python3
"""Lockstep probe of the engine's exact-preconditioner colour schedule against oracle/cpu's exact mode (C4 by
default): after every colour iteration the relative X difference, and the first iteration at which any agent's Run
or tCG counters differ.  Tells rounding growth (a smooth geometric rise) from a discrete solver decision that flips
(a jump together with a counter difference).  Probe only; prints one JSON line per checkpoint."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=48)
    ap.add_argument("--iters", type=int, default=36)
    ap.add_argument("--accel", type=int, default=0)
    ap.add_argument("--precon", default="exact", choices=["exact", "block_jacobi"])
    a = ap.parse_args()
    from dpgo_amd import hip as H
    from oracle import cpu_port
    g = H.Graph.grid3d(a.k, seed=0)
    aop = g.grid_partition(4)
    X0, _, _ = g.distributed_init(aop, 5, H.lifting_matrix(3, 5), gpu=True, rtol=1e-12, max_iters=50000,
                                  dev_layout=True)
    e = H.Rbcd(g, aop, np.zeros(64, np.int32), 0, 1, H.rbcd_params(
        r=5, acceleration=a.accel, precon=H.PRECON_EXACT if a.precon == "exact" else H.PRECON_BLOCK_JACOBI))
    e.set_X(X0)
    cpu = cpu_port.CpuRbcd(3, 5, g.arrays(), g.n, aop, 64, bool(a.accel), precon=a.precon)
    cpu.set_X(X0)
    first_flip = None
    Xg = np.zeros(X0.size)
    for it in range(a.iters):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
        cpu.iterate(threads=16)
        e.get_X_into(Xg)
        Xc = cpu.get_X()
        sg, sc = e.stats()[:, 2:4], cpu.stats()[:, 2:4]
        diff_agents = [int(x) for x in np.nonzero(np.any(sg != sc, axis=1))[0]]
        if diff_agents and first_flip is None:
            first_flip = it
        print(json.dumps({"iteration": it, "X_rel_diff": float(np.linalg.norm(Xg - Xc) / np.linalg.norm(Xc)),
                          "agents_with_different_counters": diff_agents[:8],
                          "tcg_iters_gpu": int(sg[:, 1].sum()), "tcg_iters_cpu": int(sc[:, 1].sum())}), flush=True)
    print(json.dumps({"k": a.k, "accel": a.accel, "precon": a.precon, "first_counter_flip": first_flip}), flush=True)


if __name__ == "__main__":
    main()
