#!/usr/bin/env python3
"""Exact-preconditioner parity on north_star's quantity: the engine (supernodal factor on the device) and oracle/cpu's
independent exact mode (RCM envelope Cholesky on the host) run the colour schedule in lockstep from the multi-robot
initialisation to the example's stop rule (central |RieGrad| < 0.1, examples/MultiRobotExample.cpp:229-241).  At
every check: the engine's central cost / gradient norm (dpgo_rbcd_central_eval) and the same quantities of the port's
iterate computed by numpy from the dataset's unit-weight Q (tests/_common.central_cost_gradnorm), their relative
differences, the X difference and whether any agent's Run / tCG counters differ.  Probe only; one JSON line per
check, a summary line at the end.

  python tools/exact_stop_rule.py --k 48 --robust L2 --accel 1 --check 10 --max-iters 2000"""
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
    ap.add_argument("--agents-per-axis", type=int, default=4)
    ap.add_argument("--twin", type=int, default=1, help="also run the port from X0 perturbed by 1e-15 relative")
    ap.add_argument("--robust", default="L2", choices=["L2", "GNC_TLS"])
    ap.add_argument("--accel", type=int, default=1)
    ap.add_argument("--check", type=int, default=10)
    ap.add_argument("--max-iters", type=int, default=3000)
    ap.add_argument("--tol", type=float, default=0.1)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from dpgo_amd import hip as H
    from oracle import cpu_port
    from tests._common import central_cost_gradnorm, unit_laplacian
    g = H.Graph.grid3d(a.k, seed=0)
    A = a.agents_per_axis
    aop = g.grid_partition(A)
    X0, _, _ = g.distributed_init(aop, 5, H.lifting_matrix(3, 5), gpu=True, rtol=1e-12, max_iters=50000,
                                  dev_layout=True)
    Q = unit_laplacian(g.arrays(), g.n)
    e = H.Rbcd(g, aop, np.zeros(A ** 3, np.int32), 0, 1, H.rbcd_params(
        r=5, acceleration=a.accel, robust_cost=H.ROBUST[a.robust], precon=H.PRECON_EXACT))
    e.set_X(X0)
    cpu = cpu_port.CpuRbcd(3, 5, g.arrays(), g.n, aop, A ** 3, bool(a.accel), robust=a.robust, precon="exact")
    cpu.set_X(X0)
    twin = None
    if a.twin:  # the trajectory's own sensitivity: the port from a 1e-15-perturbed start
        twin = cpu_port.CpuRbcd(3, 5, g.arrays(), g.n, aop, A ** 3, bool(a.accel), robust=a.robust, precon="exact")
        twin.set_X(X0 * (1.0 + 1e-15 * np.random.default_rng(1).standard_normal(X0.size)))
    twin_flip = None
    first_flip = None
    Xg = np.zeros(X0.size)
    rows = []
    t0 = time.time()
    it = 0
    while it < a.max_iters:
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
        cpu.iterate(threads=a.threads)
        if twin is not None:
            twin.iterate(threads=a.threads)
        it += 1
        sg, sc = e.stats()[:, 2:4], cpu.stats()[:, 2:4]
        if first_flip is None and np.any(sg != sc):
            first_flip = it
        if twin is not None and twin_flip is None and np.any(twin.stats()[:, 2:4] != sc):
            twin_flip = it
        if it % a.check:
            continue
        fg, gg = e.central_eval()
        gg = float(np.sqrt(gg.sum()))
        e.get_X_into(Xg)
        Xc = cpu.get_X()
        fc, gc = central_cost_gradnorm(Q, H.from_dev_layout(Xc, 5), 3)
        row = {"iteration": it, "f_gpu": fg, "f_cpu": fc, "f_rel": abs(fg - fc) / abs(fc), "gradnorm_gpu": gg,
               "gradnorm_cpu": gc, "gradnorm_rel": abs(gg - gc) / gc,
               "X_rel": float(np.linalg.norm(Xg - Xc) / np.linalg.norm(Xc)), "counters_equal": first_flip is None,
               "twin_counters_equal": twin_flip is None,
               "s": round(time.time() - t0, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        if twin is not None:
            Xt = twin.get_X()
            ft, gt = central_cost_gradnorm(Q, H.from_dev_layout(Xt, 5), 3)
            row.update(twin_f_rel=abs(ft - fc) / abs(fc), twin_gradnorm_rel=abs(gt - gc) / gc,
                       twin_X_rel=float(np.linalg.norm(Xt - Xc) / np.linalg.norm(Xc)))
            print(json.dumps({"iteration": it, "twin_f_rel": row["twin_f_rel"], "twin_X_rel": row["twin_X_rel"]}),
                  flush=True)
        if gg < a.tol and gc < a.tol:
            break
    summary = {"k": a.k, "agents": A ** 3, "robust": a.robust, "accel": a.accel, "iterations": it,
               "first_counter_flip": first_flip, "twin_first_counter_flip": twin_flip,
               "final": rows[-1] if rows else None}
    print(json.dumps(summary), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"summary": summary, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
