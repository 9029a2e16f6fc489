#!/usr/bin/env python3
"""Diagnostic: the engine's first update of one agent of the synthetic grid against the oracle's
QuadraticOptimizer on the same agent problem (Q, G from the neighbours' initial poses).
Usage (GPU box): python tools/agent_probe.py --k 100 --agent 42 --init chordal"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--A", type=int, default=4)
    ap.add_argument("--agent", type=int, default=42)
    ap.add_argument("--init", default="chordal")
    ap.add_argument("--accel", type=int, default=0)
    a = ap.parse_args()
    from dpgo_amd import hip as H
    from oracle import dpgo_oracle as O
    t0 = time.time()
    g = H.Graph.grid3d(a.k, seed=0)
    aop = g.grid_partition(a.A)
    r, d, b = 5, 3, 4
    YL = H.lifting_matrix(3, r)
    if a.init == "chordal":
        X0f = g.chordal_init_gpu(r, YL, rtol=1e-10, max_iters=50000, dev_layout=True)[0]
    else:
        X0f = g.chain_init_dev_layout(r, YL)
    e = H.Rbcd(g, aop, np.zeros(a.A ** 3, np.int32), 0, 1, H.rbcd_params(r=r, acceleration=a.accel))
    e.set_X(X0f)
    e.set_trace(64)
    col = e.color_of_agent[a.agent]
    e.pre_exchange(col)
    e.update(col, None)
    got = [x for x in e.get_trace(a.agent)]
    # oracle agent problem
    arr = g.arrays()
    meas = O.Measurements(3, np.zeros(g.m, np.int64), np.zeros(g.m, np.int64), arr["p1"].astype(np.int64),
                          arr["p2"].astype(np.int64), arr["R"], arr["t"], arr["kappa"], arr["tau"], np.ones(g.m), g.n)
    n = g.n
    local = np.zeros(n, np.int64)
    cnt = np.zeros(a.A ** 3, np.int64)
    for i in range(n):
        local[i] = cnt[aop[i]]
        cnt[aop[i]] += 1
    X0 = H.from_dev_layout(X0f, r)
    sel = np.nonzero((aop[meas.p1] == a.agent) | (aop[meas.p2] == a.agent))[0]
    sub = meas.subset(sel)
    sub.r1 = aop[sub.p1].astype(np.int64)
    sub.r2 = aop[sub.p2].astype(np.int64)
    gp1, gp2 = sub.p1.copy(), sub.p2.copy()
    sub.p1 = local[gp1]
    sub.p2 = local[gp2]
    priv = (sub.r1 == a.agent) & (sub.r2 == a.agent)
    odo = priv & (sub.p2 == sub.p1 + 1)
    ag = O.Agent(a.agent, O.AgentParams(3, r, a.A ** 3, robust="L2", precon=O.PRECON_BLOCK_JACOBI))
    ag.set_pose_graph(sub.subset(np.nonzero(odo)[0]), sub.subset(np.nonzero(priv & ~odo)[0]),
                      sub.subset(np.nonzero(~priv)[0]), n=int(cnt[a.agent]))
    mine = np.nonzero(aop == a.agent)[0]
    cols = np.concatenate([np.arange(p * b, (p + 1) * b) for p in mine])
    Xa = X0[:, cols]
    nd = {}
    for (rb, pl) in ag.neighbor_shared:
        gi = np.nonzero((aop == rb) & (local == pl))[0][0]
        nd[(rb, pl)] = X0[:, gi * b:(gi + 1) * b]
    assert ag.construct_G(nd)
    trace = []
    Xo, res = O.optimize(ag.problem, Xa, O.OptParams(tr_iterations=1, tr_tolerance=1e-2, tr_initial_radius=100.0,
                                                     tr_max_inner=10), trace)
    fxa = ag.problem.f(Xa)
    out = {"oracle_f_x1": fxa, "oracle_runs": [{k: t[k] for k in ("f1", "f2", "rho", "Delta", "status", "ninner")}
                                               for t in trace][:6],
           "engine_runs": [{k: x[k] for k in ("f1", "f2", "rho", "Delta", "status")} for x in got if x["op"] == 5][:6],
           "engine_steps": [{k: x[k] for k in ("j", "d_Hd", "alpha", "tau", "status")} for x in got if x["op"] == 3][:6],
           "oracle_steps": [{k: s.get(k) for k in ("j", "d_Hd", "alpha", "tau", "status")} for t in trace for s in t["tcg"]][:6],
           "seconds": time.time() - t0}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
