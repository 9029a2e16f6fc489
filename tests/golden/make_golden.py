"""Generate the committed golden fixtures (run in the build container, where the reference's
data/ directory is mounted at /root/reference).

Fixtures are DATA: the measurement arrays parsed from the reference's g2o inputs (so tests run on
the GPU box, where /root/reference does not exist) plus oracle outputs at seeded points.  The
oracle is oracle/dpgo_oracle.py (a CPU restatement; see its header for the parity status).

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import dpgo_oracle as O  # noqa: E402

REF_DATA = "/root/reference/data"
DATASETS = ["tinyGrid3D", "smallGrid3D", "sphere2500", "torus3D", "input_INTEL_g2o", "CSAIL",
            "kitti_00", "city10000"]


def save_meas(name, meas):
    np.savez_compressed(os.path.join(HERE, f"{name}.meas.npz"), d=meas.d, n=meas.num_poses,
                        r1=meas.r1, r2=meas.r2, p1=meas.p1, p2=meas.p2, R=meas.R, t=meas.t,
                        kappa=meas.kappa, tau=meas.tau, duplicates=meas.duplicates)


def load_meas(name):
    z = np.load(os.path.join(HERE, f"{name}.meas.npz"))
    m = O.Measurements(int(z["d"]), z["r1"], z["r2"], z["p1"], z["p2"], z["R"], z["t"],
                       z["kappa"], z["tau"], np.ones(len(z["p1"])), int(z["n"]), int(z["duplicates"]))
    return m


def random_point(r, d, n, seed):
    rng = O.SplitMix64(seed)
    M = np.array([[rng.normal() for _ in range((d + 1) * n)] for _ in range(r)])
    return O.lifted_project(M, d)


def random_tangent(X, d, seed):
    rng = O.SplitMix64(seed)
    V = np.array([[rng.normal() for _ in range(X.shape[1])] for _ in range(X.shape[0])])
    return O.tangent_project(X, V, d)


def eval_fixture(name, meas, r, seed):
    d, n = meas.d, meas.num_poses
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(O.connection_laplacian(meas, n))
    X = random_point(r, d, n, seed)
    V = random_tangent(X, d, seed + 1)
    # a G with a few nonzero pose blocks (as constructGMatrix produces for public poses)
    G = np.zeros_like(X)
    rng = O.SplitMix64(seed + 2)
    for j in range(0, n, max(1, n // 7)):
        for c in range(d + 1):
            for a in range(r):
                G[a, j * (d + 1) + c] = rng.normal()
    P.set_G(G)
    out = dict(X=X, V=V, G=G, f=P.f(X), EG=P.egrad(X), HV=P.ehvp(V), RG=P.riegrad(X),
               RH=P.rhvp(X, V), PV_bj=P.precondition(X, V, O.PRECON_BLOCK_JACOBI),
               PV_exact=P.precondition(X, V, O.PRECON_EXACT),
               PT=O.tangent_project(X, V, d), RT=O.retract_qf(X, V, d),
               PP=O.lifted_project(X + 0.3 * V, d))
    if n > 200:  # large graphs: keep a summary only (tests recompute the oracle live)
        out = {k: (np.array([np.linalg.norm(v), float(np.sum(v))]) if np.ndim(v) else v)
               for k, v in out.items()}
    np.savez_compressed(os.path.join(HERE, f"{name}.r{r}.eval.npz"), **out)


def rtr_fixture(name, meas, r, precon, iters, tol, radius, inner):
    d, n = meas.d, meas.num_poses
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(O.connection_laplacian(meas, n))
    P.precon_mode = precon
    X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
    trace = []
    Xo, res = O.optimize(P, X0, O.OptParams(tr_iterations=iters, tr_tolerance=tol,
                                            tr_initial_radius=radius, tr_max_inner=inner), trace)
    rows = [(t["iter"], t["f1"], t["f2"], t["rho"], t["Delta"], int(t["accepted"]), t["ngf"],
             t["status"], t["ninner"]) for t in trace]
    tcg = [[(c["j"], c["d_Hd"], c["alpha"]) for c in t["tcg"]] for t in trace]
    np.savez_compressed(os.path.join(HERE, f"{name}.r{r}.rtr.npz"), X0=X0, Xopt=Xo,
                        trace=np.array(rows, dtype=float),
                        tcg0=np.array(tcg[0], dtype=float) if tcg else np.zeros((0, 3)),
                        result=json.dumps({k: (float(v) if v is not None else None)
                                           for k, v in res.items()}))


def multirobot_exact(meas):
    """The same loop with the reference's own preconditioner (exact factor of Q + 0.1 I), which the
    C++ drop-in uses by default."""
    log, Xf = O.multi_robot_example(meas, 5, num_iters=30, precon=O.PRECON_EXACT)
    np.savez_compressed(os.path.join(HERE, "smallGrid3D.multirobot5.exact.npz"),
                        log=np.array(log, dtype=float), Xfinal=Xf)


def main():
    for name in DATASETS:
        meas = O.read_g2o(os.path.join(REF_DATA, f"{name}.g2o"))
        save_meas(name, meas)
        print(name, meas.m, meas.num_poses, "dups", meas.duplicates)
    for name, r in [("tinyGrid3D", 5), ("smallGrid3D", 5), ("smallGrid3D", 3), ("sphere2500", 5),
                    ("input_INTEL_g2o", 5), ("input_INTEL_g2o", 2)]:
        eval_fixture(name, load_meas(name), r, seed=11)
    rtr_fixture("smallGrid3D", load_meas("smallGrid3D"), 5, O.PRECON_BLOCK_JACOBI, 10, 1e-1, 10.0, 50)
    rtr_fixture("tinyGrid3D", load_meas("tinyGrid3D"), 3, O.PRECON_BLOCK_JACOBI, 10, 1e-1, 10.0, 50)
    # multi-robot serialized example (config 1): 5 robots on smallGrid3D, block-Jacobi, 30 its
    meas = load_meas("smallGrid3D")
    log, Xf = O.multi_robot_example(meas, 5, num_iters=30, precon=O.PRECON_BLOCK_JACOBI)
    np.savez_compressed(os.path.join(HERE, "smallGrid3D.multirobot5.npz"),
                        log=np.array(log, dtype=float), Xfinal=Xf)
    multirobot_exact(meas)
    # plain-text copies for the C++ test program (tests/cpp/test_dpgo.cpp)
    with open(os.path.join(HERE, "smallGrid3D.meas.txt"), "w") as f:
        f.write(f"{meas.d} {meas.num_poses} {meas.m}\n")
        for e in range(meas.m):
            vals = [int(meas.p1[e]), int(meas.p2[e])] + [f"{x:.17g}" for x in meas.R[e].ravel()] + \
                   [f"{x:.17g}" for x in meas.t[e]] + [f"{meas.kappa[e]:.17g}", f"{meas.tau[e]:.17g}"]
            f.write(" ".join(str(v) for v in vals) + "\n")
    X0 = O.lifting_matrix(3, 5) @ O.chordal_initialization(3, meas.num_poses, meas)
    with open(os.path.join(HERE, "smallGrid3D.X0.txt"), "w") as f:
        f.write(f"{X0.shape[0]} {X0.shape[1]}\n")
        for row in X0:
            f.write(" ".join(f"{x:.17g}" for x in row) + "\n")
    # synthetic grid (bitwise contract with the C++ generator)
    g = O.grid3d(4, seed=0)
    np.savez_compressed(os.path.join(HERE, "grid3d_k4.npz"), p1=g.p1, p2=g.p2, R=g.R, t=g.t,
                        gt=g.extra["ground_truth"])


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "multirobot_exact":
        multirobot_exact(load_meas("smallGrid3D"))
    else:
        main()
