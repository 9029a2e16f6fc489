"""CPU checks of the oracle itself: the reference's own known-answer tests (the only pins the
reference provides), calculus checks, and reproduction of the committed fixtures."""
import json
import os

import numpy as np
import pytest

from oracle import dpgo_oracle as O
from tests._common import GOLDEN, load_meas, random_point, random_tangent, seeded_G, rel


def _triangle():
    Tw0 = np.eye(4)
    Tw1 = np.array([[0.1436, 0.7406, 0.6564, 1], [-0.8179, -0.2845, 0.5, 1], [0.5571, -0.6087, 0.5649, 1],
                    [0, 0, 0, 1]])
    Tw2 = np.array([[-0.4069, -0.4150, -0.8138, 2], [0.4049, 0.7166, -0.5679, 2], [0.8188, -0.5606, -0.1236, 2],
                    [0, 0, 0, 1]])

    def mk(pairs):
        Rs, ts, p1, p2 = [], [], [], []
        for a, b, Ta, Tb in pairs:
            dT = np.linalg.inv(Ta) @ Tb
            Rs.append(dT[:3, :3]); ts.append(dT[:3, 3]); p1.append(a); p2.append(b)
        m = len(pairs)
        z = np.zeros(m, np.int64)
        return O.Measurements(3, z, z.copy(), np.array(p1, np.int64), np.array(p2, np.int64),
                              np.array(Rs).reshape(m, 3, 3), np.array(ts).reshape(m, 3), np.ones(m), np.ones(m),
                              np.ones(m))
    odo = mk([(0, 1, Tw0, Tw1), (1, 2, Tw1, Tw2)])
    lc = mk([(0, 2, Tw0, Tw2)])
    sh = mk([])
    return odo, lc, sh, np.hstack([Tw0[:3], Tw1[:3], Tw2[:3]])


def test_triangle_graph_fixed_point():
    """tests/testTriangleGraph.cpp:51-65 -- an exact solution stays fixed through iterate()."""
    odo, lc, sh, Ttrue = _triangle()
    ag = O.Agent(0, O.AgentParams(3, 3, 1))
    ag.set_pose_graph(odo, lc, sh)
    ag.set_X(O.lifting_matrix(3, 3) @ O.odometry_initialization(3, 3, odo))
    assert np.linalg.norm(Ttrue - ag.trajectory_local_frame()) <= 1e-4
    ag.iterate(True)
    assert ag.n == 3
    assert np.linalg.norm(Ttrue - ag.trajectory_local_frame()) <= 1e-4


def test_line_graph_runs():
    """tests/testLineGraph.cpp:7-31"""
    rng = np.random.default_rng(0)
    m = 4
    z = np.zeros(m, np.int64)
    odo = O.Measurements(3, z, z.copy(), np.arange(m), np.arange(1, m + 1), np.tile(np.eye(3), (m, 1, 1)),
                         np.tile(rng.uniform(-1, 1, 3), (m, 1)), np.ones(m), np.ones(m), np.ones(m))
    empty = odo.subset(np.zeros(m, bool))
    ag = O.Agent(0, O.AgentParams(3, 3, 1))
    ag.set_pose_graph(odo, empty, empty)
    ag.set_X(O.lifting_matrix(3, 3) @ O.odometry_initialization(3, 5, odo))
    ag.iterate(True)
    assert ag.n == 5 and ag.X.shape == (3, 20)


def test_memory_layout():
    """tests/testEigenMap.cpp:12-36 -- pose j is the contiguous r*(d+1) doubles [Y_j | p_j]."""
    r, d, n = 3, 3, 10
    X = np.zeros((r, (d + 1) * n))
    for i in range(n):
        X[:, i * 4:i * 4 + 3] = np.eye(3)
        X[:, i * 4 + 3] = [10 * i, 10 * i + 1, 10 * i + 2]
    flat = O.to_dev(X)
    for i in range(n):
        blk = flat[i * 12:(i + 1) * 12]
        assert np.array_equal(blk[:9], np.eye(3).ravel(order="F"))
        assert np.array_equal(blk[9:], [10 * i, 10 * i + 1, 10 * i + 2])
    assert np.array_equal(O.from_dev(flat, r), X)


def test_stiefel_projection():
    """tests/testUtils.cpp:12-53"""
    Y = O.lifting_matrix(3, 5)
    assert np.linalg.norm(Y.T @ Y - np.eye(3)) <= 1e-5
    rng = np.random.default_rng(1)
    for _ in range(50):
        P = O.project_to_stiefel(rng.uniform(-1, 1, (5, 3)))
        assert np.linalg.norm(P.T @ P - np.eye(3)) <= 1e-5
    X = O.lifted_project(rng.uniform(-1, 1, (5, 400)), 3)
    for i in range(100):
        Yi = X[:, 4 * i:4 * i + 3]
        assert np.linalg.norm(Yi.T @ Yi - np.eye(3)) <= 1e-5


@pytest.mark.parametrize("name,r", [("smallGrid3D", 5), ("input_INTEL_g2o", 3)])
def test_gradient_and_hessian_finite_differences(name, r):
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(O.connection_laplacian(meas, n))
    X = random_point(r, d, n, 5)
    V = random_tangent(X, d, 6)
    V /= np.linalg.norm(V)
    eps = 1e-6
    fd = (P.f(O.retract_qf(X, eps * V, d)) - P.f(O.retract_qf(X, -eps * V, d))) / (2 * eps)
    assert abs(fd - O.inner(P.riegrad(X), V)) <= 1e-5 * max(1.0, abs(fd))
    g1 = P.riegrad(O.retract_qf(X, eps * V, d))
    g0 = P.riegrad(O.retract_qf(X, -eps * V, d))
    hv = O.inner((g1 - g0) / (2 * eps), V)
    assert abs(hv - O.inner(P.rhvp(X, V), V)) <= 1e-4 * max(1.0, abs(hv))


@pytest.mark.parametrize("name,r", [("tinyGrid3D", 5), ("smallGrid3D", 5), ("smallGrid3D", 3),
                                    ("sphere2500", 5), ("input_INTEL_g2o", 5), ("input_INTEL_g2o", 2)])
def test_oracle_reproduces_eval_fixtures(name, r):
    z = np.load(os.path.join(GOLDEN, f"{name}.r{r}.eval.npz"))
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(O.connection_laplacian(meas, n))
    X = random_point(r, d, n, 11)
    V = random_tangent(X, d, 12)
    G = seeded_G(X, d, r, n, 13)
    P.set_G(G)
    got = dict(f=P.f(X), EG=P.egrad(X), HV=P.ehvp(V), RG=P.riegrad(X), RH=P.rhvp(X, V),
               PV_bj=P.precondition(X, V, O.PRECON_BLOCK_JACOBI), PV_exact=P.precondition(X, V, O.PRECON_EXACT),
               PT=O.tangent_project(X, V, d), RT=O.retract_qf(X, V, d), PP=O.lifted_project(X + 0.3 * V, d))
    for k, v in got.items():
        ref = z[k]
        if np.ndim(v) and ref.shape != np.shape(v):  # summary-only fixture: (norm, sum)
            v = np.array([np.linalg.norm(v), float(np.sum(v))])
        assert rel(v, ref) <= 1e-12, k


def test_oracle_reproduces_rtr_fixture():
    z = np.load(os.path.join(GOLDEN, "smallGrid3D.r5.rtr.npz"))
    meas = load_meas("smallGrid3D")
    P = O.QuadraticProblem(meas.num_poses, 3, 5)
    P.set_Q(O.connection_laplacian(meas, meas.num_poses))
    P.precon_mode = O.PRECON_BLOCK_JACOBI
    trace = []
    Xo, res = O.optimize(P, z["X0"], O.OptParams(tr_iterations=10, tr_tolerance=1e-1, tr_initial_radius=10.0,
                                                 tr_max_inner=50), trace)
    ref = json.loads(str(z["result"]))
    assert abs(res["fOpt"] - ref["fOpt"]) <= 1e-12 * abs(ref["fOpt"])
    assert len(trace) == z["trace"].shape[0]
    assert rel(Xo, z["Xopt"]) <= 1e-12


def test_smallgrid_converges_to_known_optimum():
    """External sanity anchor (SE-Sync literature, unverified offline): smallGrid3D optimum 2f ~ 1025.4."""
    z = np.load(os.path.join(GOLDEN, "smallGrid3D.r5.rtr.npz"))
    res = json.loads(str(z["result"]))
    assert 1024.0 < 2 * res["fOpt"] < 1027.0


def test_multirobot_log_fixture():
    z = np.load(os.path.join(GOLDEN, "smallGrid3D.multirobot5.npz"))
    log = z["log"]
    assert log.shape[0] == 30
    assert log[-1, 2] < log[0, 2]  # cost decreases from the chordal start


def test_reader_fixes_on_reference_data():
    """n = max index + 1; kitti has a blank line (no duplicate re-push)."""
    ref = "/root/reference/data"
    if not os.path.isdir(ref):
        pytest.skip("reference data not mounted (GPU box)")
    m = O.read_g2o(os.path.join(ref, "kitti_00.g2o"))
    assert m.num_poses == 4541 and m.m == 4676 and m.duplicates == 0
    m = O.read_g2o(os.path.join(ref, "smallGrid3D.g2o"))
    assert m.num_poses == 125 and np.allclose(m.kappa, 12.5) and np.allclose(m.tau, 100.0)


def test_grid3d_fixture_is_reproducible():
    z = np.load(os.path.join(GOLDEN, "grid3d_k4.npz"))
    g = O.grid3d(4, seed=0)
    assert np.array_equal(g.R, z["R"]) and np.array_equal(g.t, z["t"]) and np.array_equal(g.p1, z["p1"])
    assert g.m == 3 * 16 * 3


def test_certificate_matrix_properties():
    """Build-defined certificate (no reference counterpart): at the committed RTR optimum of
    smallGrid3D (r=5) S(X) = Q - Lambda(X) is PSD with X's rows in its null space; at a random point
    it is indefinite; X S(X) equals the Riemannian gradient."""
    meas = load_meas("smallGrid3D")
    d, n = meas.d, meas.num_poses
    Q = O.connection_laplacian(meas, n)
    z = np.load(os.path.join(GOLDEN, "smallGrid3D.r5.rtr.npz"))
    Xo = z["Xopt"]
    S = O.certificate_matrix(Q, Xo, d)
    ev = np.linalg.eigvalsh(S.toarray())
    assert ev[0] >= -1e-6 * abs(ev[-1])
    # X S(X) is the Riemannian gradient P_X(XQ) (the fixture stopped at gradnorm ~5e-2)
    P = O.QuadraticProblem(n, d, 5)
    P.set_Q(Q)
    assert rel((S @ Xo.T).T, P.riegrad(Xo)) <= 1e-9
    assert O.certificate_min_eig(S) == pytest.approx(ev[0], abs=1e-9 * abs(ev[-1]))
    X = random_point(5, d, n, 61)
    assert O.certificate_min_eig(O.certificate_matrix(Q, X, d)) < 0
