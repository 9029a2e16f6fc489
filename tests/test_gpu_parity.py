"""GPU parity: HIP kernels through the C ABI vs the CPU oracle (oracle/dpgo_oracle.py).

Tolerances (north_star): per-evaluation f / grad / HVP values 1e-12 relative (Frobenius norm of
the difference over the norm of the oracle value); final cost after optimisation 1e-9 relative.
"""
import numpy as np
import pytest

from oracle import dpgo_oracle as O
from tests._common import load_meas, random_point, random_tangent, seeded_G, rel

pytestmark = pytest.mark.gpu

TOL = 1e-12


@pytest.fixture(scope="module")
def hip():
    from dpgo_amd import hip as H
    assert H.device_count() >= 1, "no gfx950 device"
    return H


CASES = [("tinyGrid3D", 5), ("smallGrid3D", 5), ("smallGrid3D", 3), ("sphere2500", 5),
         ("input_INTEL_g2o", 5), ("input_INTEL_g2o", 2), ("city10000", 3)]


@pytest.mark.parametrize("fmt", ["bsr", "edges"])
@pytest.mark.parametrize("name,r", CASES)
def test_evaluations(hip, name, r, fmt):
    """Q uploaded as BSR (QuadraticProblem::setQ) or as its measurement stream (edge records)."""
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    Q = O.connection_laplacian(meas, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(Q)
    X = random_point(r, d, n, 11)
    V = random_tangent(X, d, 12)
    G = seeded_G(X, d, r, n, 13)
    P.set_G(G)
    H = hip.Problem(n, d, r)
    if fmt == "bsr":
        H.set_Q_scipy(0, Q)
    else:
        H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
    H.set_G_dense(0, G)
    f = H.f(X)[0]
    assert abs(f - P.f(X)) <= TOL * max(1.0, abs(P.f(X)))
    assert rel(H.egrad(X), P.egrad(X)) <= TOL
    assert rel(H.ehvp(V), P.ehvp(V)) <= TOL
    RG, norms, fv = H.riegrad(X)
    assert rel(RG, P.riegrad(X)) <= TOL
    assert abs(norms[0] - P.riegrad_norm(X)) <= TOL * P.riegrad_norm(X)
    assert rel(H.rhvp(X, V), P.rhvp(X, V)) <= TOL
    assert rel(H.precondition(X, V), P.precondition(X, V, O.PRECON_BLOCK_JACOBI)) <= TOL


@pytest.mark.parametrize("name,r", [("smallGrid3D", 5), ("input_INTEL_g2o", 2), ("sphere2500", 3)])
def test_manifold_ops(hip, name, r):
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    X = random_point(r, d, n, 21)
    V = random_tangent(X, d, 22)
    assert rel(hip.tangent_project(X, V + X, d), O.tangent_project(X, V + X, d)) <= TOL
    assert rel(hip.retract_qf(X, V, d), O.retract_qf(X, V, d)) <= 1e-13
    assert rel(hip.retract_qf(X, V, d, scale=-0.25), O.retract_qf(X, -0.25 * V, d)) <= 1e-13
    for eps in (0.3, 0.01, 2.0):  # Jacobi fallback / Newton-Schulz fast path / far from St(d,r)
        M = X + eps * V
        assert rel(hip.project_polar(M, d), O.lifted_project(M, d)) <= 1e-13


def _single_rtr(hip, name, r, iters, tol, radius, inner):
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    Q = O.connection_laplacian(meas, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(Q)
    P.precon_mode = O.PRECON_BLOCK_JACOBI
    X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
    trace = []
    Xo, res = O.optimize(P, X0, O.OptParams(tr_iterations=iters, tr_tolerance=tol,
                                            tr_initial_radius=radius, tr_max_inner=inner), trace)
    H = hip.Problem(n, d, r)
    H.set_Q_scipy(0, Q)
    p = hip.default_params(tr_iterations=iters, tr_tolerance=tol, tr_initial_radius=radius,
                           tr_max_inner=inner, precon=hip.PRECON_BLOCK_JACOBI)
    Xh, rh = H.optimize(X0, p)
    return Xo, res, trace, Xh, rh[0]


@pytest.mark.parametrize("name,r", [("smallGrid3D", 5), ("tinyGrid3D", 3), ("sphere2500", 3)])
def test_rtr_single_agent(hip, name, r):
    """PGOAgent::localPoseGraphOptimization settings (src/PGOAgent.cpp:975-984)."""
    Xo, res, trace, Xh, rh = _single_rtr(hip, name, r, 10, 1e-1, 10.0, 50)
    assert abs(rh["fInit"] - res["fInit"]) <= 1e-12 * abs(res["fInit"])
    assert abs(rh["fOpt"] - res["fOpt"]) <= 1e-9 * abs(res["fOpt"])
    assert rh["outer_iters"] == len(trace)
    assert rh["tCGStatus"] == res["tCGStatus"]
    assert rel(Xh, Xo) <= 1e-8


def test_rtr_rbcd_settings(hip):
    """PGOAgent::updateX settings: 1 iteration, 10 inner, radius 100, tol 1e-2 (:1131-1137)."""
    Xo, res, trace, Xh, rh = _single_rtr(hip, "smallGrid3D", 5, 1, 1e-2, 100.0, 10)
    assert rh["runs"] == res["runs"]
    assert abs(rh["fOpt"] - res["fOpt"]) <= 1e-11 * abs(res["fOpt"])
    assert abs(rh["gradNormOpt"] - res["gradNormOpt"]) <= 1e-9 * res["gradNormOpt"]
    assert abs(rh["relativeChange"] - res["relativeChange"]) <= 1e-9 * res["relativeChange"]
    assert rel(Xh, Xo) <= 1e-10


def test_batched_agents_match_independent(hip):
    """A batch of agents = independent QuadraticProblems solved in one set of launches."""
    meas = load_meas("smallGrid3D")
    d, r = 3, 5
    parts, robot_of, local, start = O.partition_contiguous(meas, meas.num_poses, 5)
    X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, meas.num_poses, meas)
    b = d + 1
    H = hip.Problem(None, d, r, poses_per_agent=[int(start[k + 1] - start[k]) for k in range(5)])
    oracle_out = []
    for k in range(5):
        ag = O.Agent(k, O.AgentParams(d, r, 5, robust="L2", precon=O.PRECON_BLOCK_JACOBI))
        ag.set_pose_graph(*parts[k], n=int(start[k + 1] - start[k]))
        ag.set_X(X0[:, start[k] * b:start[k + 1] * b])
        nd = {}
        for j in range(5):
            if j != k:
                nd.update({pid: X0[:, (start[pid[0]] + pid[1]) * b:(start[pid[0]] + pid[1] + 1) * b]
                           for pid in ag.neighbor_shared if pid[0] == j})
        ag.neighbor_pose = nd
        assert ag.construct_G(nd)
        H.set_Q_scipy(k, ag.problem.Q)
        H.set_G_dense(k, ag.problem.G)
        Xk, rk = O.optimize(ag.problem, ag.X, O.OptParams(tr_iterations=1, tr_tolerance=1e-2,
                                                          tr_initial_radius=100.0, tr_max_inner=10))
        oracle_out.append((Xk, rk))
    Xh, rh = H.optimize(X0, hip.default_params(tr_iterations=1, tr_tolerance=1e-2,
                                               tr_initial_radius=100.0, tr_max_inner=10))
    for k in range(5):
        Xk, rk = oracle_out[k]
        assert abs(rh[k]["fOpt"] - rk["fOpt"]) <= 1e-10 * max(1.0, abs(rk["fOpt"]))
        assert rel(Xh[:, start[k] * b:start[k + 1] * b], Xk) <= 1e-10


@pytest.mark.parametrize("want_results", [True, False])
def test_first_step_prediction_paths(hip, want_results):
    """The first tCG step is evaluated as <delta, Hess delta> alone (MODE_QF) while the previous call's
    first step stopped every agent; agents that take a CG step then get Hess[delta] (and the
    gradient) recomputed, and their candidate / rho test follow the boundary agents' speculative
    ones.  A batch mixing a near-optimal agent (CG steps) with far-off agents (boundary steps), over
    repeated calls on one handle, must match independent oracle solves every time."""
    import torch
    meas = load_meas("smallGrid3D")
    d, r, n = 3, 5, meas.num_poses
    b = d + 1
    Q = O.connection_laplacian(meas, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(Q)
    P.precon_mode = O.PRECON_BLOCK_JACOBI
    good = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
    Xs = [good, random_point(r, d, n, 31), random_point(r, d, n, 32)]
    H = hip.Problem(None, d, r, poses_per_agent=[n] * len(Xs))
    for k in range(len(Xs)):
        H.set_Q_scipy(k, Q)
    p = hip.default_params(tr_iterations=1, tr_tolerance=1e-2, tr_initial_radius=100.0, tr_max_inner=10,
                           precon=hip.PRECON_BLOCK_JACOBI)
    op = O.OptParams(tr_iterations=1, tr_tolerance=1e-2, tr_initial_radius=100.0, tr_max_inner=10)
    dev = torch.device("cuda", 0)
    kinds = set()
    for call in range(6):
        if call == 4:  # every agent far off: the prediction turns back to "first step stops" (call 5)
            Xs[0] = random_point(r, d, n, 33)
        xin = torch.from_numpy(hip.to_dev_layout(np.hstack(Xs))).to(dev)
        xout = torch.empty_like(xin)
        H.optimize_dev(xin.data_ptr(), xout.data_ptr(), p, want_results=want_results)
        torch.cuda.synchronize()
        Xh = hip.from_dev_layout(xout.cpu().numpy(), r)
        for k in range(len(Xs)):
            trace = []
            Xk, rk = O.optimize(P, Xs[k], op, trace)
            outer = [t for t in trace if "ninner" in t]
            if outer:  # tCG ran: did its first step end it?
                kinds.add(outer[0]["ninner"] == 1 and outer[0]["status"] in (O.TCG_NEGCURVTURE, O.TCG_EXCREGION))
            assert rel(Xh[:, k * n * b:(k + 1) * n * b], Xk) <= 1e-10, (call, k)
            Xs[k] = Xk
    assert kinds == {True, False}  # both kinds of first step occurred


def _agent_edges(meas, robot_of, local, k):
    """Agent k's measurement stream: private edges with local endpoints, shared edges with the
    foreign endpoint = -1 (PGOAgent::constructQMatrix, src/PGOAgent.cpp:720-781)."""
    sel = np.nonzero((robot_of[meas.p1] == k) | (robot_of[meas.p2] == k))[0]
    p1 = np.where(robot_of[meas.p1[sel]] == k, local[meas.p1[sel]], -1)
    p2 = np.where(robot_of[meas.p2[sel]] == k, local[meas.p2[sel]], -1)
    return sel, p1, p2


@pytest.mark.parametrize("name,r,robots", [("smallGrid3D", 5, 5), ("input_INTEL_g2o", 5, 4)])
def test_agent_edge_stream_matches_agent_Q(hip, name, r, robots):
    """Per-agent Q from the edge stream (shared edges: diagonal terms only) = the oracle's
    PGOAgent Q; batched over all agents in one handle, f / EucGrad / HVP / RieGrad / precond."""
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    b = d + 1
    parts, robot_of, local, start = O.partition_contiguous(meas, n, robots)
    X = random_point(r, d, n, 31)
    V = random_tangent(X, d, 32)
    H = hip.Problem(None, d, r, poses_per_agent=[int(start[k + 1] - start[k]) for k in range(robots)])
    probs = []
    for k in range(robots):
        ag = O.Agent(k, O.AgentParams(d, r, robots, robust="L2", precon=O.PRECON_BLOCK_JACOBI))
        ag.set_pose_graph(*parts[k], n=int(start[k + 1] - start[k]))
        sel, p1, p2 = _agent_edges(meas, robot_of, local, k)
        H.set_Q_edges(k, p1, p2, meas.R[sel], meas.t[sel], meas.kappa[sel], meas.tau[sel])
        G = seeded_G(X[:, start[k] * b:start[k + 1] * b], d, r, int(start[k + 1] - start[k]), 40 + k)
        ag.problem.set_G(G)
        H.set_G_dense(k, G)
        probs.append(ag.problem)
    fh = H.f(X)
    EG, HV = H.egrad(X), H.ehvp(V)
    RG, norms, _ = H.riegrad(X)
    PC = H.precondition(X, V)
    for k in range(robots):
        sl = slice(start[k] * b, start[k + 1] * b)
        P = probs[k]
        Xk, Vk = X[:, sl], V[:, sl]
        assert abs(fh[k] - P.f(Xk)) <= TOL * max(1.0, abs(P.f(Xk)))
        assert rel(EG[:, sl], P.egrad(Xk)) <= TOL
        assert rel(HV[:, sl], P.ehvp(Vk)) <= TOL
        assert rel(RG[:, sl], P.riegrad(Xk)) <= TOL
        assert abs(norms[k] - P.riegrad_norm(Xk)) <= TOL * P.riegrad_norm(Xk)
        assert rel(PC[:, sl], P.precondition(Xk, Vk, O.PRECON_BLOCK_JACOBI)) <= TOL


def test_edge_stream_rejects_bad_input(hip):
    H = hip.Problem(4, 3, 5)
    R = np.tile(np.eye(3), (1, 1, 1))
    with pytest.raises(hip.DPGOHipError):
        H.set_Q_edges(0, [0], [0], R, np.zeros((1, 3)), [1.0], [1.0])  # self-loop
    with pytest.raises(hip.DPGOHipError):
        H.set_Q_edges(0, [0], [7], R, np.zeros((1, 3)), [1.0], [1.0])  # out of range
    with pytest.raises(hip.DPGOHipError):
        H.set_Q_edges(0, [-1], [-1], R, np.zeros((1, 3)), [1.0], [1.0])  # no local endpoint


@pytest.mark.parametrize("name,r", [("smallGrid3D", 5), ("input_INTEL_g2o", 3)])
def test_device_reweighting_matches_host_weights(hip, name, r):
    """dpgo_hip_set_edge_weights_dev (on-device Q rebuild after a GNC update) gives bitwise the
    problem built on the host with the same weights, and matches the oracle's weighted Q; the exact
    preconditioner follows the new weights."""
    import torch
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    w = np.array([O.SplitMix64(900 + e).uniform() for e in range(meas.m)])
    X = random_point(r, d, n, 61)
    V = random_tangent(X, d, 62)
    Hh = hip.Problem(n, d, r)
    Hh.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, w)
    Hd = hip.Problem(n, d, r)
    Hd.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau)
    Hd.f(X)  # upload the unweighted problem first
    wd = torch.tensor(w, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    Hd.set_edge_weights_dev(wd.data_ptr())
    assert np.array_equal(Hd.egrad(X), Hh.egrad(X))
    assert np.array_equal(Hd.rhvp(X, V), Hh.rhvp(X, V))
    assert np.array_equal(Hd.precondition(X, V), Hh.precondition(X, V))
    mw = O.Measurements(meas.d, meas.r1, meas.r2, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, w, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(O.connection_laplacian(mw, n))
    assert rel(Hd.egrad(X), P.egrad(X)) <= TOL
    Hd.set_precon(hip.PRECON_EXACT)
    assert rel(Hd.precondition(X, V), P.precondition(X, V, O.PRECON_EXACT)) <= 1e-10
