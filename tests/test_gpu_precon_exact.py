"""GPU parity of the exact preconditioner: the reference factorises
P = Q + 0.1 I with CHOLMOD in QuadraticProblem::setQ (src/QuadraticProblem.cpp:37-41) and applies
P_X(V P^-1) in PreConditioner (:75-87).  Here: nested-dissection symbolic tree on the host (once per pattern),
supernodal numeric factorisation on the device (fp64 MFMA tiles) and per-level panel sweeps (k_sn_fwd / k_sn_bwd),
against the oracle's sparse LU solve and against the host numeric factorisation of the same tree.

Tolerances: the two factorisations order and round differently, so single applications agree to
cond(P) * eps (bar 1e-10 relative); full RTR runs with the exact preconditioner to 1e-9 on the final
cost with identical outer-iteration counts and tCG status."""
import numpy as np
import pytest

from oracle import dpgo_oracle as O
from tests._common import load_meas, random_point, random_tangent, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    from dpgo_amd import hip as H
    assert H.device_count() >= 1, "no gfx950 device"
    return H


@pytest.mark.parametrize("fmt", ["bsr", "edges"])
@pytest.mark.parametrize("name,r", [("tinyGrid3D", 5), ("smallGrid3D", 5), ("smallGrid3D", 3),
                                    ("sphere2500", 3), ("input_INTEL_g2o", 2), ("input_INTEL_g2o", 5)])
def test_exact_precondition(hip, name, r, fmt):
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    Q = O.connection_laplacian(meas, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(Q)
    X = random_point(r, d, n, 51)
    V = random_tangent(X, d, 52)
    H = hip.Problem(n, d, r)
    if fmt == "bsr":
        H.set_Q_scipy(0, Q)
    else:
        H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
    H.set_precon(hip.PRECON_EXACT)
    assert rel(H.precondition(X, V), P.precondition(X, V, O.PRECON_EXACT)) <= 1e-10
    # a second application reuses the factor
    V2 = random_tangent(X, d, 53)
    assert rel(H.precondition(X, V2), P.precondition(X, V2, O.PRECON_EXACT)) <= 1e-10


def _subset(meas, keep):
    return O.Measurements(meas.d, meas.r1[keep], meas.r2[keep], meas.p1[keep], meas.p2[keep], meas.R[keep],
                          meas.t[keep], meas.kappa[keep], meas.tau[keep], meas.weight[keep], meas.num_poses)


@pytest.mark.parametrize("fmt", ["bsr", "edges"])
def test_exact_precondition_dirty_reuse(hip, fmt):
    """One handle, Q re-set to a smaller pattern (QuadraticProblem::setQ again, src/QuadraticProblem.cpp:31-42): the
    factor, frontal, panel and sweep buffers of the larger first factor are reused (DevBuf::ensure keeps a larger
    allocation), so they still hold the first factor's values -- a plausible, finite stale entry wherever the new
    factorisation or sweeps read what they did not write.  Every application must still equal the oracle's sparse
    LU of its own Q + 0.1 I at 1e-10 (the round-5 report: 0.235 off after recycled allocations), and the re-set
    handle must agree bitwise with a fresh handle given the smaller Q directly."""
    meas = load_meas("sphere2500")
    d, n, r = meas.d, meas.num_poses, 3
    m = len(meas.p1)
    odo = np.abs(meas.p2 - meas.p1) == 1
    graphs = [meas, _subset(meas, odo | (np.arange(m) % 7 == 0)), _subset(meas, odo)]
    X = random_point(r, d, n, 91)
    V = random_tangent(X, d, 92)

    def set_q(H, g):
        if fmt == "bsr":
            H.set_Q_scipy(0, O.connection_laplacian(g, n))
        else:
            H.set_Q_edges(0, g.p1, g.p2, g.R, g.t, g.kappa, g.tau, g.weight)

    H = hip.Problem(n, d, r)
    H.set_precon(hip.PRECON_EXACT)
    for g in graphs:
        set_q(H, g)
        P = O.QuadraticProblem(n, d, r)
        P.set_Q(O.connection_laplacian(g, n))
        got = H.precondition(X, V)
        err = rel(got, P.precondition(X, V, O.PRECON_EXACT))
        print(f"{fmt} edges={len(g.p1)}: vs LU {err:.2e}")
        assert err <= 1e-10, (len(g.p1), err)
    F = hip.Problem(n, d, r)
    F.set_precon(hip.PRECON_EXACT)
    set_q(F, graphs[-1])
    assert np.array_equal(F.precondition(X, V), got)


def _local_graph(meas, lo, hi):
    keep = (meas.p1 >= lo) & (meas.p1 < hi) & (meas.p2 >= lo) & (meas.p2 < hi)
    return O.Measurements(meas.d, meas.r1[keep], meas.r2[keep], meas.p1[keep] - lo, meas.p2[keep] - lo, meas.R[keep],
                          meas.t[keep], meas.kappa[keep], meas.tau[keep], meas.weight[keep], hi - lo)


@pytest.mark.parametrize("fmt", ["bsr", "edges"])
def test_exact_fallback_per_agent(hip, fmt):
    """QuadraticProblem::PreConditioner falls back per problem (src/QuadraticProblem.cpp:81-86: a failed solve prints
    "Preconditioner failed" and returns its input, unprojected).  A batch of 5 agents in which agent 2's Q is negated
    (Q + 0.1 I indefinite: a non-positive pivot in the host factorisation (bsr) or the device one (edges)): agent 2's
    output is its input bitwise, the other four agents' outputs are bitwise those of the same batch with agent 2
    healthy, and exact_fallback_agents names agent 2 alone.  The healthy batch matches the oracle per agent."""
    meas = load_meas("smallGrid3D")
    d, r, n, A, bad = 3, 5, meas.num_poses, 5, 2
    b = d + 1
    per = n // A
    starts = [k * per for k in range(A)] + [n]
    graphs = [_local_graph(meas, starts[k], starts[k + 1]) for k in range(A)]
    X = random_point(r, d, n, 95)
    V = random_tangent(X, d, 96)

    def run(neg):
        H = hip.Problem(None, d, r, poses_per_agent=[starts[k + 1] - starts[k] for k in range(A)])
        H.set_precon(hip.PRECON_EXACT)
        for k, g in enumerate(graphs):
            s = -1.0 if k == neg else 1.0
            if fmt == "bsr":
                H.set_Q_scipy(k, s * O.connection_laplacian(g, g.num_poses))
            else:
                H.set_Q_edges(k, g.p1, g.p2, g.R, g.t, s * g.kappa, s * g.tau, g.weight)
        return H.precondition(X, V), H.exact_fallback_agents()

    z_ok, f_ok = run(-1)
    z_bad, f_bad = run(bad)
    assert f_ok.tolist() == [0] * A
    assert f_bad.tolist() == [int(k == bad) for k in range(A)]
    for k in range(A):
        sl = slice(starts[k] * b, starts[k + 1] * b)
        if k == bad:
            assert np.array_equal(z_bad[:, sl], V[:, sl])
        else:
            assert np.array_equal(z_bad[:, sl], z_ok[:, sl]), k
        P = O.QuadraticProblem(graphs[k].num_poses, d, r)
        P.set_Q(O.connection_laplacian(graphs[k], graphs[k].num_poses))
        assert rel(z_ok[:, sl], P.precondition(X[:, sl], V[:, sl], O.PRECON_EXACT)) <= 1e-10


@pytest.mark.parametrize("name,r", [("smallGrid3D", 5), ("tinyGrid3D", 3), ("sphere2500", 3)])
def test_rtr_exact_precon(hip, name, r):
    """PGOAgent::localPoseGraphOptimization settings with the reference's default (exact) preconditioner."""
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    Q = O.connection_laplacian(meas, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(Q)
    P.precon_mode = O.PRECON_EXACT
    X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
    trace = []
    Xo, res = O.optimize(P, X0, O.OptParams(tr_iterations=10, tr_tolerance=1e-1, tr_initial_radius=10.0,
                                            tr_max_inner=50), trace)
    H = hip.Problem(n, d, r)
    H.set_Q_scipy(0, Q)
    p = hip.default_params(tr_iterations=10, tr_tolerance=1e-1, tr_initial_radius=10.0, tr_max_inner=50,
                           precon=hip.PRECON_EXACT)
    Xh, rh = H.optimize(X0, p)
    rh = rh[0]
    assert abs(rh["fInit"] - res["fInit"]) <= 1e-12 * abs(res["fInit"])
    assert abs(rh["fOpt"] - res["fOpt"]) <= 1e-9 * abs(res["fOpt"])
    assert rh["outer_iters"] == len(trace)
    assert rh["tCGStatus"] == res["tCGStatus"]
    assert rel(Xh, Xo) <= 1e-8


def test_rbcd_settings_exact_batched(hip):
    """updateX settings (1 iteration, 10 inner, radius 100) for 5 batched agents with the exact
    preconditioner, each against an independent oracle QuadraticProblem."""
    meas = load_meas("smallGrid3D")
    d, r = 3, 5
    b = d + 1
    parts, robot_of, local, start = O.partition_contiguous(meas, meas.num_poses, 5)
    X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, meas.num_poses, meas)
    H = hip.Problem(None, d, r, poses_per_agent=[int(start[k + 1] - start[k]) for k in range(5)])
    H.set_precon(hip.PRECON_EXACT)
    outs = []
    for k in range(5):
        ag = O.Agent(k, O.AgentParams(d, r, 5, robust="L2", precon=O.PRECON_EXACT))
        ag.set_pose_graph(*parts[k], n=int(start[k + 1] - start[k]))
        ag.set_X(X0[:, start[k] * b:start[k + 1] * b])
        nd = {}
        for j in range(5):
            if j != k:
                nd.update({pid: X0[:, (start[pid[0]] + pid[1]) * b:(start[pid[0]] + pid[1] + 1) * b]
                           for pid in ag.neighbor_shared if pid[0] == j})
        assert ag.construct_G(nd)
        ag.problem.precon_mode = O.PRECON_EXACT
        H.set_Q_scipy(k, ag.problem.Q)
        H.set_G_dense(k, ag.problem.G)
        outs.append(O.optimize(ag.problem, ag.X, O.OptParams(tr_iterations=1, tr_tolerance=1e-2,
                                                             tr_initial_radius=100.0, tr_max_inner=10)))
    Xh, rh = H.optimize(X0, hip.default_params(tr_iterations=1, tr_tolerance=1e-2, tr_initial_radius=100.0,
                                               tr_max_inner=10, precon=hip.PRECON_EXACT))
    for k in range(5):
        Xk, rk = outs[k]
        assert rh[k]["runs"] == rk["runs"]
        assert abs(rh[k]["fOpt"] - rk["fOpt"]) <= 1e-10 * max(1.0, abs(rk["fOpt"]))
        assert rel(Xh[:, start[k] * b:start[k + 1] * b], Xk) <= 1e-9


@pytest.mark.parametrize("name", ["torus3D", "sphere2500"])
def test_single_agent_local_pgo(hip, name):
    """BASELINE configs[1]: PGOAgent::localPoseGraphOptimization (src/PGOAgent.cpp:964-990) on
    sphere2500 / torus3D at r = d = 3 with the reference's exact preconditioner, from the chordal
    initialisation: final cost and gradient norm to 1e-9 relative, same outer-iteration count and
    tCG status as the oracle."""
    meas = load_meas(name)
    d, n, r = meas.d, meas.num_poses, 3
    Q = O.connection_laplacian(meas, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(Q)
    P.precon_mode = O.PRECON_EXACT
    X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
    trace = []
    Xo, res = O.optimize(P, X0, O.OptParams(tr_iterations=10, tr_tolerance=1e-1, tr_initial_radius=10.0,
                                            tr_max_inner=50), trace)
    H = hip.Problem(n, d, r)
    H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
    Xh, rh = H.optimize(X0, hip.default_params(tr_iterations=10, tr_tolerance=1e-1, tr_initial_radius=10.0,
                                               tr_max_inner=50, precon=hip.PRECON_EXACT))
    rh = rh[0]
    assert abs(rh["fOpt"] - res["fOpt"]) <= 1e-9 * abs(res["fOpt"])
    assert abs(rh["gradNormOpt"] - res["gradNormOpt"]) <= 1e-9 * max(abs(res["gradNormOpt"]), 1e-12) + 1e-12
    assert rh["outer_iters"] == len(trace)
    assert rh["tCGStatus"] == res["tCGStatus"]


def test_exact_lookahead_bitwise(hip):
    """The classic tCG sequence of the exact preconditioner queued one iteration ahead of a published status
    (tuning key TUNE_TCG_LOOKAHEAD = 1) or every iteration at once (2; 0 = adaptive): agents that stopped skip
    their tiles and their supernodes, so the iterates, counters and per-iteration traces are bitwise the same."""
    g = hip.Graph.grid3d(10, seed=3)
    aop = g.grid_partition(2)
    X0, _, _ = g.distributed_init(aop, 5, hip.lifting_matrix(3, 5), gpu=True, rtol=1e-12, dev_layout=True)
    out = []
    for la in (1, 2, 0):
        hip.set_tuning(7, la)
        try:
            e = hip.Rbcd(g, aop, np.zeros(8, np.int32), 0, 1,
                         hip.rbcd_params(r=5, acceleration=1, precon=hip.PRECON_EXACT))
            e.set_trace(512)
            e.set_X(X0)
            for it in range(24):
                e.pre_exchange(it % e.num_colors)
                e.update(it % e.num_colors, None)
            X = np.zeros(X0.size)
            e.get_X_into(X)
            out.append((X, e.stats().copy(), [e.get_trace(a) for a in range(8)]))
        finally:
            hip.set_tuning(7, 0)
    for o in out[1:]:
        assert np.array_equal(out[0][0], o[0])
        assert np.array_equal(out[0][1][:, :12], o[1][:, :12])
        for a in range(8):
            assert len(out[0][2][a]) == len(o[2][a])
            for x, y in zip(out[0][2][a], o[2][a]):
                assert x == y
    assert out[0][1][:, 10].sum() > 0  # CG steps were taken


def _grid_meas(hip, k, seed):
    g = hip.Graph.grid3d(k, seed=seed)
    a = g.arrays()
    meas = O.Measurements(3, np.zeros(g.m, np.int64), np.zeros(g.m, np.int64), a["p1"].astype(np.int64),
                          a["p2"].astype(np.int64), a["R"], a["t"], a["kappa"], a["tau"], np.ones(g.m), g.n)
    return g, meas


@pytest.mark.parametrize("k", [12, 20, pytest.param(25, marks=pytest.mark.timeout(900))])
def test_device_factor_large_separator(hip, k):
    """The exact preconditioner at d = 3, r = 5 on one agent large enough that its top separator spans many 64-row
    tiles (grid3d k = 20: 8000 poses, a 400-pose top separator = 25 tile rows, the C5 agents' shape at 1/8 the
    volume; k = 25: 15,625 poses, exactly one C5 agent's size and shape), with the numeric factorisation on the device
    (tile-parallel k_snf_* / k_sn_factor, TUNE_DEVICE_CHOL = 1, the default) and on the host (0): single applications
    against the oracle's sparse LU at 1e-10, and the two factorisations against each other at 1e-12 (the same
    symbolic structure; only the summation order of the dense steps differs)."""
    g, meas = _grid_meas(hip, k, 7)
    d, n, r = 3, g.n, 5
    Q = O.connection_laplacian(meas, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(Q)
    X = random_point(r, d, n, 61)
    V = random_tangent(X, d, 62)
    ref = P.precondition(X, V, O.PRECON_EXACT)
    got = {}
    for dev in (1, 0):
        H = hip.Problem(n, d, r)
        H.set_tuning(12, dev)
        H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
        H.set_precon(hip.PRECON_EXACT)
        got[dev] = H.precondition(X, V)
        info = H.exact_factor_info()
        assert info["factor_count"] == dev
        if k >= 20:
            assert info["max_s_tiles"] >= 8, info
        assert rel(got[dev], ref) <= 1e-10, (dev, rel(got[dev], ref))
    print(f"k={k}: device vs LU {rel(got[1], ref):.2e}, host vs LU {rel(got[0], ref):.2e}, "
          f"device vs host {rel(got[1], got[0]):.2e}")
    assert rel(got[1], got[0]) <= 1e-12


@pytest.mark.parametrize("k", [12, 20])
def test_device_factor_tiled_levels_bitwise(hip, k, monkeypatch):
    """The tile-parallel factorisation of the large top levels (k_snf_asm / k_snf_tile, one launch per step of the
    right-looking K loop) applies every tile the same operations in the same order as the one-workgroup-per-node
    kernel: the preconditioner outputs agree bitwise (DPGO_FAC_TILED_MAX_NODES=0 forces k_sn_factor everywhere)."""
    g, meas = _grid_meas(hip, k, 7)
    d, n, r = 3, g.n, 5
    X = random_point(r, d, n, 61)
    V = random_tangent(X, d, 62)
    got = {}
    for lim in ("0", "4096"):
        monkeypatch.setenv("DPGO_FAC_TILED_MAX_NODES", lim)
        H = hip.Problem(n, d, r)
        H.set_tuning(12, 1)
        H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
        H.set_precon(hip.PRECON_EXACT)
        got[lim] = H.precondition(X, V)
    assert np.array_equal(got["0"], got["4096"]), float(np.abs(got["0"] - got["4096"]).max())


@pytest.mark.parametrize("k,r", [(12, 5), (20, 5), (16, 3)])
def test_forward_small_nodes_bitwise(hip, k, r, monkeypatch):
    """The narrow supernodes' forward items (at most kSnSmallNs S column tiles) through k_sn_fwd_small: the same
    products in the same order as k_sn_fwd, so the preconditioner outputs agree bitwise (DPGO_SN_FWD_SMALL=0 sends
    every item through k_sn_fwd), and both equal the oracle's sparse LU to 1e-10."""
    g, meas = _grid_meas(hip, k, 7)
    d, n = 3, g.n
    Q = O.connection_laplacian(meas, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(Q)
    X = random_point(r, d, n, 81)
    V = random_tangent(X, d, 82)
    ref = P.precondition(X, V, O.PRECON_EXACT)
    got = {}
    for small in ("0", "1"):
        monkeypatch.setenv("DPGO_SN_FWD_SMALL", small)
        H = hip.Problem(n, d, r)
        H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
        H.set_precon(hip.PRECON_EXACT)
        got[small] = H.precondition(X, V)
    assert np.array_equal(got["0"], got["1"]), float(np.abs(got["0"] - got["1"]).max())
    assert rel(got["1"], ref) <= 1e-10


@pytest.mark.parametrize("name,r", [("input_INTEL_g2o", 3), ("sphere2500", 3), ("smallGrid3D", 5)])
def test_device_factor_tiled_every_level_bitwise(hip, name, r, monkeypatch):
    """Every tree level forced through the tile-parallel kernels (DPGO_FAC_TILED_MIN_TILES=1), for d = 2 (b = 3) and
    d = 3: the preconditioner equals the one-workgroup-per-node factor's bitwise and the oracle's sparse LU to
    1e-10."""
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    Q = O.connection_laplacian(meas, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(Q)
    X = random_point(r, d, n, 71)
    V = random_tangent(X, d, 72)
    ref = P.precondition(X, V, O.PRECON_EXACT)
    got = {}
    for lim in ("0", "1000000"):
        monkeypatch.setenv("DPGO_FAC_TILED_MAX_NODES", lim)
        monkeypatch.setenv("DPGO_FAC_TILED_MIN_TILES", "1")
        H = hip.Problem(n, d, r)
        H.set_tuning(12, 1)
        H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
        H.set_precon(hip.PRECON_EXACT)
        got[lim] = H.precondition(X, V)
        assert H.exact_factor_info()["factor_count"] == 1
    assert np.array_equal(got["0"], got["1000000"]), float(np.abs(got["0"] - got["1000000"]).max())
    assert rel(got["1000000"], ref) <= 1e-10


def test_device_refactor_after_reweighting(hip):
    """set_edge_weights_dev (the on-device GNC reweighting) leaves the pattern and refreshes only the numeric half:
    the next application re-runs k_sn_factor on the new weights and matches the oracle's LU of the reweighted Q."""
    g, meas = _grid_meas(hip, 8, 9)
    d, n, r = 3, g.n, 5
    rng = np.random.default_rng(3)
    w = rng.uniform(0.05, 1.0, g.m)
    X = random_point(r, d, n, 63)
    V = random_tangent(X, d, 64)
    H = hip.Problem(n, d, r)
    H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
    H.set_precon(hip.PRECON_EXACT)
    H.precondition(X, V)
    import torch
    wd = torch.tensor(w, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    H.set_edge_weights_dev(wd.data_ptr())
    z = H.precondition(X, V)
    assert H.exact_factor_info()["factor_count"] == 2
    mw = O.Measurements(3, meas.r1, meas.r2, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, w, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(O.connection_laplacian(mw, n))
    assert rel(z, P.precondition(X, V, O.PRECON_EXACT)) <= 1e-10


@pytest.mark.parametrize("robust", ["L2", "GNC_TLS"])
def test_engine_exact_matches_oracle(hip, robust):
    """The engine's colour schedule with the exact preconditioner (the reference's default) on grid3d k = 24 with 8
    agents of 12^3 poses (L2), and k = 8 with outliers under GNC_TLS (reweighting every 3 iterations: the factor is
    refreshed on the device after each), against the oracle's PGOAgent colour schedule at 1e-9 with the same
    solver counters."""
    k, A, r = (24, 2, 5) if robust == "L2" else (8, 2, 5)
    iters = 6 if robust == "L2" else 8
    g, meas = _grid_meas(hip, k, 11)
    if robust != "L2":
        a = g.arrays()
        p1, p2 = a["p1"].astype(np.int64), a["p2"].astype(np.int64)
        t = a["t"].copy()
        lc = np.nonzero(np.abs(p2 - p1) != 1)[0]
        bad = np.random.default_rng(5).choice(lc, size=max(1, len(lc) // 10), replace=False)
        t[bad] += np.random.default_rng(6).normal(0.0, 5.0, size=(len(bad), 3))
        g0 = g
        g = hip.Graph.from_arrays(3, g0.n, p1, p2, a["R"], t, a["kappa"], a["tau"])
        meas = O.Measurements(3, np.zeros(len(p1), np.int64), np.zeros(len(p1), np.int64), p1, p2, a["R"], t,
                              a["kappa"], a["tau"], np.ones(len(p1)), g0.n)
        aop = g0.grid_partition(A)
        X0 = g0.chain_init(r, O.lifting_matrix(3, r))
    else:
        aop = g.grid_partition(A)
        X0 = g.chain_init(r, O.lifting_matrix(3, r))
    e = hip.Rbcd(g, aop, np.zeros(A ** 3, np.int32), 0, 1,
                 hip.rbcd_params(r=r, acceleration=1, robust_cost=hip.ROBUST[robust], robust_opt_inner_iters=3,
                                 precon=hip.PRECON_EXACT))
    e.set_X(X0)
    for it in range(iters):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
    out = np.zeros(X0.size)
    e.get_X_into(out)
    Xo, _ = O.colour_rbcd(meas, aop, A ** 3, X0, iters, r, acceleration=True, robust=robust,
                          robust_opt_inner_iters=3, precon=O.PRECON_EXACT)
    assert rel(hip.from_dev_layout(out, r), Xo) <= 1e-9
    if robust != "L2":
        assert sum(e.exact_factor_info(c)["factor_count"] for c in range(e.num_colors)) >= 3


@pytest.mark.parametrize("k,r", [(12, 5), (20, 5), (16, 3)])
def test_compact_narrow_panels_bitwise(hip, k, r, monkeypatch):
    """Narrow supernodes' compact panels (SnView::cpanel: no 64 x 64 tile padding, which is 2-2.4x the useful panel on
    the deep nested-dissection levels) read by every sweep kernel: the same products in the same order, the tile
    padding read as exact zeros, so the preconditioner outputs equal the tile-only path's bitwise (DPGO_SN_COMPACT=0),
    on the host and the device factorisation alike, and the oracle's sparse LU to 1e-10."""
    g, meas = _grid_meas(hip, k, 7)
    d, n = 3, g.n
    Q = O.connection_laplacian(meas, n)
    P = O.QuadraticProblem(n, d, r)
    P.set_Q(Q)
    X = random_point(r, d, n, 83)
    V = random_tangent(X, d, 84)
    ref = P.precondition(X, V, O.PRECON_EXACT)
    got = {}
    for cmp in ("0", "1"):
        for dev in (1, 0):
            monkeypatch.setenv("DPGO_SN_COMPACT", cmp)
            H = hip.Problem(n, d, r)
            H.set_tuning(12, dev)
            H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
            H.set_precon(hip.PRECON_EXACT)
            got[cmp, dev] = H.precondition(X, V)
    for dev in (1, 0):
        assert np.array_equal(got["0", dev], got["1", dev]), float(np.abs(got["0", dev] - got["1", dev]).max())
        assert rel(got["1", dev], ref) <= 1e-10
