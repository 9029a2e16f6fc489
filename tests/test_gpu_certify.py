"""GPU certificate lambda_min(Q - Lambda(X)).  The reference has no certification
(SURVEY section 1, item 8), so this is pinned against the oracle's explicit matrix
(oracle.certificate_matrix) and numpy/ARPACK eigenvalues only.

Tolerances: Lanczos stops when the Ritz residual <= tol * |lambda|max; the Ritz value is then within
residual of an eigenvalue, so |lambda_gpu - lambda_oracle| <= 1e-6 * |lambda|max is asserted, and the
returned Ritz vector v must satisfy ||v S - lambda v|| <= 1e-6 * |lambda|max against the oracle S."""
import numpy as np
import pytest

from oracle import dpgo_oracle as O
from tests._common import load_meas, random_point, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    from dpgo_amd import hip as H
    assert H.device_count() >= 1, "no gfx950 device"
    return H


def _check(H, Q, X, d, max_iters, tol=1e-10):
    S = O.certificate_matrix(Q, X, d)
    lam_o = O.certificate_min_eig(S)
    lam_max = float(np.abs(np.linalg.eigvalsh(S.toarray())).max()) if S.shape[0] <= 3000 else \
        float(abs(O.spla.eigsh(S, k=1, which="LM")[0][0]))
    lam, res, it, v = H.certify(X, max_iters=max_iters, tol=tol, want_vector=True)
    assert abs(lam - lam_o) <= 1e-6 * lam_max, (lam, lam_o, res, it)
    assert abs(np.linalg.norm(v) - 1.0) <= 1e-8
    Rv = np.asarray((S @ v.T).T) - lam * v
    assert np.linalg.norm(Rv) <= 1e-6 * lam_max
    return lam, lam_o, it


@pytest.mark.parametrize("fmt", ["bsr", "edges"])
@pytest.mark.parametrize("name,r", [("tinyGrid3D", 3), ("smallGrid3D", 5), ("input_INTEL_g2o", 3)])
def test_certificate_random_point(hip, name, r, fmt):
    """At a random point the certificate fails: lambda_min < 0, matching the explicit matrix."""
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    Q = O.connection_laplacian(meas, n)
    X = random_point(r, d, n, 61)
    H = hip.Problem(n, d, r)
    if fmt == "bsr":
        H.set_Q_scipy(0, Q)
    else:
        H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
    lam, lam_o, _ = _check(H, Q, X, d, max_iters=min(600, r * (d + 1) * n))
    assert lam < 0 and lam_o < 0


@pytest.mark.parametrize("name,r", [("tinyGrid3D", 5), ("smallGrid3D", 5)])
def test_certificate_at_optimum(hip, name, r):
    """After RTR from chordal initialisation on clean grids, S(X) is PSD up to rounding: the smallest
    eigenvalue is ~0 (the rows of X span its null space)."""
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    Q = O.connection_laplacian(meas, n)
    X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
    H = hip.Problem(n, d, r)
    H.set_Q_scipy(0, Q)
    Xo, _ = H.optimize(X0, hip.default_params(tr_iterations=100, tr_tolerance=1e-10, tr_max_inner=200,
                                              precon=hip.PRECON_EXACT))
    S = O.certificate_matrix(Q, Xo, d)
    lam_max = float(np.abs(np.linalg.eigvalsh(S.toarray())).max())
    lam, res, it, _ = H.certify(Xo, max_iters=600, tol=1e-10)
    lam_o = O.certificate_min_eig(S)
    assert abs(lam - lam_o) <= 1e-6 * lam_max
    assert lam >= -1e-6 * lam_max
    # X S(X) = grad f(X) (identity checked in test_oracle), ~0 at the critical point RTR returns
    assert float(np.linalg.norm((S @ Xo.T).T)) <= 1e-6 * lam_max


def test_certificate_rejects_batched(hip):
    H = hip.Problem(None, 3, 3, poses_per_agent=[4, 4])
    with pytest.raises(Exception):
        H.certify(np.zeros((3, 32)))


@pytest.mark.parametrize("name,agents,iters", [("smallGrid3D", 5, 400), ("city10000", 8, 300)])
def test_graph_certify_engine_iterate(hip, name, agents, iters):
    """Certified gap of the multi-agent engine's iterate over the whole graph (dpgo_graph_certify):
    f(X), the SE(d) rounding (PGOAgent::getTrajectoryInLocalFrame) and its cost against the oracle;
    lambda_min as an eigenvalue of the oracle's explicit S (Ritz residual; exact value below 3000
    rows)."""
    meas = load_meas(name)
    d, n, r = meas.d, meas.num_poses, 5
    aop = np.minimum(np.arange(n) // (n // agents), agents - 1).astype(np.int32)
    g = hip.Graph.from_arrays(d, n, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau)
    X0, _, _ = g.distributed_init(aop, r, O.lifting_matrix(d, r), gpu=True, rtol=1e-12, dev_layout=True)
    e = hip.Rbcd(g, aop, np.zeros(agents, np.int32), 0, 1, hip.rbcd_params(r=r, acceleration=1))
    e.set_X(X0)
    gn = None
    for it in range(iters):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
        if it % 100 == 99:
            _, gsq = e.central_eval()
            gn = float(np.sqrt(np.sum(gsq)))
            if gn < 1e-7:
                break
    Xd = np.zeros(X0.size)
    e.get_X_into(Xd)
    c = g.certify(Xd, r, max_iters=1500 if n < 1000 else 400, tol=1e-10, want_rounded=True, want_vector=True)
    X = hip.from_dev_layout(Xd, r)
    Q = O.connection_laplacian(meas, n)
    assert abs(c["f_relax"] - O.central_cost(meas, X)) <= 1e-11 * abs(c["f_relax"])  # f: a sum of cancelling terms
    T = O.round_to_se(X, d)
    assert rel(c["T_rounded"], T) <= 1e-10
    assert abs(c["f_rounded"] - O.central_cost(meas, T)) <= 1e-10 * abs(c["f_rounded"])
    S = O.certificate_matrix(Q, X, d)
    lam_bound = float(abs(S).sum(axis=1).max())  # >= |lambda|max (Gershgorin)
    v = c["eigvec"]
    assert abs(np.linalg.norm(v) - 1.0) <= 1e-8
    # lambda_min lies within the Ritz residual of an eigenvalue of S; the reported residual is the true one
    res = np.linalg.norm(np.asarray((S @ v.T).T) - c["lambda_min"] * v)
    assert abs(res - c["residual"]) <= 1e-3 * res + 1e-9 * lam_bound, (res, c["residual"])
    assert res <= 1e-3 * lam_bound
    if S.shape[0] <= 3000:
        lam_o = float(np.linalg.eigvalsh(S.toarray())[0])
        assert abs(c["lambda_min"] - lam_o) <= 1e-6 * lam_bound


@pytest.mark.parametrize("name", ["smallGrid3D", "tinyGrid3D"])
def test_graph_certify_certified_gap(hip, name):
    """At the relaxation's global optimum (RTR from chordal initialisation) the central certificate
    holds and f_rounded - f(X) >= 0 is a certified suboptimality bound of the SE(d) rounding."""
    meas = load_meas(name)
    d, n, r = meas.d, meas.num_poses, 5
    Q = O.connection_laplacian(meas, n)
    X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
    H = hip.Problem(n, d, r)
    H.set_Q_scipy(0, Q)
    Xo, _ = H.optimize(X0, hip.default_params(tr_iterations=100, tr_tolerance=1e-10, tr_max_inner=200,
                                              precon=hip.PRECON_EXACT))
    g = hip.Graph.from_arrays(d, n, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau)
    c = g.certify(Xo, r, max_iters=1500, tol=1e-10)
    S = O.certificate_matrix(Q, Xo, d)
    lam_bound = float(abs(S).sum(axis=1).max())
    assert abs(c["lambda_min"] - float(np.linalg.eigvalsh(S.toarray())[0])) <= 1e-6 * lam_bound
    assert c["lambda_min"] >= -1e-6 * lam_bound
    assert c["gap"] >= -1e-9 * abs(c["f_relax"])
    assert abs(c["f_rounded"] - O.central_cost(meas, O.round_to_se(Xo, d))) <= 1e-10 * abs(c["f_rounded"])


def _seed_blocks(S, X, d=3):
    """The seed block's exact quantities for row 0 of the lifted layout: U = X's principal row directions and
    the translation gauge, orthonormalised,
    lambda_min(U^T S U), lambda_min of S compressed to U's complement, |(I - U U^T) S U|_F."""
    import scipy.linalg as sl
    Sd = S.toarray()
    U, sv, _ = np.linalg.svd(X.T, full_matrices=False)
    U = U[:, sv >= 1e-3 * sv[0]]  # X's principal row directions, as dpgo_hip_certify_ex seeds them
    gauge = np.zeros(X.shape[1])
    gauge[d::d + 1] = 1.0
    U, _ = np.linalg.qr(np.column_stack([U, gauge]))  # + the translation gauge (exact null vector)
    N = sl.null_space(U.T)
    SU = Sd @ U
    return (float(np.linalg.eigvalsh(U.T @ SU)[0]), float(np.linalg.eigvalsh(N.T @ Sd @ N)[0]),
            float(np.linalg.norm(SU - U @ (U.T @ SU))), U.shape[1])


@pytest.mark.parametrize("seed_x", [False, True])
@pytest.mark.parametrize("name,r", [("tinyGrid3D", 3), ("smallGrid3D", 5)])
def test_certificate_thick_restart(hip, name, r, seed_x):
    """dpgo_hip_certify_ex with a basis far below the iteration count (thick restarts), optionally with the
    rows of X as a locked seed block: lambda_min of the explicit matrix (no seeds) or the block quantities
    of S = [A_s B^T; B C] and the sandwich lower_bound <= lambda_min(S) <= lambda (seeds); true residuals."""
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    Q = O.connection_laplacian(meas, n)
    X = random_point(r, d, n, 62)
    H = hip.Problem(n, d, r)
    H.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
    S = O.certificate_matrix(Q, X, d)
    ev = np.linalg.eigvalsh(S.toarray())
    lam_max = float(np.abs(ev).max())
    lam, res, it, v = H.certify(X, max_iters=4000, tol=1e-10, want_vector=True, basis=40, seed_x=seed_x)
    info = H.last_certificate
    assert abs(np.linalg.norm(v) - 1.0) <= 1e-8
    true_res = np.linalg.norm(np.asarray((S @ v.T).T) - lam * v)
    assert abs(true_res - res) <= 1e-3 * true_res + 1e-9 * lam_max, (true_res, res)
    assert info["restarts"] >= 1 or info["iters"] <= 40, info  # tinyGrid3D's row-0 space is exhausted first
    if not seed_x:
        assert abs(lam - ev[0]) <= 1e-6 * lam_max, (lam, ev[0], res, it)
        assert true_res <= 1e-6 * lam_max
        return
    lam_s, lam_c, coup, ns = _seed_blocks(S, X, d)
    assert info["seeds"] == ns
    assert abs(info["lambda_seed"] - lam_s) <= 1e-9 * lam_max, (info, lam_s)
    assert abs(info["lambda_complement"] - lam_c) <= 1e-6 * lam_max, (info, lam_c)
    assert info["residual_complement"] <= 1e-6 * lam_max
    assert abs(info["coupling"] - coup) <= 1e-9 * lam_max + 1e-6 * coup, (info, coup)
    assert info["lower_bound"] <= ev[0] + 1e-9 * lam_max <= lam + 2e-9 * lam_max, (info, ev[0], lam)
    assert lam == min(info["lambda_seed"], info["lambda_complement"])
    assert float(np.abs(v[1:]).max()) == 0.0  # the search space lives on row 0 of the lifted layout


def test_graph_certify_seeded_at_optimum(hip):
    """At the RTR optimum of smallGrid3D (S(X) X^T ~ 0) the locked seed block carries the near-null cluster,
    its coupling to the complement is ~0 and the bound certifies: lower_bound >= -eps, with
    lower_bound <= lambda_min(S) <= lambda_min (reported)."""
    meas = load_meas("smallGrid3D")
    d, n, r = meas.d, meas.num_poses, 5
    Q = O.connection_laplacian(meas, n)
    X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
    H = hip.Problem(n, d, r)
    H.set_Q_scipy(0, Q)
    Xo, _ = H.optimize(X0, hip.default_params(tr_iterations=100, tr_tolerance=1e-10, tr_max_inner=200,
                                              precon=hip.PRECON_EXACT))
    g = hip.Graph.from_arrays(d, n, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau)
    c = g.certify(Xo, r, max_iters=3000, tol=1e-10, basis=60, seed_x=True)
    S = O.certificate_matrix(Q, Xo, d)
    ev = np.linalg.eigvalsh(S.toarray())
    lam_bound = float(abs(S).sum(axis=1).max())
    lam_s, lam_c, coup, ns = _seed_blocks(S, Xo, d)
    assert c["seeds"] == ns
    assert abs(c["lambda_complement"] - lam_c) <= 1e-6 * lam_bound, (c, lam_c)
    assert abs(c["coupling"] - coup) <= 1e-8 * lam_bound + 1e-5 * coup, (c, coup)
    assert c["coupling"] <= 1e-6 * lam_bound
    assert c["lower_bound"] <= ev[0] + 1e-9 * lam_bound <= c["lambda_min"] + 2e-9 * lam_bound, (c, ev[:4])
    assert c["lower_bound"] >= -1e-6 * lam_bound
    assert c["gap"] >= -1e-9 * abs(c["f_relax"])
