"""Shared test helpers: fixture loading and oracle setup (test infrastructure)."""
import os

import numpy as np

from oracle import dpgo_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_meas(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.meas.npz"))
    return O.Measurements(int(z["d"]), z["r1"], z["r2"], z["p1"], z["p2"], z["R"], z["t"],
                          z["kappa"], z["tau"], np.ones(len(z["p1"])), int(z["n"]),
                          int(z["duplicates"]))


def random_point(r, d, n, seed):
    rng = O.SplitMix64(seed)
    M = np.array([[rng.normal() for _ in range((d + 1) * n)] for _ in range(r)])
    return O.lifted_project(M, d)


def random_tangent(X, d, seed):
    rng = O.SplitMix64(seed)
    V = np.array([[rng.normal() for _ in range(X.shape[1])] for _ in range(X.shape[0])])
    return O.tangent_project(X, V, d)


def seeded_G(X, d, r, n, seed):
    G = np.zeros_like(X)
    rng = O.SplitMix64(seed)
    for j in range(0, n, max(1, n // 7)):
        for c in range(d + 1):
            for a in range(r):
                G[a, j * (d + 1) + c] = rng.normal()
    return G


def rel(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    den = max(np.linalg.norm(b), 1e-300)
    return float(np.linalg.norm(a - b) / den)


def unit_laplacian(arrays, n):
    """The dataset's connection Laplacian at unit weights (the example's QCentral, examples/MultiRobotExample.cpp:
    229-235), assembled vectorised with the per-edge blocks of O.connection_laplacian (src/DPGO_utils.cpp's
    constructConnectionLaplacianSE): Q_ii += T Om T^T, Q_jj += Om, Q_ij = -T Om, Q_ji = -Om T^T."""
    import scipy.sparse as sp
    p1 = np.asarray(arrays["p1"], np.int64)
    p2 = np.asarray(arrays["p2"], np.int64)
    R = np.asarray(arrays["R"], np.float64).reshape(len(p1), 3, 3)
    t = np.asarray(arrays["t"], np.float64).reshape(len(p1), 3)
    m, b = len(p1), 4
    T = np.zeros((m, b, b))
    T[:, :3, :3] = R
    T[:, :3, 3] = t
    T[:, 3, 3] = 1.0
    om = np.zeros((m, b))
    om[:, :3] = np.asarray(arrays["kappa"], np.float64)[:, None]
    om[:, 3] = np.asarray(arrays["tau"], np.float64)
    TOm = T * om[:, None, :]
    blocks = [(p1, p1, TOm @ np.swapaxes(T, 1, 2)), (p2, p2, om[:, :, None] * np.eye(b)[None]),
              (p1, p2, -TOm), (p2, p1, -np.swapaxes(TOm, 1, 2))]
    rr, cc = np.meshgrid(np.arange(b), np.arange(b), indexing="ij")
    rows = np.concatenate([(bi[:, None, None] * b + rr).ravel() for bi, _, _ in blocks])
    cols = np.concatenate([(bj[:, None, None] * b + cc).ravel() for _, bj, _ in blocks])
    vals = np.concatenate([B.ravel() for _, _, B in blocks])
    Q = sp.coo_matrix((vals, (rows, cols)), shape=(b * n, b * n)).tocsr()
    Q.sum_duplicates()
    return Q


def central_cost_gradnorm(Q, X, d):
    """The example's central evaluation of X (r x (d+1) n) with G = 0: f = 1/2 tr(X Q X^T) and |P_X(X Q)|_F
    (QuadraticProblem::f / RieGrad, src/QuadraticProblem.cpp:50-56, 89-97), in numpy."""
    XQ = np.asarray((Q @ X.T).T)
    f = 0.5 * float(np.sum(XQ * X))
    return f, float(np.linalg.norm(O.tangent_project(X, XQ, d)))
