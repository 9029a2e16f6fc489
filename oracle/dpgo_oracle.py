"""CPU oracle for the DPGO RBCD hot path -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.

This module is a numpy/scipy restatement of the reference (lajoiepy/dpgo @ 2024_10_08)
arithmetic on the Riemannian block-coordinate-descent hot path.  It exists only to check the
HIP implementation: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it, and only as the checker.  The product path
(``dpgo_amd``) never imports it.

Every function cites the reference file:line it restates (paths relative to the reference
root).  Parity status (see DESIGN.md "Oracle"):

* pinned by the reference's own known-answer tests: the triangle graph stays fixed through
  ``iterate`` (tests/testTriangleGraph.cpp:51-65), pose-block memory layout
  (tests/testEigenMap.cpp:12-36), Stiefel/polar projection orthonormality
  (tests/testUtils.cpp:12-53);
* the reference cannot be built or run here (Eigen3, CHOLMOD/SPQR, Boost and the un-vendored
  ROPTLIB are absent: SURVEY.md 8c), so RTR / tCG iterates, rho and Delta follow the ROPTLIB
  semantics restated in SURVEY.md Appendix A.4 and are **parity unpinned** against the
  reference binary.

Conventions: d in {2,3}, b = d+1, X is r x (b*n), pose j is the column block
``X[:, j*b:(j+1)*b] = [Y_j | p_j]``.  On the device the same matrix is stored column-major,
i.e. ``X.T`` in C order (``to_dev`` / ``from_dev``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

# ----------------------------------------------------------------------------------------
# Repo-defined deterministic RNG: SplitMix64 -> 53-bit uniform -> Box-Muller.
# The C++ generator (dpgo_amd/csrc/graph.cpp) implements the identical stream.
# ----------------------------------------------------------------------------------------
_M64 = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed: int):
        self.state = seed & _M64
        self._cached = None

    def next_u64(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & _M64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
        return z ^ (z >> 31)

    def uniform(self) -> float:
        """Uniform in [0, 1) with 53 random bits."""
        return (self.next_u64() >> 11) * (1.0 / 9007199254740992.0)

    def normal(self) -> float:
        if self._cached is not None:
            v, self._cached = self._cached, None
            return v
        u1 = 1.0 - self.uniform()  # (0, 1]
        u2 = self.uniform()
        rad = math.sqrt(-2.0 * math.log(u1))
        ang = 6.283185307179586 * u2
        self._cached = rad * math.sin(ang)
        return rad * math.cos(ang)


# ----------------------------------------------------------------------------------------
# Measurements (include/DPGO/RelativeSEMeasurement.h:21-71)
# ----------------------------------------------------------------------------------------
@dataclass
class Measurements:
    d: int
    r1: np.ndarray  # robot of first pose
    r2: np.ndarray
    p1: np.ndarray  # pose index
    p2: np.ndarray
    R: np.ndarray  # (m, d, d)
    t: np.ndarray  # (m, d)
    kappa: np.ndarray
    tau: np.ndarray
    weight: np.ndarray
    num_poses: int = 0
    duplicates: int = 0
    extra: dict = field(default_factory=dict)

    @property
    def m(self) -> int:
        return int(self.p1.shape[0])

    def subset(self, mask) -> "Measurements":
        idx = np.nonzero(mask)[0] if np.asarray(mask).dtype == bool else np.asarray(mask)
        return Measurements(self.d, self.r1[idx].copy(), self.r2[idx].copy(), self.p1[idx].copy(),
                            self.p2[idx].copy(), self.R[idx].copy(), self.t[idx].copy(),
                            self.kappa[idx].copy(), self.tau[idx].copy(), self.weight[idx].copy(),
                            self.num_poses)


def key_to_robot_keyframe(key: int):
    """src/DPGO_utils.cpp:21-33 (GTSAM symbol: 8-bit chr | 8-bit label | 48-bit index)."""
    chr_ = (key >> 56) & 0xFF
    idx = key & ((1 << 48) - 1)
    return chr_, idx


def quat_to_rot_eigen(qw, qx, qy, qz):
    """Eigen::Quaterniond(w,x,y,z).toRotationMatrix() -- no normalisation
    (src/DPGO_utils.cpp:169)."""
    tx, ty, tz = 2.0 * qx, 2.0 * qy, 2.0 * qz
    twx, twy, twz = tx * qw, ty * qw, tz * qw
    txx, txy, txz = tx * qx, ty * qx, tz * qx
    tyy, tyz, tzz = ty * qy, tz * qy, tz * qz
    return np.array([[1.0 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1.0 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1.0 - (txx + tyy)]])


def eigen_inverse_trace_2(a, b, d):
    """trace(M^-1) for M = [[a, b], [b, d]] with Eigen's fixed-size 2x2 inverse
    (Eigen/src/LU/InverseImpl.h compute_inverse_size2: invdet = 1/det, r_ii = m_jj * invdet)."""
    det = a * d - b * b
    invdet = 1.0 / det
    return d * invdet + a * invdet


def eigen_inverse_trace_3(M):
    """trace(M^-1) with Eigen's fixed-size 3x3 cofactor inverse (compute_inverse_size3)."""
    m = M
    c00 = m[1][1] * m[2][2] - m[1][2] * m[2][1]
    c10 = m[2][1] * m[0][2] - m[2][2] * m[0][1]
    c20 = m[0][1] * m[1][2] - m[0][2] * m[1][1]
    det = c00 * m[0][0] + c10 * m[1][0] + c20 * m[2][0]
    invdet = 1.0 / det
    c11 = m[2][2] * m[0][0] - m[2][0] * m[0][2]
    c22 = m[0][0] * m[1][1] - m[0][1] * m[1][0]
    return c00 * invdet + c11 * invdet + c22 * invdet


def read_g2o(path: str) -> Measurements:
    """src/DPGO_utils.cpp:78-212 with the SURVEY Appendix B fixes:
    B1 num_poses = max pose index + 1; B2 blank lines skipped, FIX / unknown tokens ignored,
    exact duplicates counted (kept, as the reference keeps them)."""
    r1, r2, p1, p2, Rs, ts, kap, tau = [], [], [], [], [], [], [], []
    d = 0
    for line in open(path):
        tok = line.split()
        if not tok:
            continue
        if tok[0] == "EDGE_SE2":
            i, j = int(tok[1]), int(tok[2])
            dx, dy, dth = map(float, tok[3:6])
            I11, I12, I13, I22, I23, I33 = map(float, tok[6:12])
            ci, cj = key_to_robot_keyframe(i), key_to_robot_keyframe(j)
            c, s = math.cos(dth), math.sin(dth)
            R = np.array([[c, -s], [s, c]])
            tau.append(2.0 / eigen_inverse_trace_2(I11, I12, I22))  # :129-131
            kap.append(I33)  # :133
            t = np.array([dx, dy])
            d = 2
        elif tok[0] == "EDGE_SE3:QUAT":
            i, j = int(tok[1]), int(tok[2])
            v = list(map(float, tok[3:]))
            dx, dy, dz, qx, qy, qz, qw = v[:7]
            I = v[7:28]
            (I11, I12, I13, I14, I15, I16, I22, I23, I24, I25, I26, I33, I34, I35, I36,
             I44, I45, I46, I55, I56, I66) = I
            ci, cj = key_to_robot_keyframe(i), key_to_robot_keyframe(j)
            R = quat_to_rot_eigen(qw, qx, qy, qz)
            Tc = [[I11, I12, I13], [I12, I22, I23], [I13, I23, I33]]
            Rc = [[I44, I45, I46], [I45, I55, I56], [I46, I56, I66]]
            tau.append(3.0 / eigen_inverse_trace_3(Tc))  # :176-178
            kap.append(3.0 / (2.0 * eigen_inverse_trace_3(Rc)))  # :183-185
            t = np.array([dx, dy, dz])
            d = 3
        else:
            continue  # VERTEX_* (initial guesses, unused), FIX, unknown: ignored
        r1.append(ci[0]); r2.append(cj[0]); p1.append(ci[1]); p2.append(cj[1])
        Rs.append(R); ts.append(t)
    p1a = np.array(p1, dtype=np.int64); p2a = np.array(p2, dtype=np.int64)
    n = int(max(p1a.max(), p2a.max()) + 1) if len(p1) else 0
    pairs = set()
    dup = 0
    for a, b2 in zip(p1, p2):
        if (a, b2) in pairs:
            dup += 1
        pairs.add((a, b2))
    m = len(p1)
    return Measurements(d, np.array(r1, np.int64), np.array(r2, np.int64), p1a, p2a,
                        np.array(Rs).reshape(m, d, d), np.array(ts).reshape(m, d),
                        np.array(kap, float), np.array(tau, float), np.ones(m), n, dup)


# ----------------------------------------------------------------------------------------
# Synthetic 3D grid (stands in for the missing g2o100k / 1M graphs)
# ----------------------------------------------------------------------------------------
def _snake_xy(idx, k):
    yy = idx // k
    xx = idx % k
    if yy & 1:
        xx = k - 1 - xx
    return xx, yy


def grid3d_coords(k: int) -> np.ndarray:
    """Boustrophedon ordering of the k^3 lattice; consecutive indices are lattice neighbours."""
    n = k ** 3
    out = np.empty((n, 3), dtype=np.int64)
    kk = k * k
    for i in range(n):
        z = i // kk
        idx = i % kk
        if z & 1:
            idx = kk - 1 - idx
        x, y = _snake_xy(idx, k)
        out[i] = (x, y, z)
    return out


def grid3d_edges(k: int):
    """All 3 k^2 (k-1) axis-aligned lattice-neighbour pairs, oriented low -> high index,
    ordered by (low index, high index)."""
    coords = grid3d_coords(k)
    n = k ** 3
    lut = np.empty((k, k, k), dtype=np.int64)
    lut[coords[:, 0], coords[:, 1], coords[:, 2]] = np.arange(n)
    pairs = []
    for ax in range(3):
        sl_lo = [slice(None)] * 3
        sl_hi = [slice(None)] * 3
        sl_lo[ax] = slice(0, k - 1)
        sl_hi[ax] = slice(1, k)
        a = lut[tuple(sl_lo)].ravel()
        b2 = lut[tuple(sl_hi)].ravel()
        pairs.append(np.stack([np.minimum(a, b2), np.maximum(a, b2)], 1))
    e = np.concatenate(pairs)
    order = np.lexsort((e[:, 1], e[:, 0]))
    return e[order], coords


def _rodrigues(w):
    """Exp: so(3) -> SO(3), written with a fixed operation order (mirrored in C++)."""
    wx, wy, wz = w
    th2 = wx * wx + wy * wy + wz * wz
    th = math.sqrt(th2)
    K = [[0.0, -wz, wy], [wz, 0.0, -wx], [-wy, wx, 0.0]]
    if th < 1e-12:
        A, B = 1.0, 0.5
    else:
        A = math.sin(th) / th
        B = (1.0 - math.cos(th)) / th2
    R = [[0.0] * 3 for _ in range(3)]
    for i in range(3):
        for j in range(3):
            kk = K[i][0] * K[0][j] + K[i][1] * K[1][j] + K[i][2] * K[2][j]
            R[i][j] = (1.0 if i == j else 0.0) + A * K[i][j] + B * kk
    return R


def _quat_rot(q):
    w, x, y, z = q
    nrm = math.sqrt(w * w + x * x + y * y + z * z)
    w, x, y, z = w / nrm, x / nrm, y / nrm, z / nrm
    return [[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
            [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
            [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]]


def _mm3(A, B):
    return [[A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j] for j in range(3)]
            for i in range(3)]


def grid3d(k: int, seed: int = 0, rot_sigma: float = 0.2, trans_sigma: float = 0.1):
    """Synthetic grid pose graph.  Info = smallGrid3D's (trans 100 I, rot 25 I), so the reader
    formulas give kappa = 12.5, tau = 100.  Scalar Python loops (bit-identical to the C++
    generator); intended for k <= ~20 in tests."""
    edges, coords = grid3d_edges(k)
    n = k ** 3
    rng = SplitMix64(seed)
    Rgt = []
    for i in range(n):
        q = [rng.normal() for _ in range(4)]
        Rgt.append(_quat_rot(q))
    m = edges.shape[0]
    R = np.empty((m, 3, 3))
    t = np.empty((m, 3))
    for e in range(m):
        i, j = int(edges[e, 0]), int(edges[e, 1])
        Ri, Rj = Rgt[i], Rgt[j]
        RiT = [[Ri[c][r] for c in range(3)] for r in range(3)]
        eps = [rot_sigma * rng.normal() for _ in range(3)]
        nz = [trans_sigma * rng.normal() for _ in range(3)]
        Rij = _mm3(_mm3(RiT, Rj), _rodrigues(eps))
        dt = [float(coords[j, c] - coords[i, c]) for c in range(3)]
        tij = [RiT[r][0] * dt[0] + RiT[r][1] * dt[1] + RiT[r][2] * dt[2] + nz[r] for r in range(3)]
        R[e] = Rij
        t[e] = tij
    ones = np.ones(m)
    meas = Measurements(3, np.zeros(m, np.int64), np.zeros(m, np.int64), edges[:, 0].copy(),
                        edges[:, 1].copy(), R, t, 12.5 * ones, 100.0 * ones, ones.copy(), n)
    gt = np.zeros((3, 4 * n))
    for i in range(n):
        gt[:, 4 * i:4 * i + 3] = np.array(Rgt[i])
        gt[:, 4 * i + 3] = coords[i]
    meas.extra["ground_truth"] = gt
    meas.extra["coords"] = coords
    return meas


# ----------------------------------------------------------------------------------------
# Connection Laplacian (src/DPGO_utils.cpp:214-286)
# ----------------------------------------------------------------------------------------
def homogeneous(R, t):
    d = R.shape[0]
    T = np.zeros((d + 1, d + 1))
    T[:d, :d] = R
    T[:d, d] = t
    T[d, d] = 1.0
    return T


def connection_laplacian(meas: Measurements, n: int | None = None) -> sp.csr_matrix:
    """Q = A Omega A^T, assembled per edge: Q_ii += T Om T^T, Q_jj += Om, Q_ij = -T Om,
    Q_ji = -Om T^T.  ``n`` defaults to max index + 1 as at :223-228."""
    d = meas.d
    b = d + 1
    if n is None:
        n = int(max(meas.p1.max(), meas.p2.max()) + 1)
    rows, cols, vals = [], [], []
    for e in range(meas.m):
        i, j = int(meas.p1[e]), int(meas.p2[e])
        T = homogeneous(meas.R[e], meas.t[e])
        Om = np.diag([meas.weight[e] * meas.kappa[e]] * d + [meas.weight[e] * meas.tau[e]])
        blocks = [(i, i, T @ Om @ T.T), (j, j, Om), (i, j, -T @ Om), (j, i, -Om @ T.T)]
        for bi, bj, B in blocks:
            rr, cc = np.meshgrid(np.arange(b), np.arange(b), indexing="ij")
            rows.append((bi * b + rr).ravel()); cols.append((bj * b + cc).ravel())
            vals.append(B.ravel())
    if not rows:
        return sp.csr_matrix((b * n, b * n))
    Q = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(b * n, b * n)).tocsr()
    Q.sum_duplicates()
    return Q


def q_to_bsr(Q: sp.csr_matrix, b: int):
    """Block-row storage used by the device: for block-row j, (block col i, B = Q[jb.., ib..])
    with B stored row-major (== block (i,j) column-major, Q symmetric)."""
    Qb = sp.bsr_matrix(Q, blocksize=(b, b))
    Qb.sort_indices()
    return Qb.indptr.astype(np.int32), Qb.indices.astype(np.int32), np.ascontiguousarray(Qb.data)


# ----------------------------------------------------------------------------------------
# Manifold: (St(d, r) x R^r)^n with ROPTLIB Stiefel Set3
# ----------------------------------------------------------------------------------------
def to_poses(X, r, d):
    b = d + 1
    n = X.shape[1] // b
    return X.reshape(r, n, b).transpose(1, 0, 2)


def from_poses(P):
    n, r, b = P.shape
    return P.transpose(1, 0, 2).reshape(r, n * b)


def to_dev(X):
    """r x bn matrix -> device (column-major) flat array."""
    return np.ascontiguousarray(X.T).ravel()


def from_dev(a, r):
    return np.ascontiguousarray(np.asarray(a).reshape(-1, r).T)


def sym(A):
    return 0.5 * (A + np.swapaxes(A, -1, -2))


def tangent_project(X, V, d):
    """ROPTLIB ProductManifold::Projection, Stiefel extrinsic (A.2):
    V_Y - Y sym(Y^T V_Y); translation part unchanged."""
    r = X.shape[0]
    Xp, Vp = to_poses(X, r, d), to_poses(V, r, d)
    Y = Xp[:, :, :d]
    VY = Vp[:, :, :d]
    out = Vp.copy()
    out[:, :, :d] = VY - Y @ sym(np.swapaxes(Y, 1, 2) @ VY)
    return from_poses(out)


def qf(M):
    """Q factor of thin QR with diag(R) > 0 (batched)."""
    Qm, Rm = np.linalg.qr(M)
    s = np.sign(np.diagonal(Rm, axis1=-2, axis2=-1))
    s[s == 0] = 1.0
    return Qm * s[..., None, :]


def retract_qf(X, V, d):
    """ROPTLIB Stiefel QF retraction (A.2): [qf(Y+V_Y) | p+V_p]."""
    r = X.shape[0]
    P = to_poses(X + V, r, d).copy()
    P[:, :, :d] = qf(P[:, :, :d])
    return from_poses(P)


def project_to_stiefel(M):
    """src/DPGO_utils.cpp:494-500: U V^T from the thin SVD (batched)."""
    U, _, Vt = np.linalg.svd(M, full_matrices=False)
    return U @ Vt


def project_to_rotation(M):
    """src/DPGO_utils.cpp:478-492."""
    U, _, Vt = np.linalg.svd(M)
    if np.linalg.det(U) * np.linalg.det(Vt) > 0:
        return U @ Vt
    U = U.copy()
    U[:, -1] *= -1
    return U @ Vt


def lifted_project(M, d):
    """LiftedSEManifold::project (src/manifold/LiftedSEManifold.cpp:34-45)."""
    r = M.shape[0]
    P = to_poses(M, r, d).copy()
    P[:, :, :d] = project_to_stiefel(P[:, :, :d])
    return from_poses(P)


# ----------------------------------------------------------------------------------------
# QuadraticProblem (src/QuadraticProblem.cpp:16-101)
# ----------------------------------------------------------------------------------------
PRECON_EXACT = 0
PRECON_BLOCK_JACOBI = 1
PRECON_NONE = 2


class QuadraticProblem:
    def __init__(self, n, d, r):
        assert r >= d
        self.n, self.d, self.r = n, d, r
        self.b = d + 1
        self.set_Q(sp.csr_matrix((self.b * n, self.b * n)))
        self.G = np.zeros((r, self.b * n))
        self.precon_mode = PRECON_EXACT

    def set_Q(self, Q):
        """:31-42. P = Q + 0.1 I factorised (CHOLMOD in the reference; sparse LU here, exact up to
        rounding).  Block-Jacobi inverses (the north_star's deviation) are cached alongside."""
        N = self.b * self.n
        self.Q = sp.csr_matrix(Q)
        P = (self.Q + 0.1 * sp.identity(N, format="csr")).tocsc()
        try:
            self._lu = spla.splu(P)
        except RuntimeError:
            self._lu = None
        b = self.b
        Pd = P.toarray() if N <= 0 else None  # noqa: F841 (kept for clarity; unused)
        blocks = np.zeros((self.n, b, b))
        Qc = self.Q.tocsr()
        for j in range(self.n):
            blocks[j] = Qc[j * b:(j + 1) * b, j * b:(j + 1) * b].toarray()
        blocks += 0.1 * np.eye(b)
        self.bj_inv = np.linalg.inv(blocks)

    def set_G(self, G):
        """:44-48 (dense r x bn here)."""
        self.G = np.asarray(G, dtype=float).reshape(self.r, self.b * self.n)

    def XQ(self, X):
        return np.asarray((self.Q @ X.T).T)  # Q symmetric

    def f(self, X):
        """:50-60: 0.5 * sum((X Q) o X) + sum(X o G)."""
        return 0.5 * float(np.sum(self.XQ(X) * X)) + float(np.sum(X * self.G))

    def egrad(self, X):
        """:62-66: X Q + G."""
        return self.XQ(X) + self.G

    def ehvp(self, V):
        """:68-73: V Q."""
        return self.XQ(V)

    def riegrad(self, X):
        """:89-97: P_X(X Q + G)."""
        return tangent_project(X, self.egrad(X), self.d)

    def riegrad_norm(self, X):
        return float(np.linalg.norm(self.riegrad(X)))

    def rhvp(self, X, V, EG=None):
        """Riemannian Hessian (A.3): P_X(V Q - [V_Y sym(Y^T EG_Y) | 0])."""
        d, r = self.d, self.r
        if EG is None:
            EG = self.egrad(X)
        HV = to_poses(self.ehvp(V), r, d).copy()
        Xp, Vp, Gp = to_poses(X, r, d), to_poses(V, r, d), to_poses(EG, r, d)
        S = sym(np.swapaxes(Xp[:, :, :d], 1, 2) @ Gp[:, :, :d])
        HV[:, :, :d] -= Vp[:, :, :d] @ S
        return tangent_project(X, from_poses(HV), d)

    def precondition(self, X, V, mode=None):
        """:75-87: P_X(V (Q + 0.1 I)^-1).  EXACT: sparse factor; BLOCK_JACOBI: per-pose
        (Q_jj + 0.1 I)^-1 (north_star deviation); NONE: identity."""
        mode = self.precon_mode if mode is None else mode
        d, r = self.d, self.r
        if mode == PRECON_NONE:
            return V.copy()
        if mode == PRECON_EXACT:
            if self._lu is None:
                return V.copy()  # :84-85 fallback (unprojected)
            out = self._lu.solve(np.ascontiguousarray(V.T)).T
        else:
            Vp = to_poses(V, r, d)
            out = from_poses(Vp @ self.bj_inv)
        return tangent_project(X, out, d)


def certificate_matrix(Q, X, d):
    """Build-defined certificate (absent from the reference so parity-unpinned
    against it): S(X) = Q - Lambda(X), Lambda = blockdiag([sym(Y_j^T (XQ)_{Y_j}) 0; 0 0]).  With
    f = 0.5 tr(X Q X^T) (src/QuadraticProblem.cpp:50-60), X is globally optimal for the rank-r
    relaxation when S(X) >= 0 (the SE-Sync certificate)."""
    Q = sp.csr_matrix(Q)
    b = d + 1
    n = Q.shape[0] // b
    r = X.shape[0]
    EG = np.asarray((Q @ X.T).T)
    Xp, Gp = to_poses(X, r, d), to_poses(EG, r, d)
    S = sym(np.swapaxes(Xp[:, :, :d], 1, 2) @ Gp[:, :, :d])
    L = np.zeros((n, b, b))
    L[:, :d, :d] = S
    return (Q - sp.block_diag(list(L), format="csr")).tocsr()


def round_to_se(X, d):
    """PGOAgent::getTrajectoryInLocalFrame (src/PGOAgent.cpp:481-498): T = Y_0^T X, every rotation
    block projected to SO(d), translations relative to pose 0 (d x (d+1) n)."""
    b = d + 1
    T = X[:, :d].T @ X
    t0 = T[:, d].copy()
    for i in range(X.shape[1] // b):
        T[:, i * b:i * b + d] = project_to_rotation(T[:, i * b:i * b + d])
        T[:, i * b + d] -= t0
    return T


def certificate_min_eig(S):
    """lambda_min of the certificate matrix (dense below 3000 rows, else ARPACK 'SA')."""
    if S.shape[0] <= 3000:
        return float(np.linalg.eigvalsh(S.toarray())[0])
    return float(spla.eigsh(S, k=1, which="SA", tol=1e-12, maxiter=100000)[0][0])


# ----------------------------------------------------------------------------------------
# Riemannian trust region (ROPTLIB RTRNewton / SolversTR, restated in SURVEY Appendix A.4)
# ----------------------------------------------------------------------------------------
TCG_NEGCURVTURE = 0
TCG_EXCREGION = 1
TCG_LCON = 2
TCG_SCON = 3
TCG_MAXITER = 4
TCG_NAMES = ["NEGCURVTURE", "EXCREGION", "LCON", "SCON", "MAXITER"]


def inner(A, B):
    return float(np.sum(A * B))


def tcg(problem: QuadraticProblem, X, grad, EG, Delta, max_inner, min_inner=0, theta=1.0,
        kappa=0.1, trace=None):
    """Preconditioned Steihaug-Toint truncated CG from eta = 0 (A.4)."""
    d = problem.d
    eta = np.zeros_like(X)
    Heta = np.zeros_like(X)
    rvec = grad.copy()
    e_Pe = 0.0
    z = problem.precondition(X, rvec)
    z_r = inner(z, rvec)
    d_Pd = z_r
    delta = -z
    e_Pd = 0.0
    norm_r0 = math.sqrt(inner(rvec, rvec))
    status = TCG_MAXITER
    j = 0
    for j in range(max_inner):
        Hd = problem.rhvp(X, delta, EG)
        d_Hd = inner(delta, Hd)
        alpha = z_r / d_Hd if d_Hd != 0 else math.inf
        e_Pe_new = e_Pe + 2.0 * alpha * e_Pd + alpha * alpha * d_Pd
        rec = dict(j=j, d_Hd=d_Hd, alpha=alpha, e_Pe_new=e_Pe_new)
        if d_Hd <= 0 or e_Pe_new >= Delta * Delta:
            tau = (-e_Pd + math.sqrt(e_Pd * e_Pd + d_Pd * (Delta * Delta - e_Pe))) / d_Pd
            eta = eta + tau * delta
            Heta = Heta + tau * Hd
            status = TCG_NEGCURVTURE if d_Hd <= 0 else TCG_EXCREGION
            rec.update(tau=tau, status=status)
            if trace is not None:
                trace.append(rec)
            j += 1
            break
        e_Pe = e_Pe_new
        eta = eta + alpha * delta
        Heta = Heta + alpha * Hd
        rvec = rvec + alpha * Hd
        norm_r = math.sqrt(inner(rvec, rvec))
        rec.update(norm_r=norm_r)
        if j >= min_inner and norm_r <= norm_r0 * min(norm_r0 ** theta, kappa):
            status = TCG_LCON if kappa < norm_r0 ** theta else TCG_SCON
            rec.update(status=status)
            if trace is not None:
                trace.append(rec)
            j += 1
            break
        z = problem.precondition(X, rvec)
        zold_rold = z_r
        z_r = inner(z, rvec)
        beta = z_r / zold_rold
        delta = -z + beta * delta
        e_Pd = beta * (e_Pd + alpha * d_Pd)
        d_Pd = z_r + beta * beta * d_Pd
        rec.update(z_r=z_r, beta=beta)
        if trace is not None:
            trace.append(rec)
    else:
        j = max_inner
    return eta, Heta, status, j


def rtr_run(problem: QuadraticProblem, X0, tol, Delta0, Delta_max, max_iter, max_inner,
            trace=None):
    """One ROPTLIB RTRNewton::Run() (A.4).  Returns (x, accepted_last, tcg_status, info)."""
    d = problem.d
    x1 = X0.copy()
    EG = problem.egrad(x1)
    f1 = 0.5 * inner(problem.XQ(x1), x1) + inner(x1, problem.G)
    g = tangent_project(x1, EG, d)
    ngf = math.sqrt(inner(g, g))
    Delta = Delta0
    it = 0
    accepted = False
    status = None
    while not (ngf < tol) and it < max_iter:
        tr = [] if trace is not None else None
        eta, Heta, status, ninner = tcg(problem, x1, g, EG, Delta, max_inner, trace=tr)
        x2 = retract_qf(x1, eta, d)
        f2 = problem.f(x2)
        denom = -inner(g, eta) - 0.5 * inner(eta, Heta)
        rho = (f1 - f2) / denom
        accepted = rho > 0.1
        if trace is not None:
            trace.append(dict(iter=it, f1=f1, f2=f2, rho=rho, Delta=Delta, accepted=accepted,
                              ngf=ngf, status=status, ninner=ninner, tcg=tr))
        if rho < 0.25:
            Delta = 0.25 * Delta
        elif rho > 0.75 and status in (TCG_EXCREGION, TCG_NEGCURVTURE):
            Delta = min(2.0 * Delta, Delta_max)
        if accepted:
            x1 = x2
            f1 = f2
            EG = problem.egrad(x1)
            g = tangent_project(x1, EG, d)
            ngf = math.sqrt(inner(g, g))
        it += 1
    return x1, accepted, status, dict(iters=it, ngf=ngf, f=f1, Delta=Delta)


class OptParams:
    """QuadraticOptimizer defaults (src/QuadraticOptimizer.cpp:20-30)."""

    def __init__(self, algorithm="RTR", rgd_stepsize=1e-3, tr_iterations=1, tr_tolerance=1e-2,
                 tr_initial_radius=1e1, tr_max_inner=50):
        self.algorithm = algorithm
        self.rgd_stepsize = rgd_stepsize
        self.tr_iterations = tr_iterations
        self.tr_tolerance = tr_tolerance
        self.tr_initial_radius = tr_initial_radius
        self.tr_max_inner = tr_max_inner


def optimize(problem: QuadraticProblem, Y, params: OptParams, trace=None):
    """QuadraticOptimizer::optimize + trustRegion + gradientDescent
    (src/QuadraticOptimizer.cpp:34-149).  Returns (YOpt, result dict)."""
    res = dict(fInit=problem.f(Y), gradNormInit=problem.riegrad_norm(Y), tCGStatus=None,
               runs=0)
    if params.algorithm == "RTR":
        gn0 = res["gradNormInit"]
        if gn0 < params.tr_tolerance:  # :68-70
            YOpt = Y.copy()
        elif params.tr_iterations == 1:  # :92-110
            radius = params.tr_initial_radius
            total_steps = 0
            while True:
                x, acc, status, info = rtr_run(problem, Y, params.tr_tolerance, radius, radius, 1,
                                               params.tr_max_inner, trace)
                res["runs"] += 1
                res["tCGStatus"] = status
                if acc:
                    YOpt = x
                    break
                elif total_steps > 10:
                    YOpt = Y.copy()
                    break
                radius /= 4.0
                total_steps += 1
        else:
            x, acc, status, info = rtr_run(problem, Y, params.tr_tolerance,
                                           params.tr_initial_radius, 5 * params.tr_initial_radius,
                                           params.tr_iterations, params.tr_max_inner, trace)
            res["runs"] += 1
            res["tCGStatus"] = status
            YOpt = x
    else:  # RGD :124-149
        rg = problem.riegrad(Y)
        YOpt = retract_qf(Y, -params.rgd_stepsize * rg, problem.d)
    res["fOpt"] = problem.f(YOpt)
    res["gradNormOpt"] = problem.riegrad_norm(YOpt)
    res["relativeChange"] = math.sqrt(float(np.sum((YOpt - Y) ** 2)) / problem.n)
    res["success"] = True
    return YOpt, res


# ----------------------------------------------------------------------------------------
# Initialisation helpers (src/DPGO_utils.cpp:377-476) -- one-time host work, test inputs only
# ----------------------------------------------------------------------------------------
def odometry_initialization(d, n, odo: Measurements):
    """src/DPGO_utils.cpp:426-447 (edges must form the chain 0->1->...->n-1)."""
    T = np.zeros((d, n * (d + 1)))
    T[:, :d] = np.eye(d)
    for src in range(odo.m):
        assert odo.p1[src] == src and odo.p2[src] == src + 1
        Rs = T[:, src * (d + 1):src * (d + 1) + d]
        ts = T[:, src * (d + 1) + d]
        dst = src + 1
        T[:, dst * (d + 1):dst * (d + 1) + d] = Rs @ odo.R[src]
        T[:, dst * (d + 1) + d] = ts + Rs @ odo.t[src]
    return T


def chain_initialization(d, n, meas: Measurements):
    """Odometry initialisation along the p2 = p1 + 1 edges of a global chain (used for the
    synthetic grid's snake ordering)."""
    sel = meas.p2 == meas.p1 + 1
    order = np.argsort(meas.p1[sel])
    odo = meas.subset(np.nonzero(sel)[0][order])
    return odometry_initialization(d, n, odo)


def chordal_initialization(d, n, meas: Measurements):
    """src/DPGO_utils.cpp:377-424 with the correct n (B1).  Sparse least squares via the
    normal equations instead of SPQR (same minimiser)."""
    m = meas.m
    d2 = d * d
    # B3: rotations
    rows, cols, vals = [], [], []
    for e in range(m):
        i, j = int(meas.p1[e]), int(meas.p2[e])
        sk = math.sqrt(meas.kappa[e])
        Rm = meas.R[e]
        for r_ in range(d):
            for c in range(d):
                for l in range(d):
                    rows.append(e * d2 + d * r_ + l); cols.append(i * d2 + d * c + l)
                    vals.append(-sk * Rm[c, r_])
        for l in range(d2):
            rows.append(e * d2 + l); cols.append(j * d2 + l); vals.append(sk)
    B3 = sp.csr_matrix((vals, (rows, cols)), shape=(d2 * m, d2 * n))
    Idv = np.eye(d).ravel(order="F")
    cR = B3[:, :d2] @ Idv
    B3r = B3[:, d2:]
    rvec = -spla.spsolve((B3r.T @ B3r).tocsc(), B3r.T @ cR)
    Rch = np.zeros((d, d * n))
    Rch[:, :d] = np.eye(d)
    Rch[:, d:] = rvec.reshape(d, (n - 1) * d, order="F")
    for i in range(1, n):
        Rch[:, i * d:(i + 1) * d] = project_to_rotation(Rch[:, i * d:(i + 1) * d])
    # B1, B2: translations
    rows, cols, vals = [], [], []
    for e in range(m):
        i, j = int(meas.p1[e]), int(meas.p2[e])
        st = math.sqrt(meas.tau[e])
        for l in range(d):
            rows += [e * d + l, e * d + l]; cols += [i * d + l, j * d + l]; vals += [-st, st]
    B1 = sp.csr_matrix((vals, (rows, cols)), shape=(d * m, d * n))
    rows, cols, vals = [], [], []
    for e in range(m):
        i = int(meas.p1[e])
        st = math.sqrt(meas.tau[e])
        for k_ in range(d):
            for r_ in range(d):
                rows.append(d * e + r_); cols.append(d2 * i + d * k_ + r_)
                vals.append(-st * meas.t[e][k_])
    B2 = sp.csr_matrix((vals, (rows, cols)), shape=(d * m, d2 * n))
    c = B2 @ Rch.ravel(order="F")
    B1r = B1[:, d:]
    tred = -spla.spsolve((B1r.T @ B1r).tocsc(), B1r.T @ c)
    tt = np.zeros((d, n))
    tt[:, 1:] = tred.reshape(d, n - 1, order="F")
    T = np.zeros((d, n * (d + 1)))
    for i in range(n):
        T[:, i * (d + 1):i * (d + 1) + d] = Rch[:, i * d:(i + 1) * d]
        T[:, i * (d + 1) + d] = tt[:, i]
    return T


def _bfs_centre(adj, start, member):
    """Middle of a longest breadth-first path found by two sweeps (restates init.cpp's bfs_centre:
    the same visiting order, so the same pose)."""
    def sweep(s):
        dist = {s: 0}
        par = {s: -1}
        q = [s]
        h = 0
        last = s
        while h < len(q):
            v = q[h]
            h += 1
            last = v
            for u in adj[v]:
                if member[u] and u not in dist:
                    dist[u] = dist[v] + 1
                    par[u] = v
                    q.append(u)
        return last, par
    x, _ = sweep(start)
    y, par = sweep(x)
    path = []
    v = y
    while v >= 0:
        path.append(v)
        v = par[v]
    return path[len(path) // 2]


def distributed_initialization(meas: Measurements, agent_of_pose, num_agents):
    """PGOAgent::localInitialization on every agent (chordalInitialization of its private graph,
    src/PGOAgent.cpp:947-962, src/DPGO_utils.cpp:377-476) anchored at the agent's breadth-first centre,
    then initializeInGlobalFrame (:369-432) with an L2 frame average over the shared loop closures,
    agents joining in breadth-first order from the agent holding pose 0.  Returns T (d x (d+1) n)."""
    d = meas.d
    b = d + 1
    n = len(agent_of_pose)
    aop = np.asarray(agent_of_pose)
    adj = [[] for _ in range(n)]
    priv = [e for e in range(meas.m) if aop[meas.p1[e]] == aop[meas.p2[e]]]
    for e in priv:
        i, j = int(meas.p1[e]), int(meas.p2[e])
        adj[i].append(j)
        adj[j].append(i)
    T = np.zeros((d, n * b))
    for a in range(num_agents):
        verts = np.nonzero(aop == a)[0]
        member = aop == a
        c = _bfs_centre(adj, int(verts[0]), member)
        # relabel: anchor first, then the agent's other poses in ascending order
        order = [c] + [int(v) for v in verts if v != c]
        loc = {v: k for k, v in enumerate(order)}
        es = [e for e in priv if aop[meas.p1[e]] == a]
        sub = meas.subset(np.array(es, dtype=np.int64))
        sub.p1 = np.array([loc[int(v)] for v in meas.p1[es]], dtype=np.int64)
        sub.p2 = np.array([loc[int(v)] for v in meas.p2[es]], dtype=np.int64)
        Ta = chordal_initialization(d, len(order), sub)
        for k, v in enumerate(order):
            T[:, v * b:(v + 1) * b] = Ta[:, k * b:(k + 1) * b]
    shared = [[] for _ in range(num_agents)]
    nbr = [set() for _ in range(num_agents)]
    for e in range(meas.m):
        ai, aj = int(aop[meas.p1[e]]), int(aop[meas.p2[e]])
        if ai != aj:
            shared[ai].append(e)
            shared[aj].append(e)
            nbr[ai].add(aj)
            nbr[aj].add(ai)
    FR = np.zeros((num_agents, d, d))
    Ft = np.zeros((num_agents, d))
    done = np.zeros(num_agents, bool)
    root = int(aop[0])
    FR[root] = np.eye(d)
    done[root] = True
    order = [root]

    def world(p):
        a = aop[p]
        return FR[a] @ T[:, p * b:p * b + d], FR[a] @ T[:, p * b + d] + Ft[a]

    h = 0
    while h < len(order):
        for A in sorted(nbr[order[h]]):
            if done[A]:
                continue
            est = []
            for e in shared[A]:
                i, j = int(meas.p1[e]), int(meas.p2[e])
                a_is_j = aop[j] == A
                other = i if a_is_j else j
                if not done[aop[other]]:
                    continue
                Ro, to = world(other)
                if a_is_j:
                    Rw = Ro @ meas.R[e]
                    tw = to + Ro @ meas.t[e]
                else:
                    Rw = Ro @ meas.R[e].T
                    tw = to - Rw @ meas.t[e]
                est.append((j if a_is_j else i, Rw, tw, meas.kappa[e], meas.tau[e]))
            if not est:
                continue
            M = sum(k * (Rw @ T[:, p * b:p * b + d].T) for p, Rw, tw, k, w in est)
            FR[A] = project_to_rotation(M)
            Ft[A] = sum(w * (tw - FR[A] @ T[:, p * b + d]) for p, Rw, tw, k, w in est) / sum(e_[4] for e_ in est)
            done[A] = True
            order.append(A)
        h += 1
    out = np.zeros_like(T)
    for p in range(n):
        Rw, tw = world(p)
        out[:, p * b:p * b + d] = Rw
        out[:, p * b + d] = tw
    return out


def lifting_matrix(d, r, seed=2):
    """Repo-defined YLift: Q factor of a seeded Gaussian r x d (SplitMix64)."""
    rng = SplitMix64(seed)
    M = np.array([[rng.normal() for _ in range(d)] for _ in range(r)])
    return qf(M)


def measurement_error(R, t, Y1, p1, Y2, p2, kappa, tau):
    """src/DPGO_utils.cpp:509-515."""
    return kappa * float(np.sum((Y1 @ R - Y2) ** 2)) + tau * float(np.sum((p2 - p1 - Y1 @ t) ** 2))


# ----------------------------------------------------------------------------------------
# Robust cost weights (src/DPGO_robust.cpp:23-103)  (GNC is SURVEY 8f "next"; oracle only)
# ----------------------------------------------------------------------------------------
class RobustCost:
    def __init__(self, kind="L2", gnc_max_iters=100, gnc_barc=10.0, gnc_mu_step=1.4,
                 gnc_init_mu=1e-4, huber=3.0, tls=10.0):
        self.kind = kind
        self.p = dict(max_iters=gnc_max_iters, barc=gnc_barc, mu_step=gnc_mu_step,
                      init_mu=gnc_init_mu, huber=huber, tls=tls)
        self.reset()

    def reset(self):
        self.mu = self.p["init_mu"]
        self.iteration = 0

    def weight(self, rr):
        k = self.kind
        if k == "L2":
            return 1.0
        if k == "L1":
            return 1.0 / rr
        if k == "Huber":
            return 1.0 if rr < self.p["huber"] else self.p["huber"] / rr
        if k == "TLS":
            return 1.0 if rr < self.p["tls"] else 0.0
        if k == "GM":
            a = 1 + rr * rr
            return 1.0 / (a * a)
        if k == "GNC_TLS":
            rsq = rr * rr
            bc = self.p["barc"] ** 2
            mu = self.mu
            if rsq >= (mu + 1) / mu * bc:
                return 0.0
            if rsq <= mu / (mu + 1) * bc:
                return 1.0
            return math.sqrt(bc * mu * (mu + 1) / rsq) - mu
        raise ValueError(k)

    def update(self):
        if self.kind != "GNC_TLS":
            return
        self.iteration += 1
        if self.iteration > self.p["max_iters"]:
            return
        self.mu = self.p["mu_step"] * self.mu


# ----------------------------------------------------------------------------------------
# PGOAgent RBCD-round portion (src/PGOAgent.cpp:55-124, 434-479, 642-859, 1033-1165)
# ----------------------------------------------------------------------------------------
class AgentParams:
    """include/DPGO/PGOAgent.h:59-136 defaults."""

    def __init__(self, d, r, num_robots=1, algorithm="RTR", acceleration=False,
                 restart_interval=30, robust="GNC_TLS", robust_opt_inner_iters=30,
                 robust_opt_min_convergence_ratio=0.8, rel_change_tol=5e-3,
                 precon=PRECON_EXACT):
        self.d, self.r, self.num_robots = d, r, num_robots
        self.algorithm = algorithm
        self.acceleration = acceleration
        self.restart_interval = restart_interval
        self.robust = robust
        self.robust_opt_inner_iters = robust_opt_inner_iters
        self.robust_opt_min_convergence_ratio = robust_opt_min_convergence_ratio
        self.rel_change_tol = rel_change_tol
        self.precon = precon


class Agent:
    def __init__(self, agent_id, params: AgentParams):
        self.id = agent_id
        self.p = params
        self.d, self.r = params.d, params.r
        self.n = 1
        self.iteration = 0
        self.initialized = False
        self.robust = RobustCost(params.robust)
        self.neighbor_pose = {}
        self.neighbor_aux_pose = {}
        self.X = None
        self.gamma = self.alpha = 0.0
        self.last_result = None
        self.status_relative_change = 0.0
        self.ready_to_terminate = False

    # --- setPoseGraph (:126-195) --------------------------------------------------------
    def set_pose_graph(self, odometry: Measurements, private_lc: Measurements,
                       shared_lc: Measurements, n=None):
        self.odometry, self.private_lc, self.shared_lc = odometry, private_lc, shared_lc
        nmax = 1
        for M_ in (odometry, private_lc):
            if M_.m:
                nmax = max(nmax, int(max(M_.p1.max(), M_.p2.max())) + 1)
        for e in range(shared_lc.m):
            own = shared_lc.p1[e] if shared_lc.r1[e] == self.id else shared_lc.p2[e]
            nmax = max(nmax, int(own) + 1)
        self.n = nmax if n is None else n
        self.local_shared = set()
        self.neighbor_shared = set()
        for e in range(shared_lc.m):
            if shared_lc.r1[e] == self.id:
                self.local_shared.add((self.id, int(shared_lc.p1[e])))
                self.neighbor_shared.add((int(shared_lc.r2[e]), int(shared_lc.p2[e])))
            else:
                self.local_shared.add((self.id, int(shared_lc.p2[e])))
                self.neighbor_shared.add((int(shared_lc.r1[e]), int(shared_lc.p1[e])))
        self.problem = QuadraticProblem(self.n, self.d, self.r)
        self.problem.precon_mode = self.p.precon
        self.construct_Q()

    def private_measurements(self) -> Measurements:
        return _concat(self.odometry, self.private_lc)

    # --- constructQMatrix (:720-781) ----------------------------------------------------
    def construct_Q(self):
        d, b = self.d, self.d + 1
        Q = connection_laplacian(self.private_measurements(), self.n).tolil()
        sh = self.shared_lc
        for e in range(sh.m):
            T = homogeneous(sh.R[e], sh.t[e])
            Om = np.diag([sh.weight[e] * sh.kappa[e]] * d + [sh.weight[e] * sh.tau[e]])
            if sh.r1[e] == self.id:
                idx = int(sh.p1[e])
                W = T @ Om @ T.T
            else:
                idx = int(sh.p2[e])
                W = Om
            Q[idx * b:(idx + 1) * b, idx * b:(idx + 1) * b] = \
                Q[idx * b:(idx + 1) * b, idx * b:(idx + 1) * b].toarray() + W
        self.problem.set_Q(Q.tocsr())

    # --- constructGMatrix (:783-859) ----------------------------------------------------
    def construct_G(self, pose_dict):
        d, b, r = self.d, self.d + 1, self.r
        G = np.zeros((r, b * self.n))
        sh = self.shared_lc
        for e in range(sh.m):
            T = homogeneous(sh.R[e], sh.t[e])
            Om = np.diag([sh.weight[e] * sh.kappa[e]] * d + [sh.weight[e] * sh.tau[e]])
            if sh.r1[e] == self.id:
                key = (int(sh.r2[e]), int(sh.p2[e]))
                if key not in pose_dict:
                    return False
                L = -pose_dict[key] @ Om @ T.T
                idx = int(sh.p1[e])
            else:
                key = (int(sh.r1[e]), int(sh.p1[e]))
                if key not in pose_dict:
                    return False
                L = -pose_dict[key] @ T @ Om
                idx = int(sh.p2[e])
            G[:, idx * b:(idx + 1) * b] += L
        self.problem.set_G(G)
        return True

    # --- poses ---------------------------------------------------------------------------
    def set_X(self, X):
        """:55-68"""
        self.X = np.array(X, dtype=float)
        self.initialized = True
        if self.p.acceleration:
            self.initialize_acceleration()

    def initialize_acceleration(self):
        """:1062-1071"""
        self.XPrev = self.X.copy()
        self.gamma = 0.0
        self.alpha = 0.0
        self.V = self.X.copy()
        self.Y = self.X.copy()

    def shared_pose_dict(self, aux=False):
        """:95-118"""
        src = self.Y if aux else self.X
        b = self.d + 1
        return {pid: src[:, pid[1] * b:(pid[1] + 1) * b].copy() for pid in sorted(self.local_shared)}

    def update_neighbor_poses(self, neighbor_id, pose_dict, aux=False):
        """:434-479 (both agents initialised)."""
        dst = self.neighbor_aux_pose if aux else self.neighbor_pose
        for pid, v in pose_dict.items():
            assert pid[0] == neighbor_id
            if pid in self.neighbor_shared:
                dst[pid] = v.copy()

    # --- Nesterov (:1033-1091) -----------------------------------------------------------
    def update_gamma(self):
        N = self.p.num_robots
        self.gamma = (1 + math.sqrt(1 + 4 * N ** 2 * self.gamma ** 2)) / (2 * N)

    def update_alpha(self):
        self.alpha = 1 / (self.gamma * self.p.num_robots)

    def update_Y(self):
        self.Y = lifted_project((1 - self.alpha) * self.X + self.alpha * self.V, self.d)

    def update_V(self):
        self.V = lifted_project(self.V + self.gamma * (self.X - self.Y), self.d)

    # --- updateX (:1093-1165) ------------------------------------------------------------
    def update_X(self, do_opt, accel, trace=None):
        if not do_opt:
            if accel:
                self.X = self.Y
            return True
        if self.p.robust != "L2":
            self.construct_Q()
        ok = self.construct_G(self.neighbor_aux_pose if accel else self.neighbor_pose)
        if not ok:
            return False
        params = OptParams(algorithm=self.p.algorithm, tr_iterations=1, tr_tolerance=1e-2,
                           tr_initial_radius=100.0, tr_max_inner=10)
        X0 = self.Y if accel else self.X
        self.X, self.last_result = optimize(self.problem, X0, params, trace)
        return True

    # --- GNC (:1174-1289) ------------------------------------------------------------------
    def should_update_weights(self):
        if self.p.robust == "L2":
            return False
        return (self.iteration + 1) % self.p.robust_opt_inner_iters == 0

    def update_loop_closure_weights(self):
        d, b = self.d, self.d + 1
        X = self.X
        pl = self.private_lc
        for e in range(pl.m):
            i, j = int(pl.p1[e]), int(pl.p2[e])
            res = math.sqrt(measurement_error(pl.R[e], pl.t[e], X[:, i * b:i * b + d],
                                              X[:, i * b + d], X[:, j * b:j * b + d],
                                              X[:, j * b + d], pl.kappa[e], pl.tau[e]))
            pl.weight[e] = self.robust.weight(res)
        sh = self.shared_lc
        for e in range(sh.m):
            if sh.r1[e] == self.id:
                if sh.r2[e] < self.id:
                    continue
                i = int(sh.p1[e])
                Y1, q1 = X[:, i * b:i * b + d], X[:, i * b + d]
                key = (int(sh.r2[e]), int(sh.p2[e]))
                if key not in self.neighbor_pose:
                    continue
                X2 = self.neighbor_pose[key]
                Y2, q2 = X2[:, :d], X2[:, d]
            else:
                if sh.r1[e] < self.id:
                    continue
                j = int(sh.p2[e])
                Y2, q2 = X[:, j * b:j * b + d], X[:, j * b + d]
                key = (int(sh.r1[e]), int(sh.p1[e]))
                if key not in self.neighbor_pose:
                    continue
                X1 = self.neighbor_pose[key]
                Y1, q1 = X1[:, :d], X1[:, d]
            res = math.sqrt(measurement_error(sh.R[e], sh.t[e], Y1, q1, Y2, q2, sh.kappa[e],
                                              sh.tau[e]))
            sh.weight[e] = self.robust.weight(res)

    # --- iterate (:642-718) ----------------------------------------------------------------
    def iterate(self, do_opt=True, trace=None):
        self.iteration += 1
        if self.should_update_weights():
            self.update_loop_closure_weights()
            self.robust.update()
            if self.p.acceleration:
                self.initialize_acceleration()
        if not self.initialized:
            return
        self.XPrev = self.X.copy()
        if self.p.acceleration:
            self.update_gamma()
            self.update_alpha()
            self.update_Y()
            success = self.update_X(do_opt, True, trace)
            self.update_V()
            if (self.iteration + 1) % self.p.restart_interval == 0:  # shouldRestart :1033-1038
                self.X = self.XPrev
                self.update_X(do_opt, False, trace)
                self.V = self.X.copy()
                self.Y = self.X.copy()
                self.gamma = 0.0
                self.alpha = 0.0
        else:
            success = self.update_X(do_opt, False, trace)
        if do_opt:
            self.status_relative_change = math.sqrt(float(np.sum((self.X - self.XPrev) ** 2)) / self.n)
            ready = bool(success) and not (self.status_relative_change > self.p.rel_change_tol)
            if self.converged_loop_closure_ratio() < self.p.robust_opt_min_convergence_ratio:
                ready = False
            self.ready_to_terminate = ready

    def converged_loop_closure_ratio(self):
        """computeConvergedLoopClosureRatio (:1247-1289): GNC_TLS only; loop closures whose weight is
        exactly 1 or 0 over all private and shared loop closures (0/0 = NaN, as there)."""
        if self.p.robust != "GNC_TLS":
            return 1.0
        w = np.concatenate([self.private_lc.weight, self.shared_lc.weight])
        conv = float(np.sum((w == 1.0) | (w == 0.0)))
        return conv / len(w) if len(w) else float("nan")

    def trajectory_local_frame(self):
        """:481-498"""
        d, b = self.d, self.d + 1
        T = self.X[:, :d].T @ self.X
        t0 = T[:, d].copy()
        for i in range(self.n):
            T[:, i * b:i * b + d] = project_to_rotation(T[:, i * b:i * b + d])
            T[:, i * b + d] = T[:, i * b + d] - t0
        return T


def _concat(a: Measurements, b2: Measurements) -> Measurements:
    return Measurements(a.d if a.m else b2.d, np.concatenate([a.r1, b2.r1]),
                        np.concatenate([a.r2, b2.r2]), np.concatenate([a.p1, b2.p1]),
                        np.concatenate([a.p2, b2.p2]),
                        np.concatenate([a.R, b2.R]).reshape(-1, a.d or b2.d, a.d or b2.d),
                        np.concatenate([a.t, b2.t]).reshape(-1, a.d or b2.d),
                        np.concatenate([a.kappa, b2.kappa]), np.concatenate([a.tau, b2.tau]),
                        np.concatenate([a.weight, b2.weight]), max(a.num_poses, b2.num_poses))


# ----------------------------------------------------------------------------------------
# Partitioning + drivers (examples/MultiRobotExample.cpp:73-264)
# ----------------------------------------------------------------------------------------
def partition_contiguous(meas: Measurements, n, num_robots):
    """:73-121: contiguous index ranges; the last robot takes the remainder."""
    per = n // num_robots
    assert per > 0
    robot_of = np.minimum(np.arange(n) // per, num_robots - 1)
    start = np.array([rb * per for rb in range(num_robots)] + [n])
    local = np.arange(n) - start[robot_of]
    return _split(meas, robot_of, local, num_robots), robot_of, local, start


def _split(meas, robot_of, local, num_robots):
    odo = [[] for _ in range(num_robots)]
    priv = [[] for _ in range(num_robots)]
    shared = [[] for _ in range(num_robots)]
    sr = robot_of[meas.p1]; dr = robot_of[meas.p2]
    sl = local[meas.p1]; dl = local[meas.p2]
    for e in range(meas.m):
        if sr[e] == dr[e]:
            (odo if sl[e] + 1 == dl[e] else priv)[sr[e]].append(e)
        else:
            shared[sr[e]].append(e)
            shared[dr[e]].append(e)
    out = []
    for rb in range(num_robots):
        parts = []
        for lst in (odo[rb], priv[rb], shared[rb]):
            idx = np.array(lst, dtype=np.int64)
            M_ = meas.subset(idx) if len(idx) else Measurements(
                meas.d, np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64),
                np.zeros(0, np.int64), np.zeros((0, meas.d, meas.d)), np.zeros((0, meas.d)),
                np.zeros(0), np.zeros(0), np.zeros(0))
            if len(idx):
                M_.r1 = sr[idx].astype(np.int64); M_.r2 = dr[idx].astype(np.int64)
                M_.p1 = sl[idx].astype(np.int64); M_.p2 = dl[idx].astype(np.int64)
            parts.append(M_)
        out.append(tuple(parts))
    return out


def multi_robot_example(meas: Measurements, num_robots, r=5, num_iters=100, acceleration=True,
                        robust="GNC_TLS", precon=PRECON_EXACT, X_init=None, verbose=False, robust_opt_inner_iters=30):
    """Serialized greedy RBCD (examples/MultiRobotExample.cpp:21-282) with the App. B fixes.
    Returns a per-iteration log [(iter, robot, 2f, gradnorm)] and the final X."""
    d = meas.d
    n = meas.num_poses or int(max(meas.p1.max(), meas.p2.max()) + 1)
    Qc = connection_laplacian(meas, n)
    central = QuadraticProblem(n, d, r)
    central.Q = Qc
    parts, robot_of, local, start = partition_contiguous(meas, n, num_robots)
    agents = []
    for rb in range(num_robots):
        ag = Agent(rb, AgentParams(d, r, num_robots, acceleration=acceleration, robust=robust,
                                   precon=precon, robust_opt_inner_iters=robust_opt_inner_iters))
        ag.set_pose_graph(*parts[rb], n=int(start[rb + 1] - start[rb]))
        agents.append(ag)
    if X_init is None:
        T = chordal_initialization(d, n, meas)
        X_init = lifting_matrix(d, r) @ T
    b = d + 1
    for rb, ag in enumerate(agents):
        ag.set_X(X_init[:, start[rb] * b:start[rb + 1] * b])
    log = []
    selected = 0
    Xopt = X_init.copy()
    for it in range(num_iters):
        sel = agents[selected]
        for ag in agents:
            if ag.id != selected:
                ag.iterate(False)
        for ag in agents:
            if ag.id == selected:
                continue
            sel.update_neighbor_poses(ag.id, ag.shared_pose_dict(False), aux=False)
        if acceleration:
            for ag in agents:
                if ag.id == selected:
                    continue
                sel.update_neighbor_poses(ag.id, ag.shared_pose_dict(True), aux=True)
        sel.iterate(True)
        for rb, ag in enumerate(agents):
            Xopt[:, start[rb] * b:start[rb + 1] * b] = ag.X
        RG = tangent_project(Xopt, central.XQ(Xopt), d)
        gn = float(np.linalg.norm(RG))
        cost = 2 * 0.5 * inner(central.XQ(Xopt), Xopt)
        log.append((it, selected, cost, gn))
        if verbose:
            print(f"Iter = {it} | robot = {selected} | cost = {cost:.6g} | gradnorm = {gn:.6g}")
        if gn < 0.1:
            break
        neighbors = sorted({int(x[0]) for x in sel.neighbor_shared})
        if not neighbors:
            selected = sel.id
        else:
            norms = [float(np.linalg.norm(RG[:, start[rb] * b:start[rb + 1] * b]))
                     for rb in range(num_robots)]
            selected = int(np.argmax(norms))
    return log, Xopt


def central_cost(meas: Measurements, X, n=None):
    """Full-graph f(X) with G = 0 (the drivers print 2f)."""
    d = meas.d
    Qc = connection_laplacian(meas, n)
    return 0.5 * inner(np.asarray((Qc @ X.T).T), X)


def greedy_colors(meas: Measurements, agent_of_pose, num_agents):
    """Greedy colouring of the agent-adjacency graph in agent-id order (repo-defined schedule)."""
    adj = [set() for _ in range(num_agents)]
    for e in range(meas.m):
        a1, a2 = int(agent_of_pose[meas.p1[e]]), int(agent_of_pose[meas.p2[e]])
        if a1 != a2:
            adj[a1].add(a2)
            adj[a2].add(a1)
    col = [-1] * num_agents
    for a in range(num_agents):
        used = {col[b2] for b2 in adj[a] if col[b2] >= 0}
        c = 0
        while c in used:
            c += 1
        col[a] = c
    return col


def colour_rbcd(meas: Measurements, agent_of_pose, num_agents, X0, num_iters, r,
                acceleration=False, robust="L2", precon=PRECON_BLOCK_JACOBI, trace=None,
                robust_opt_inner_iters=30, agents_out=None, algorithm="RTR"):
    """Colour-class RBCD schedule run with the PGOAgent restatement: at iteration t the agents of
    colour t mod C are selected; the others run iterate(false) first (their public X / aux Y are
    then delivered, as in examples/MultiRobotExample.cpp:181-213), then the selected agents run
    iterate(true).  Returns the global X after num_iters iterations."""
    d = meas.d
    b = d + 1
    n = len(agent_of_pose)
    agent_of_pose = np.asarray(agent_of_pose)
    local = np.zeros(n, np.int64)
    counts = np.zeros(num_agents, np.int64)
    for i in range(n):
        a = agent_of_pose[i]
        local[i] = counts[a]
        counts[a] += 1
    parts = _split(meas, agent_of_pose, local, num_agents)
    glob = [np.nonzero(agent_of_pose == a)[0] for a in range(num_agents)]
    agents = []
    for a in range(num_agents):
        ag = Agent(a, AgentParams(d, r, num_agents, acceleration=acceleration, robust=robust,
                                  precon=precon, robust_opt_inner_iters=robust_opt_inner_iters,
                                  algorithm=algorithm))
        ag.set_pose_graph(*parts[a], n=int(counts[a]))
        cols = np.concatenate([np.arange(p * b, (p + 1) * b) for p in glob[a]])
        ag.set_X(X0[:, cols])
        agents.append(ag)
    if agents_out is not None:
        agents_out.extend(agents)
    colors = greedy_colors(meas, agent_of_pose, num_agents)
    C = max(colors) + 1
    for it in range(num_iters):
        c = it % C
        for ag in agents:
            if colors[ag.id] != c:
                ag.iterate(False)
        for ag in agents:
            if colors[ag.id] != c:
                continue
            for other in agents:
                if other.id == ag.id:
                    continue
                ag.update_neighbor_poses(other.id, other.shared_pose_dict(False), aux=False)
                if acceleration:
                    ag.update_neighbor_poses(other.id, other.shared_pose_dict(True), aux=True)
        for ag in agents:
            if colors[ag.id] == c:
                ag.iterate(True, trace)  # RTR outer records of the update, then (it, agent, result)
                if trace is not None:
                    trace.append((it, ag.id, ag.last_result))
    X = np.zeros_like(X0)
    for a, ag in enumerate(agents):
        cols = np.concatenate([np.arange(p * b, (p + 1) * b) for p in glob[a]])
        X[:, cols] = ag.X
    return X, colors
