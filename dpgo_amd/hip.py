"""ctypes binding of libdpgo_hip.so (include/dpgo_hip.h).

This is the Python-side binding a maintainer would add next to the reference's C++ API; it is
used by the test-suite, ``bench.py`` and the multi-GPU RBCD driver.  It never falls back to a
CPU implementation: if the shared library or a gfx950 device is missing, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdpgo_hip.so")

PRECON_EXACT, PRECON_BLOCK_JACOBI, PRECON_NONE = 0, 1, 2
ALG_RTR, ALG_RGD = 0, 1
TCG_NAMES = {-1: "NONE", 0: "NEGCURVTURE", 1: "EXCREGION", 2: "LCON", 3: "SCON", 4: "MAXITER"}

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


class OptParams(C.Structure):
    _fields_ = [("algorithm", C.c_int), ("rgd_stepsize", C.c_double), ("tr_iterations", C.c_int),
                ("tr_tolerance", C.c_double), ("tr_initial_radius", C.c_double),
                ("tr_max_inner", C.c_int), ("verbose", C.c_int), ("precon", C.c_int)]


class OptResult(C.Structure):
    _fields_ = [("success", C.c_int), ("fInit", C.c_double), ("gradNormInit", C.c_double),
                ("fOpt", C.c_double), ("gradNormOpt", C.c_double), ("relativeChange", C.c_double),
                ("elapsedMs", C.c_double), ("tCGStatus", C.c_int), ("runs", C.c_int),
                ("outer_iters", C.c_int), ("inner_iters", C.c_int), ("gave_up", C.c_int)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class DPGOHipError(RuntimeError):
    pass


_lib = None

# (name, argtypes, restype)
_SIGS = [
    ("dpgo_hip_version", [], C.c_char_p),
    ("dpgo_hip_last_error", [], C.c_char_p),
    ("dpgo_hip_device_count", [], C.c_int),
    ("dpgo_hip_default_params", [C.POINTER(OptParams)], None),
    ("dpgo_hip_problem_create", [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    ("dpgo_hip_problem_create_batch", [C.c_int, _ip, C.c_int, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    ("dpgo_hip_problem_destroy", [C.c_void_p], C.c_int),
    ("dpgo_hip_problem_set_stream", [C.c_void_p, C.c_void_p], C.c_int),
    ("dpgo_hip_problem_info", [C.c_void_p, _ip, _ip, _ip, _ip], C.c_int),
    ("dpgo_hip_set_precon", [C.c_void_p, C.c_int], C.c_int),
    ("dpgo_hip_set_Q_csr", [C.c_void_p, C.c_int, C.c_int, _ip, _ip, _dp], C.c_int),
    ("dpgo_hip_set_Q_bsr", [C.c_void_p, C.c_int, C.c_int, _ip, _ip, _dp], C.c_int),
    ("dpgo_hip_set_G", [C.c_void_p, C.c_int, C.c_int, _ip, _dp], C.c_int),
    ("dpgo_hip_set_G_dense", [C.c_void_p, C.c_int, _dp], C.c_int),
    ("dpgo_hip_f", [C.c_void_p, _dp, _dp], C.c_int),
    ("dpgo_hip_egrad", [C.c_void_p, _dp, _dp], C.c_int),
    ("dpgo_hip_ehvp", [C.c_void_p, _dp, _dp], C.c_int),
    ("dpgo_hip_riegrad", [C.c_void_p, _dp, _dp, _dp, _dp], C.c_int),
    ("dpgo_hip_rhvp", [C.c_void_p, _dp, _dp, _dp], C.c_int),
    ("dpgo_hip_precondition", [C.c_void_p, _dp, _dp, _dp], C.c_int),
    ("dpgo_hip_tangent_project", [C.c_int, C.c_int, C.c_int, _dp, _dp, _dp], C.c_int),
    ("dpgo_hip_retract_qf", [C.c_int, C.c_int, C.c_int, _dp, _dp, C.c_double, _dp], C.c_int),
    ("dpgo_hip_project_polar", [C.c_int, C.c_int, C.c_int, _dp, _dp], C.c_int),
    ("dpgo_hip_optimize", [C.c_void_p, C.POINTER(OptParams), _dp, _dp, C.POINTER(OptResult)], C.c_int),
    ("dpgo_hip_f_dev", [C.c_void_p, C.c_void_p, _dp], C.c_int),
    ("dpgo_hip_egrad_dev", [C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    ("dpgo_hip_ehvp_dev", [C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    ("dpgo_hip_riegrad_dev", [C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    ("dpgo_hip_rhvp_dev", [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    ("dpgo_hip_project_polar_dev", [C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    ("dpgo_hip_polar_combine_dev", [C.c_void_p, C.c_void_p, C.c_void_p, _dp, _dp, C.c_void_p], C.c_int),
    ("dpgo_hip_optimize_dev", [C.c_void_p, C.POINTER(OptParams), C.c_void_p, C.c_void_p, _ip,
                               C.POINTER(OptResult)], C.c_int),
    ("dpgo_hip_synchronize", [C.c_void_p], C.c_int),
    ("dpgo_hip_spmm_bytes", [C.c_void_p], C.c_double),
    ("dpgo_hip_bench_spmm", [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, _dp], C.c_int),
]

EXPORTED_SYMBOLS = [s[0] for s in _SIGS]


def lib():
    """Load libdpgo_hip.so (built in-tree by __graft_entry__.build()).  Raises if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DPGOHipError(f"{LIB_PATH} not built: run __graft_entry__.build() (no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, args, res in _SIGS:
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise DPGOHipError(f"dpgo_hip error {rc}: {lib().dpgo_hip_last_error().decode()}")


def _f64(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(_dp)


def _i32(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(_ip)


def device_count() -> int:
    return int(lib().dpgo_hip_device_count())


def default_params(**kw) -> OptParams:
    p = OptParams()
    lib().dpgo_hip_default_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


# ----------------------------------------------------------------------------------------
# Layout helpers: the C ABI uses the reference's column-major r x (b n) layout.
# ----------------------------------------------------------------------------------------
def to_dev_layout(X: np.ndarray) -> np.ndarray:
    """r x (b n) matrix -> flat column-major buffer."""
    return np.ascontiguousarray(np.asarray(X, dtype=np.float64).T).ravel()


def from_dev_layout(a: np.ndarray, r: int) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a).reshape(-1, r).T)


class Problem:
    """Batched QuadraticProblem handle (one agent = the reference's QuadraticProblem)."""

    def __init__(self, n, d, r, poses_per_agent=None):
        self.d, self.r, self.b = d, r, d + 1
        h = C.c_void_p()
        if poses_per_agent is None:
            _check(lib().dpgo_hip_problem_create(int(n), d, r, C.byref(h)))
            self.poses = [int(n)]
        else:
            arr, ptr = _i32(poses_per_agent)
            _check(lib().dpgo_hip_problem_create_batch(len(arr), ptr, d, r, C.byref(h)))
            self.poses = [int(x) for x in arr]
        self.h = h
        self.K = len(self.poses)
        self.N = int(sum(self.poses))
        self.offsets = np.concatenate([[0], np.cumsum(self.poses)]).astype(np.int64)

    def close(self):
        if getattr(self, "h", None):
            lib().dpgo_hip_problem_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def vec_len(self):
        return self.N * self.r * self.b

    def set_stream(self, stream_ptr: int | None):
        _check(lib().dpgo_hip_problem_set_stream(self.h, C.c_void_p(stream_ptr or 0)))

    def set_precon(self, mode):
        _check(lib().dpgo_hip_set_precon(self.h, mode))

    def set_Q_bsr(self, agent, browptr, bcol, blocks_colmajor):
        rp, rpp = _i32(browptr)
        cc, ccp = _i32(bcol)
        bb, bbp = _f64(blocks_colmajor)
        self._keep = (rp, cc, bb)
        _check(lib().dpgo_hip_set_Q_bsr(self.h, agent, len(rp) - 1, rpp, ccp, bbp))

    def set_Q_csr(self, agent, indptr, indices, data):
        rp, rpp = _i32(indptr)
        cc, ccp = _i32(indices)
        dd, ddp = _f64(data)
        _check(lib().dpgo_hip_set_Q_csr(self.h, agent, len(rp) - 1, rpp, ccp, ddp))

    def set_Q_scipy(self, agent, Q):
        """Q: scipy sparse (b n_a x b n_a) symmetric; uploaded as BSR with column-major blocks."""
        import scipy.sparse as sp
        Qb = sp.bsr_matrix(Q, blocksize=(self.b, self.b))
        Qb.sort_indices()
        self.set_Q_bsr(agent, Qb.indptr, Qb.indices, np.ascontiguousarray(Qb.data.transpose(0, 2, 1)))

    def set_G_dense(self, agent, G):
        """G: r x (b n_a) matrix."""
        g, gp = _f64(to_dev_layout(G))
        _check(lib().dpgo_hip_set_G_dense(self.h, agent, gp))

    def set_G_blocks(self, agent, pose_idx, blocks):
        """blocks: (count, r, b) pose blocks."""
        idx, ip = _i32(pose_idx)
        bl = np.ascontiguousarray(np.asarray(blocks, dtype=np.float64).transpose(0, 2, 1)).ravel()
        bl, bp = _f64(bl)
        _check(lib().dpgo_hip_set_G(self.h, agent, len(idx), ip, bp))

    # --- evaluations on host matrices (r x (b N)) ----------------------------------------
    def _in(self, X):
        return _f64(to_dev_layout(X))

    def _out(self):
        o = np.empty(self.vec_len)
        return o, o.ctypes.data_as(_dp)

    def f(self, X):
        x, xp = self._in(X)
        out = np.empty(self.K)
        _check(lib().dpgo_hip_f(self.h, xp, out.ctypes.data_as(_dp)))
        return out

    def egrad(self, X):
        x, xp = self._in(X)
        o, op = self._out()
        _check(lib().dpgo_hip_egrad(self.h, xp, op))
        return from_dev_layout(o, self.r)

    def ehvp(self, V):
        x, xp = self._in(V)
        o, op = self._out()
        _check(lib().dpgo_hip_ehvp(self.h, xp, op))
        return from_dev_layout(o, self.r)

    def riegrad(self, X):
        x, xp = self._in(X)
        o, op = self._out()
        norms = np.empty(self.K)
        fv = np.empty(self.K)
        _check(lib().dpgo_hip_riegrad(self.h, xp, op, norms.ctypes.data_as(_dp), fv.ctypes.data_as(_dp)))
        return from_dev_layout(o, self.r), norms, fv

    def rhvp(self, X, V):
        x, xp = self._in(X)
        v, vp = self._in(V)
        o, op = self._out()
        _check(lib().dpgo_hip_rhvp(self.h, xp, vp, op))
        return from_dev_layout(o, self.r)

    def precondition(self, X, V):
        x, xp = self._in(X)
        v, vp = self._in(V)
        o, op = self._out()
        _check(lib().dpgo_hip_precondition(self.h, xp, vp, op))
        return from_dev_layout(o, self.r)

    def optimize(self, X, params: OptParams | None = None):
        x, xp = self._in(X)
        o, op = self._out()
        res = (OptResult * self.K)()
        p = params or default_params()
        _check(lib().dpgo_hip_optimize(self.h, C.byref(p), xp, op, res))
        return from_dev_layout(o, self.r), [r.as_dict() for r in res]

    # --- device pointers ---------------------------------------------------------------------
    def optimize_dev(self, X_dev: int, X_out_dev: int, params: OptParams | None = None, enabled=None):
        res = (OptResult * self.K)()
        p = params or default_params()
        if enabled is not None:
            en, enp = _i32(enabled)
        else:
            enp = None
        _check(lib().dpgo_hip_optimize_dev(self.h, C.byref(p), C.c_void_p(X_dev), C.c_void_p(X_out_dev),
                                           enp, res))
        return [r.as_dict() for r in res]

    def polar_combine_dev(self, A_dev, B_dev, ca, cb, out_dev):
        a, ap = _f64(ca)
        if B_dev is not None:
            b, bp = _f64(cb)
        else:
            bp = None
        _check(lib().dpgo_hip_polar_combine_dev(self.h, C.c_void_p(A_dev), C.c_void_p(B_dev or 0), ap, bp,
                                                C.c_void_p(out_dev)))

    def spmm_bytes(self) -> float:
        return float(lib().dpgo_hip_spmm_bytes(self.h))

    def bench_spmm(self, X_dev: int, Y_dev: int, reps: int) -> float:
        ms = C.c_double()
        _check(lib().dpgo_hip_bench_spmm(self.h, C.c_void_p(X_dev), C.c_void_p(Y_dev), reps, C.byref(ms)))
        return ms.value

    def synchronize(self):
        _check(lib().dpgo_hip_synchronize(self.h))


def tangent_project(X, V, d):
    r = X.shape[0]
    n = X.shape[1] // (d + 1)
    x, xp = _f64(to_dev_layout(X))
    v, vp = _f64(to_dev_layout(V))
    o = np.empty_like(x)
    _check(lib().dpgo_hip_tangent_project(r, d, n, xp, vp, o.ctypes.data_as(_dp)))
    return from_dev_layout(o, r)


def retract_qf(X, V, d, scale=1.0):
    r = X.shape[0]
    n = X.shape[1] // (d + 1)
    x, xp = _f64(to_dev_layout(X))
    v, vp = _f64(to_dev_layout(V))
    o = np.empty_like(x)
    _check(lib().dpgo_hip_retract_qf(r, d, n, xp, vp, scale, o.ctypes.data_as(_dp)))
    return from_dev_layout(o, r)


def project_polar(M, d):
    r = M.shape[0]
    n = M.shape[1] // (d + 1)
    x, xp = _f64(to_dev_layout(M))
    o = np.empty_like(x)
    _check(lib().dpgo_hip_project_polar(r, d, n, xp, o.ctypes.data_as(_dp)))
    return from_dev_layout(o, r)
