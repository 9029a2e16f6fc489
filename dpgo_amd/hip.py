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
# DPGO_HIP_LIB: another build of the library (tools/ A/B runs against a previous build only)
LIB_PATH = os.environ.get("DPGO_HIP_LIB") or os.path.join(_HERE, "libdpgo_hip.so")

PRECON_EXACT, PRECON_BLOCK_JACOBI, PRECON_NONE = 0, 1, 2
QFMT_BSR, QFMT_EDGES = 0, 1
ROBUST = {"L2": 0, "L1": 1, "TLS": 2, "Huber": 3, "GM": 4, "GNC_TLS": 5}
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
    ("dpgo_hip_set_Q_edges", [C.c_void_p, C.c_int, C.c_int, _ip, _ip, _dp, _dp, _dp, _dp, _dp], C.c_int),
    ("dpgo_hip_set_edge_weights_dev", [C.c_void_p, C.c_void_p], C.c_int),
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
    ("dpgo_hip_set_tuning", [C.c_int, C.c_int], C.c_int),
    ("dpgo_hip_get_tuning", [C.c_int, C.POINTER(C.c_int)], C.c_int),
    ("dpgo_hip_exact_factor_info", [C.c_void_p, C.POINTER(C.c_longlong), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                    C.POINTER(C.c_longlong), C.POINTER(C.c_double), C.POINTER(C.c_int)], C.c_int),
    ("dpgo_hip_exact_factor_flops", [C.c_void_p, _dp, _dp], C.c_int),
    ("dpgo_hip_exact_fallback_agents", [C.c_void_p, _ip, _ip], C.c_int),
    ("dpgo_hip_exact_sweep_bytes", [C.c_void_p, _dp, _dp], C.c_int),
    ("dpgo_hip_bench_precond", [C.c_void_p, C.c_void_p, C.c_int, _dp, _dp, _dp], C.c_int),
    ("dpgo_hip_problem_set_tuning", [C.c_void_p, C.c_int, C.c_int], C.c_int),
    ("dpgo_hip_spmm_bytes", [C.c_void_p], C.c_double),
    ("dpgo_hip_bench_spmm", [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, _dp], C.c_int),
    ("dpgo_hip_spmm_bytes_bsr", [C.c_void_p], C.c_double),
    ("dpgo_hip_certify", [C.c_void_p, _dp, C.c_int, C.c_double, _dp, _dp, _ip, _dp], C.c_int),
    ("dpgo_hip_certify_ex", [C.c_void_p, _dp, C.c_int, C.c_int, C.c_int, C.c_double, _dp, _dp, C.c_void_p],
     C.c_int),
    ("dpgo_hip_bench_hvp", [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, _dp], C.c_int),
    ("dpgo_hip_stats", [C.c_void_p, _ip], C.c_int),
    ("dpgo_hip_set_trace", [C.c_void_p, C.c_int], C.c_int),
    ("dpgo_hip_get_trace", [C.c_void_p, C.c_int, _dp, C.c_int, _ip], C.c_int),
    ("dpgo_hip_build_id", [], C.c_char_p),
]
STATS_INTS = 13
STATS_FIELDS = ["calls", "early", "runs", "tcg_iters", "NEGCURVTURE", "EXCREGION", "LCON", "SCON", "MAXITER",
                "gave_up", "cg_steps", "implicit", "first_full"]
TRACE_WIDTH = 16
TRACE_FIELDS = ["op", "j", "f1", "f2", "rho", "Delta", "alpha", "beta", "tau", "d_Hd", "norm_r", "z_r", "status",
                "accepted", "ngf", "run"]
SPMM_MODES = ["XQ", "XQ_G", "EVAL", "HESS", "F", "EVAL_TCG", "CERT", "QF", "HESS_QF", "HESS_M", "HESS_QF_M"]

EXPORTED_SYMBOLS = [s[0] for s in _SIGS]


def lib():
    """Load libdpgo_hip.so (built in-tree by __graft_entry__.build()).  Raises if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DPGOHipError(f"{LIB_PATH} not built: run __graft_entry__.build() (no CPU fallback)")
        # torch-ROCm bundles its own libamdhip64 (SONAME libamdhip64.so.7, NEEDED as
        # "libamdhip64.so").  Load torch first so our NEEDED libamdhip64.so.7 binds to that same
        # runtime; loading ours first would put two HIP runtimes in one process.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, args, res in _SIGS:
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
        # DPGO_TUNE="key=value,...": process defaults of tuning keys (A/B and profiling runs of tools/ and bench.py)
        for kv in filter(None, os.environ.get("DPGO_TUNE", "").split(",")):
            k, v = kv.split("=")
            _check(L.dpgo_hip_set_tuning(int(k), int(v)))
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


def build_id() -> str:
    """Source hash compiled into the loaded libdpgo_hip.so (__graft_entry__.source_hash())."""
    return lib().dpgo_hip_build_id().decode()


def rccl_unique_id() -> bytes:
    """ncclGetUniqueId through the library's RCCL (128 opaque bytes)."""
    buf = C.create_string_buffer(128)
    _check(lib().dpgo_rccl_unique_id(buf))
    return buf.raw


def get_tuning(key: int) -> int:
    """Process default of a tuning key."""
    v = C.c_int()
    _check(lib().dpgo_hip_get_tuning(int(key), C.byref(v)))
    return v.value


def set_tuning(key: int, value: int):
    """Process default of a tuning key: handles created afterwards copy it (Problem / Rbcd.set_tuning change
    an existing one)."""
    _check(lib().dpgo_hip_set_tuning(int(key), int(value)))


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

    def set_Q_edges(self, agent, p1, p2, R, t, kappa, tau, weight=None):
        """Q of one agent from its measurements (agent-local endpoints, -1 = other agent)."""
        a1, a1p = _i32(p1)
        a2, a2p = _i32(p2)
        Rr, Rp = _f64(np.asarray(R, dtype=np.float64).reshape(-1))
        tt, tp = _f64(np.asarray(t, dtype=np.float64).reshape(-1))
        kk, kp = _f64(kappa)
        ta, tap = _f64(tau)
        if weight is not None:
            ww, wp = _f64(weight)
        else:
            wp = None
        _check(lib().dpgo_hip_set_Q_edges(self.h, agent, len(a1), a1p, a2p, Rp, tp, kp, tap, wp))

    def set_edge_weights_dev(self, w_dev_ptr: int):
        _check(lib().dpgo_hip_set_edge_weights_dev(self.h, C.c_void_p(w_dev_ptr)))

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
    def optimize_dev(self, X_dev: int, X_out_dev: int, params: OptParams | None = None, enabled=None,
                     want_results=True):
        """want_results=False: no statistics (the RBCD engine's call: f(x2) only, direct X_out)."""
        res = (OptResult * self.K)() if want_results else None
        p = params or default_params()
        if enabled is not None:
            en, enp = _i32(enabled)
        else:
            enp = None
        _check(lib().dpgo_hip_optimize_dev(self.h, C.byref(p), C.c_void_p(X_dev), C.c_void_p(X_out_dev),
                                           enp, res))
        return [r.as_dict() for r in res] if want_results else None

    def polar_combine_dev(self, A_dev, B_dev, ca, cb, out_dev):
        a, ap = _f64(ca)
        if B_dev is not None:
            b, bp = _f64(cb)
        else:
            bp = None
        _check(lib().dpgo_hip_polar_combine_dev(self.h, C.c_void_p(A_dev), C.c_void_p(B_dev or 0), ap, bp,
                                                C.c_void_p(out_dev)))

    def certify(self, X, max_iters=300, tol=1e-8, want_vector=False, basis=0, seed_x=False):
        """lambda_min of S(X) = Q - Lambda(X) (Lanczos on the device): (lambda_min, residual, iters, vec).
        basis > 0: thick restart at that basis size; seed_x: the rows of X in the start block
        (dpgo_hip_certify_ex)."""
        x, xp = self._in(X)
        lam, info = C.c_double(), CertInfo()
        v = np.empty(self.vec_len) if want_vector else None
        _check(lib().dpgo_hip_certify_ex(self.h, xp, int(max_iters), int(basis), 1 if seed_x else 0, float(tol),
                                         C.byref(lam), v.ctypes.data_as(_dp) if v is not None else None,
                                         C.byref(info)))
        self.last_certificate = info.as_dict()
        return lam.value, info.residual, info.iters, (from_dev_layout(v, self.r) if v is not None else None)

    def spmm_bytes(self) -> float:
        return float(lib().dpgo_hip_spmm_bytes(self.h))

    def bench_spmm(self, X_dev: int, Y_dev: int, reps: int) -> float:
        ms = C.c_double()
        _check(lib().dpgo_hip_bench_spmm(self.h, C.c_void_p(X_dev), C.c_void_p(Y_dev), reps, C.byref(ms)))
        return ms.value

    def synchronize(self):
        _check(lib().dpgo_hip_synchronize(self.h))

    def stats(self):
        """Cumulative solver counters per agent: list of dicts (STATS_FIELDS)."""
        out = np.zeros(self.K * STATS_INTS, np.int32)
        _check(lib().dpgo_hip_stats(self.h, out.ctypes.data_as(_ip)))
        return [dict(zip(STATS_FIELDS, (int(v) for v in out[a * STATS_INTS:(a + 1) * STATS_INTS])))
                for a in range(self.K)]

    def set_trace(self, capacity):
        _check(lib().dpgo_hip_set_trace(self.h, int(capacity)))
        self._trace_cap = int(capacity)

    def exact_factor_info(self):
        """The exact preconditioner's factor: supernodes, levels, widest separator (64-row tiles), panel doubles,
        last device factorisation ms, device factorisations so far."""
        n, lv, mt, pd, ms, cnt = C.c_longlong(), C.c_int(), C.c_int(), C.c_longlong(), C.c_double(), C.c_int()
        _check(lib().dpgo_hip_exact_factor_info(self.h, C.byref(n), C.byref(lv), C.byref(mt), C.byref(pd), C.byref(ms),
                                                C.byref(cnt)))
        fl, ifl = C.c_double(), C.c_double()
        _check(lib().dpgo_hip_exact_factor_flops(self.h, C.byref(fl), C.byref(ifl)))
        return {"nodes": n.value, "levels": lv.value, "max_s_tiles": mt.value, "panel_doubles": pd.value,
                "factor_ms": ms.value, "factor_count": cnt.value, "cholesky_flops": fl.value,
                "inverse_flops": ifl.value}

    def exact_fallback_agents(self):
        """Per agent 1 where the last exact factorisation met a non-positive pivot (that agent's preconditioner is
        the identity, src/QuadraticProblem.cpp:81-86; the other agents keep their factors)."""
        flags = np.zeros(self.K, np.int32)
        cnt = C.c_int()
        _check(lib().dpgo_hip_exact_fallback_agents(self.h, flags.ctypes.data_as(_ip), C.byref(cnt)))
        assert int(flags.sum()) == cnt.value
        return flags

    def set_tuning(self, key, value):
        """A tuning key on this handle only (dpgo_hip_problem_set_tuning)."""
        _check(lib().dpgo_hip_problem_set_tuning(self.h, int(key), int(value)))

    def get_trace(self, agent=0):
        """Per-iteration records of one agent: list of dicts (TRACE_FIELDS)."""
        cap = getattr(self, "_trace_cap", 0)
        buf = np.zeros(max(cap, 1) * TRACE_WIDTH)
        n = C.c_int()
        _check(lib().dpgo_hip_get_trace(self.h, int(agent), buf.ctypes.data_as(_dp), cap, C.byref(n)))
        k = min(n.value, cap)
        return [dict(zip(TRACE_FIELDS, buf[i * TRACE_WIDTH:(i + 1) * TRACE_WIDTH].tolist())) for i in range(k)]


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


# ----------------------------------------------------------------------------------------
# Pose graphs + multi-agent RBCD engine (include/dpgo_rbcd.h)
# ----------------------------------------------------------------------------------------
class CertInfo(C.Structure):
    """dpgo_cert_info (include/dpgo_hip.h)."""
    _fields_ = [("iters", C.c_int), ("restarts", C.c_int), ("seeds", C.c_int), ("residual", C.c_double),
                ("lambda_seed", C.c_double), ("lambda_complement", C.c_double), ("residual_complement", C.c_double),
                ("coupling", C.c_double), ("lower_bound", C.c_double), ("ritz", C.c_double * 8)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "ritz"}
        d["ritz"] = [float(x) for x in self.ritz]
        return d


class RbcdParams(C.Structure):
    _fields_ = [("r", C.c_int), ("acceleration", C.c_int), ("restart_interval", C.c_int),
                ("max_inner", C.c_int), ("initial_radius", C.c_double), ("tolerance", C.c_double),
                ("precon", C.c_int), ("algorithm", C.c_int), ("q_format", C.c_int),
                ("robust_cost", C.c_int), ("robust_opt_inner_iters", C.c_int), ("gnc_max_iters", C.c_int),
                ("gnc_barc", C.c_double), ("gnc_mu_step", C.c_double), ("gnc_init_mu", C.c_double),
                ("huber_threshold", C.c_double), ("tls_threshold", C.c_double),
                ("status", C.c_int), ("rel_change_tol", C.c_double), ("min_convergence_ratio", C.c_double)]


_lp = C.POINTER(C.c_longlong)
_SIGS2 = [
    ("dpgo_graph_read_g2o", [C.c_char_p, C.POINTER(C.c_void_p)], C.c_int),
    ("dpgo_graph_grid3d", [C.c_int, C.c_ulonglong, C.c_double, C.c_double, C.POINTER(C.c_void_p)], C.c_int),
    ("dpgo_graph_from_arrays", [C.c_int, C.c_int, C.c_int, _ip, _ip, _dp, _dp, _dp, _dp,
                                C.POINTER(C.c_void_p)], C.c_int),
    ("dpgo_graph_info", [C.c_void_p, _ip, _ip, _ip, _ip], C.c_int),
    ("dpgo_graph_copy_out", [C.c_void_p, _ip, _ip, _dp, _dp, _dp, _dp], C.c_int),
    ("dpgo_graph_destroy", [C.c_void_p], C.c_int),
    ("dpgo_graph_laplacian_bsr", [C.c_void_p, _lp, _ip, _ip, _dp], C.c_int),
    ("dpgo_graph_chain_init", [C.c_void_p, C.c_int, _dp, _dp], C.c_int),
    ("dpgo_graph_chordal_init", [C.c_void_p, C.c_int, _dp, _dp], C.c_int),
    ("dpgo_chordal_initialization", [C.c_int, C.c_int, C.c_int, _ip, _ip, _dp, _dp, _dp, _dp, _dp], C.c_int),
    ("dpgo_graph_grid_partition", [C.c_void_p, C.c_int, _ip], C.c_int),
    ("dpgo_graph_certify", [C.c_void_p, C.c_int, _dp, C.c_int, C.c_double, _dp, _dp, _ip, _dp, _dp, _dp, _dp],
     C.c_int),
    ("dpgo_graph_certify_ex", [C.c_void_p, C.c_int, _dp, C.c_int, C.c_int, C.c_int, C.c_double, _dp, _dp, _dp, _dp,
                               _dp, C.c_void_p], C.c_int),
    ("dpgo_chordal_initialization_gpu", [C.c_int, C.c_int, C.c_int, _ip, _ip, _dp, _dp, _dp, _dp, C.c_double,
                                         C.c_int, _dp, _ip, _dp], C.c_int),
    ("dpgo_graph_chordal_init_gpu", [C.c_void_p, C.c_int, _dp, C.c_double, C.c_int, _dp, _ip, _dp], C.c_int),
    ("dpgo_graph_distributed_init", [C.c_void_p, C.c_int, _ip, C.c_int, _dp, C.c_int, C.c_double, C.c_int, _dp, _ip,
                                     _dp], C.c_int),
    ("dpgo_rbcd_default_params", [C.POINTER(RbcdParams)], None),
    ("dpgo_rbcd_plan", [C.c_void_p, C.c_int, _ip, _ip, C.c_int, C.c_int, _lp, _lp, _ip, _ip], C.c_int),
    ("dpgo_rbcd_create", [C.c_void_p, C.c_int, _ip, _ip, C.c_int, C.c_int, C.POINTER(RbcdParams),
                          C.POINTER(C.c_void_p)], C.c_int),
    ("dpgo_rbcd_destroy", [C.c_void_p], C.c_int),
    ("dpgo_rbcd_set_stream", [C.c_void_p, C.c_void_p], C.c_int),
    ("dpgo_rbcd_info", [C.c_void_p, _ip, _ip, _ip, _ip], C.c_int),
    ("dpgo_rbcd_color_of_agent", [C.c_void_p, _ip], C.c_int),
    ("dpgo_rbcd_exchange_counts", [C.c_void_p, _lp, _lp], C.c_int),
    ("dpgo_rbcd_set_X", [C.c_void_p, _dp], C.c_int),
    ("dpgo_rbcd_get_X", [C.c_void_p, _dp], C.c_int),
    ("dpgo_rbcd_pre_exchange", [C.c_void_p, C.c_int], C.c_int),
    ("dpgo_rbcd_pack", [C.c_void_p, C.c_void_p], C.c_int),
    ("dpgo_rbcd_update", [C.c_void_p, C.c_int, C.c_void_p, C.POINTER(OptResult)], C.c_int),
    ("dpgo_rbcd_set_selected", [C.c_void_p, _ip], C.c_int),
    ("dpgo_rbcd_bench_spmm", [C.c_void_p, C.c_int, C.c_int, _dp, _dp], C.c_int),
    ("dpgo_rbcd_counters", [C.c_void_p, _lp, _lp], C.c_int),
    ("dpgo_rbcd_spmm_bytes", [C.c_void_p, C.c_int, _dp, _dp], C.c_int),
    ("dpgo_rbcd_bench_hvp", [C.c_void_p, C.c_int, C.c_int, _dp], C.c_int),
    ("dpgo_rbcd_reset_stream", [C.c_void_p], C.c_int),
    ("dpgo_rbcd_central_eval", [C.c_void_p, C.c_void_p, _dp, _dp], C.c_int),
    ("dpgo_rbcd_status", [C.c_void_p, _dp, _ip], C.c_int),
    ("dpgo_rbcd_stats", [C.c_void_p, _ip], C.c_int),
    ("dpgo_rbcd_bytes", [C.c_void_p, _dp, _dp], C.c_int),
    ("dpgo_rbcd_mode_bytes", [C.c_void_p, C.c_int, _dp], C.c_int),
    ("dpgo_rccl_unique_id", [C.c_void_p], C.c_int),
    ("dpgo_rbcd_comm_init", [C.c_void_p, C.c_void_p], C.c_int),
    ("dpgo_rbcd_comm_attach", [C.c_void_p, C.c_void_p], C.c_int),
    ("dpgo_rbcd_comm_info", [C.c_void_p, _ip, _ip], C.c_int),
    ("dpgo_rbcd_exact_factor_info", [C.c_void_p, C.c_int, C.POINTER(C.c_longlong), C.POINTER(C.c_int),
                                     C.POINTER(C.c_int), C.POINTER(C.c_longlong), C.POINTER(C.c_double),
                                     C.POINTER(C.c_int)], C.c_int),
    ("dpgo_rbcd_exact_factor_flops", [C.c_void_p, C.c_int, _dp, _dp], C.c_int),
    ("dpgo_rbcd_bench_precond", [C.c_void_p, C.c_int, C.c_int, _dp, _dp, _dp], C.c_int),
    ("dpgo_rbcd_exact_sweep_bytes", [C.c_void_p, C.c_int, _dp, _dp], C.c_int),
    ("dpgo_rbcd_exchange", [C.c_void_p, C.POINTER(C.c_void_p)], C.c_int),
    ("dpgo_rbcd_set_kernel_timing", [C.c_void_p, C.c_int], C.c_int),
    ("dpgo_rbcd_set_tuning", [C.c_void_p, C.c_int, C.c_int], C.c_int),
    ("dpgo_rbcd_set_trace", [C.c_void_p, C.c_int], C.c_int),
    ("dpgo_rbcd_get_trace", [C.c_void_p, C.c_int, _dp, C.c_int, _ip], C.c_int),
    ("dpgo_rbcd_kernel_times", [C.c_void_p, _dp, _lp], C.c_int),
    ("dpgo_rbcd_kernel_times_ex", [C.c_void_p, _dp, _lp, _dp], C.c_int),
    ("dpgo_rbcd_plan_color", [C.c_void_p, C.c_int, _ip, _ip, C.c_int, C.c_int, C.c_int, _lp, _lp, _ip, _ip], C.c_int),
    ("dpgo_rbcd_exchange_counts_color", [C.c_void_p, C.c_int, _lp, _lp], C.c_int),
    ("dpgo_rbcd_pack_color", [C.c_void_p, C.c_int, C.c_void_p], C.c_int),
    ("dpgo_rbcd_update_color", [C.c_void_p, C.c_int, C.c_void_p, C.POINTER(OptResult)], C.c_int),
    ("dpgo_rbcd_exchange_color", [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
]
_SIGS.extend(_SIGS2)
EXPORTED_SYMBOLS.extend(s[0] for s in _SIGS2)


class Graph:
    """Pose graph held by the native library (g2o reader / synthetic grid / arrays)."""

    def __init__(self, handle):
        self.h = handle
        d, n, m, dup = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _check(lib().dpgo_graph_info(self.h, C.byref(d), C.byref(n), C.byref(m), C.byref(dup)))
        self.d, self.n, self.m, self.duplicates = d.value, n.value, m.value, dup.value

    @classmethod
    def read_g2o(cls, path):
        h = C.c_void_p()
        _check(lib().dpgo_graph_read_g2o(path.encode(), C.byref(h)))
        return cls(h)

    @classmethod
    def grid3d(cls, k, seed=0, rot_sigma=0.2, trans_sigma=0.1):
        h = C.c_void_p()
        _check(lib().dpgo_graph_grid3d(int(k), int(seed), rot_sigma, trans_sigma, C.byref(h)))
        return cls(h)

    @classmethod
    def from_arrays(cls, d, n, p1, p2, R, t, kappa, tau):
        a1, a1p = _i32(p1)
        a2, a2p = _i32(p2)
        Rr, Rp = _f64(np.asarray(R).reshape(-1))
        tt, tp = _f64(np.asarray(t).reshape(-1))
        kk, kp = _f64(kappa)
        ta, tap = _f64(tau)
        h = C.c_void_p()
        _check(lib().dpgo_graph_from_arrays(d, int(n), len(a1), a1p, a2p, Rp, tp, kp, tap, C.byref(h)))
        return cls(h)

    def close(self):
        if getattr(self, "h", None):
            lib().dpgo_graph_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def arrays(self):
        d, m = self.d, self.m
        p1 = np.empty(m, np.int32); p2 = np.empty(m, np.int32)
        R = np.empty(m * d * d); t = np.empty(m * d); k = np.empty(m); ta = np.empty(m)
        _check(lib().dpgo_graph_copy_out(self.h, p1.ctypes.data_as(_ip), p2.ctypes.data_as(_ip),
                                         R.ctypes.data_as(_dp), t.ctypes.data_as(_dp),
                                         k.ctypes.data_as(_dp), ta.ctypes.data_as(_dp)))
        return dict(p1=p1, p2=p2, R=R.reshape(m, d, d), t=t.reshape(m, d), kappa=k, tau=ta)

    def laplacian_bsr(self):
        """Whole-graph Q: (browptr, bcol, blocks[nnzb, b, b] column-major)."""
        nnz = C.c_longlong()
        _check(lib().dpgo_graph_laplacian_bsr(self.h, C.byref(nnz), None, None, None))
        b = self.d + 1
        rp = np.empty(self.n + 1, np.int32); col = np.empty(nnz.value, np.int32)
        blk = np.empty(nnz.value * b * b)
        _check(lib().dpgo_graph_laplacian_bsr(self.h, C.byref(nnz), rp.ctypes.data_as(_ip),
                                              col.ctypes.data_as(_ip), blk.ctypes.data_as(_dp)))
        return rp, col, blk

    def chain_init(self, r, YLift):
        """YLift (r x d) times the odometry-chain initialisation; returns r x (d+1) n."""
        Y, Yp = _f64(np.asarray(YLift, dtype=np.float64).T.ravel())  # column-major
        out = np.empty(self.n * (self.d + 1) * r)
        _check(lib().dpgo_graph_chain_init(self.h, r, Yp, out.ctypes.data_as(_dp)))
        return from_dev_layout(out, r)

    def chordal_init(self, r, YLift):
        """YLift (r x d) times chordalInitialization (host); returns r x (d+1) n."""
        Y, Yp = _f64(np.asarray(YLift, dtype=np.float64).T.ravel())
        out = np.empty(self.n * (self.d + 1) * r)
        _check(lib().dpgo_graph_chordal_init(self.h, r, Yp, out.ctypes.data_as(_dp)))
        return from_dev_layout(out, r)

    def chordal_init_gpu(self, r, YLift, rtol=1e-12, max_iters=20000, dev_layout=False):
        """chordalInitialization by Jacobi-PCG on the GPU; returns (X, PCG iterations, relative residual)."""
        Y, Yp = _f64(np.asarray(YLift, dtype=np.float64).T.ravel())
        out = np.empty(self.n * (self.d + 1) * r)
        it, rr = C.c_int(), C.c_double()
        _check(lib().dpgo_graph_chordal_init_gpu(self.h, r, Yp, float(rtol), int(max_iters), out.ctypes.data_as(_dp),
                                                 C.byref(it), C.byref(rr)))
        return (out if dev_layout else from_dev_layout(out, r)), it.value, rr.value

    def distributed_init(self, agent_of_pose, r, YLift, gpu=True, rtol=1e-12, max_iters=20000, dev_layout=False):
        """Per-agent chordal (localInitialization) + breadth-first frame alignment (initializeInGlobalFrame);
        returns (X, PCG iterations, relative residual)."""
        aop, ap = _i32(agent_of_pose)
        Y, Yp = _f64(np.asarray(YLift, dtype=np.float64).T.ravel())
        out = np.empty(self.n * (self.d + 1) * r)
        it, rr = C.c_int(), C.c_double()
        _check(lib().dpgo_graph_distributed_init(self.h, int(aop.max()) + 1, ap, r, Yp, int(bool(gpu)), float(rtol),
                                                 int(max_iters), out.ctypes.data_as(_dp), C.byref(it), C.byref(rr)))
        return (out if dev_layout else from_dev_layout(out, r)), it.value, rr.value

    def chain_init_dev_layout(self, r, YLift):
        Y, Yp = _f64(np.asarray(YLift, dtype=np.float64).T.ravel())
        out = np.empty(self.n * (self.d + 1) * r)
        _check(lib().dpgo_graph_chain_init(self.h, r, Yp, out.ctypes.data_as(_dp)))
        return out

    def certify(self, X, r, max_iters=300, tol=1e-8, want_rounded=False, want_vector=False, basis=0, seed_x=False):
        """Certified optimality gap of X (flat r x (d+1) n column-major buffer, or the r x (d+1) n
        matrix) for the whole graph: dict(lambda_min, residual, iters, f_relax, f_rounded, gap, rel_gap
        [, T_rounded d x (d+1) n])."""
        X = np.asarray(X, dtype=np.float64)
        flat = np.ascontiguousarray(X.T).ravel() if X.ndim == 2 else np.ascontiguousarray(X).ravel()
        if flat.size != r * (self.d + 1) * self.n:
            raise DPGOHipError("X has the wrong size")
        lam, fx, fr, info = C.c_double(), C.c_double(), C.c_double(), CertInfo()
        T = np.empty(self.d * (self.d + 1) * self.n) if want_rounded else None
        V = np.empty(flat.size) if want_vector else None
        _check(lib().dpgo_graph_certify_ex(self.h, int(r), flat.ctypes.data_as(_dp), int(max_iters), int(basis),
                                           1 if seed_x else 0, float(tol), C.byref(lam), C.byref(fx), C.byref(fr),
                                           T.ctypes.data_as(_dp) if T is not None else None,
                                           V.ctypes.data_as(_dp) if V is not None else None, C.byref(info)))
        out = dict(lambda_min=lam.value, f_relax=fx.value, f_rounded=fr.value, gap=fr.value - fx.value,
                   rel_gap=(fr.value - fx.value) / fx.value if fx.value else float("nan"))
        out.update(info.as_dict())
        if T is not None:
            out["T_rounded"] = from_dev_layout(T, self.d)
        if V is not None:
            out["eigvec"] = V.reshape(-1, r).T if V.ndim == 1 else V  # r x (d+1) n
        return out

    def grid_partition(self, agents_per_axis):
        out = np.empty(self.n, np.int32)
        _check(lib().dpgo_graph_grid_partition(self.h, int(agents_per_axis), out.ctypes.data_as(_ip)))
        return out


def chordal_initialization(d, n, p1, p2, R, t, kappa, tau):
    """chordalInitialization (src/DPGO_utils.cpp:377-424), host: T (d x (d+1) n)."""
    a1, a1p = _i32(p1)
    a2, a2p = _i32(p2)
    Rr, Rp = _f64(np.asarray(R).reshape(-1))
    tt, tp = _f64(np.asarray(t).reshape(-1))
    kk, kp = _f64(kappa)
    ta, tap = _f64(tau)
    out = np.empty(d * (d + 1) * n)
    _check(lib().dpgo_chordal_initialization(d, int(n), len(a1), a1p, a2p, Rp, tp, kp, tap, out.ctypes.data_as(_dp)))
    return from_dev_layout(out, d)


def chordal_initialization_gpu(d, n, p1, p2, R, t, kappa, tau, rtol=1e-12, max_iters=20000):
    """chordalInitialization with both solves by Jacobi-PCG on the GPU: (T, iterations, rel. residual)."""
    a1, a1p = _i32(p1)
    a2, a2p = _i32(p2)
    Rr, Rp = _f64(np.asarray(R).reshape(-1))
    tt, tp = _f64(np.asarray(t).reshape(-1))
    kk, kp = _f64(kappa)
    ta, tap = _f64(tau)
    out = np.empty(d * (d + 1) * n)
    it, rr = C.c_int(), C.c_double()
    _check(lib().dpgo_chordal_initialization_gpu(d, int(n), len(a1), a1p, a2p, Rp, tp, kp, tap, float(rtol),
                                                 int(max_iters), out.ctypes.data_as(_dp), C.byref(it), C.byref(rr)))
    return from_dev_layout(out, d), it.value, rr.value


def exchange_plan(graph: "Graph", agent_of_pose, agent_rank, rank, world):
    """Host-only exchange plan (no GPU): ([send pose ids per peer], [recv pose ids per peer])."""
    aop, ap = _i32(agent_of_pose)
    ar, arp = _i32(agent_rank)
    sc = np.empty(world, np.int64); rc = np.empty(world, np.int64)
    _check(lib().dpgo_rbcd_plan(graph.h, len(ar), ap, arp, rank, world, sc.ctypes.data_as(_lp),
                                rc.ctypes.data_as(_lp), None, None))
    sp_ = np.empty(max(int(sc.sum()), 1), np.int32); rp_ = np.empty(max(int(rc.sum()), 1), np.int32)
    _check(lib().dpgo_rbcd_plan(graph.h, len(ar), ap, arp, rank, world, None, None,
                                sp_.ctypes.data_as(_ip), rp_.ctypes.data_as(_ip)))
    so = np.concatenate([[0], np.cumsum(sc)]); ro = np.concatenate([[0], np.cumsum(rc)])
    return ([sp_[so[p]:so[p + 1]] for p in range(world)], [rp_[ro[p]:ro[p + 1]] for p in range(world)])


def exchange_plan_color(graph: "Graph", agent_of_pose, agent_rank, color, rank, world):
    """Host-only per-colour halo plan (the poses colour `color`'s agents read): ([send ids per peer],
    [recv ids per peer])."""
    aop, ap = _i32(agent_of_pose)
    ar, arp = _i32(agent_rank)
    sc = np.empty(world, np.int64); rc = np.empty(world, np.int64)
    _check(lib().dpgo_rbcd_plan_color(graph.h, len(ar), ap, arp, int(color), rank, world, sc.ctypes.data_as(_lp),
                                      rc.ctypes.data_as(_lp), None, None))
    sp_ = np.empty(max(int(sc.sum()), 1), np.int32); rp_ = np.empty(max(int(rc.sum()), 1), np.int32)
    _check(lib().dpgo_rbcd_plan_color(graph.h, len(ar), ap, arp, int(color), rank, world, None, None,
                                      sp_.ctypes.data_as(_ip), rp_.ctypes.data_as(_ip)))
    so = np.concatenate([[0], np.cumsum(sc)]); ro = np.concatenate([[0], np.cumsum(rc)])
    return ([sp_[so[p]:so[p + 1]] for p in range(world)], [rp_[ro[p]:ro[p + 1]] for p in range(world)])


def lifting_matrix(d, r, seed=2):
    """Repo-defined lifting matrix YLift in St(d, r) (replaces ROPTLIB's RNG)."""
    M = np.random.default_rng(seed).standard_normal((r, d))
    Qm, Rm = np.linalg.qr(M)
    s = np.sign(np.diag(Rm))
    s[s == 0] = 1
    return Qm * s


def rbcd_params(**kw) -> RbcdParams:
    p = RbcdParams()
    lib().dpgo_rbcd_default_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class Rbcd:
    """Colour-class RBCD over N agents; this process owns the agents with agent_rank == rank."""

    def __init__(self, graph: Graph, agent_of_pose, agent_rank, rank=0, world=1, params=None):
        self.graph = graph
        aop, ap = _i32(agent_of_pose)
        ar, arp = _i32(agent_rank)
        self.num_agents = len(ar)
        self.params = params or rbcd_params()
        h = C.c_void_p()
        _check(lib().dpgo_rbcd_create(graph.h, self.num_agents, ap, arp, rank, world,
                                      C.byref(self.params), C.byref(h)))
        self.h = h
        self.rank, self.world = rank, world
        nc, na, npz = C.c_int(), C.c_int(), C.c_int()
        _check(lib().dpgo_rbcd_info(self.h, C.byref(nc), C.byref(na), C.byref(npz), None))
        self.num_colors, self.owned_agents, self.owned_poses = nc.value, na.value, npz.value
        per = np.empty(self.num_colors, np.int32)
        _check(lib().dpgo_rbcd_info(self.h, None, None, None, per.ctypes.data_as(_ip)))
        self.agents_per_color = per
        col = np.empty(self.num_agents, np.int32)
        _check(lib().dpgo_rbcd_color_of_agent(self.h, col.ctypes.data_as(_ip)))
        self.color_of_agent = col
        sc = np.empty(world, np.int64); rc = np.empty(world, np.int64)
        _check(lib().dpgo_rbcd_exchange_counts(self.h, sc.ctypes.data_as(_lp), rc.ctypes.data_as(_lp)))
        self.send_counts, self.recv_counts = sc, rc
        # per-colour halos (doubles per peer)
        self.send_counts_color, self.recv_counts_color = [], []
        for c in range(self.num_colors):
            sc = np.empty(world, np.int64); rc = np.empty(world, np.int64)
            _check(lib().dpgo_rbcd_exchange_counts_color(self.h, c, sc.ctypes.data_as(_lp), rc.ctypes.data_as(_lp)))
            self.send_counts_color.append(sc)
            self.recv_counts_color.append(rc)

    def close(self):
        if getattr(self, "h", None):
            lib().dpgo_rbcd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr):
        _check(lib().dpgo_rbcd_set_stream(self.h, C.c_void_p(stream_ptr)))

    def set_X(self, X):
        x, xp = _f64(to_dev_layout(X) if X.ndim == 2 else X)
        _check(lib().dpgo_rbcd_set_X(self.h, xp))

    def get_X_into(self, Xflat):
        """Write owned poses into a global flat (device-layout) host array."""
        assert Xflat.dtype == np.float64 and Xflat.flags.c_contiguous
        need = self.graph.n * (self.graph.d + 1) * self.params.r
        if Xflat.size < need:
            raise ValueError(f"X buffer holds {Xflat.size} doubles, the graph needs {need}")
        _check(lib().dpgo_rbcd_get_X(self.h, Xflat.ctypes.data_as(_dp)))

    def reset_stream(self):
        _check(lib().dpgo_rbcd_reset_stream(self.h))

    def central_eval(self, recv_ptr=None):
        """(this rank's central cost share, |RieGrad|^2 per agent [num_agents]) at the current X."""
        f = C.c_double()
        g = np.zeros(self.num_agents)
        _check(lib().dpgo_rbcd_central_eval(self.h, C.c_void_p(recv_ptr or 0), C.byref(f), g.ctypes.data_as(_dp)))
        return f.value, g

    def status(self):
        """(relativeChange[num_agents], readyToTerminate[num_agents]); NaN / -1 for other ranks' agents."""
        rc = np.full(self.num_agents, np.nan)
        rd = np.full(self.num_agents, -1, np.int32)
        _check(lib().dpgo_rbcd_status(self.h, rc.ctypes.data_as(_dp), rd.ctypes.data_as(_ip)))
        return rc, rd

    def ready_votes(self):
        """This rank's share of PGOAgent::shouldTerminate (src/PGOAgent.cpp:1007-1031): (owned agents
        ready to terminate, owned agents).  Every agent of the team is ready iff the sums over ranks are
        equal (the caller all-reduces them); the maxNumIters cap is the caller's loop bound."""
        _, rd = self.status()
        mine = rd >= 0
        return int(np.sum(rd[mine] == 1)), int(np.sum(mine))

    def stats(self):
        """Cumulative solver counters per agent: int array [num_agents, STATS_INTS] (zeros elsewhere)."""
        out = np.zeros(self.num_agents * STATS_INTS, np.int32)
        _check(lib().dpgo_rbcd_stats(self.h, out.ctypes.data_as(_ip)))
        return out.reshape(self.num_agents, STATS_INTS)

    def bytes(self):
        """(cumulative algorithmic bytes of all launches, EVAL_TCG bytes per colour pass [num_colors])."""
        b = C.c_double()
        per = np.zeros(self.num_colors)
        _check(lib().dpgo_rbcd_bytes(self.h, C.byref(b), per.ctypes.data_as(_dp)))
        return b.value, per

    def comm_init(self, uid: bytes):
        """Create the engine's RCCL communicator (collective over the engine's ranks); uid from
        rccl_unique_id() on one rank, shared by the caller."""
        buf = C.create_string_buffer(bytes(uid), 128)
        _check(lib().dpgo_rbcd_comm_init(self.h, buf))

    def exact_factor_info(self, color):
        """Problem.exact_factor_info of the colour's batched problem."""
        n, lv, mt, pd, ms, cnt = C.c_longlong(), C.c_int(), C.c_int(), C.c_longlong(), C.c_double(), C.c_int()
        _check(lib().dpgo_rbcd_exact_factor_info(self.h, int(color), C.byref(n), C.byref(lv), C.byref(mt), C.byref(pd),
                                                 C.byref(ms), C.byref(cnt)))
        fl, ifl = C.c_double(), C.c_double()
        _check(lib().dpgo_rbcd_exact_factor_flops(self.h, int(color), C.byref(fl), C.byref(ifl)))
        out = {"nodes": n.value, "levels": lv.value, "max_s_tiles": mt.value, "panel_doubles": pd.value,
               "factor_ms": ms.value, "factor_count": cnt.value, "cholesky_flops": fl.value, "inverse_flops": ifl.value}
        if ms.value > 0:
            out["factor_tflops"] = fl.value / (ms.value * 1e-3) / 1e12
            out["factor_tflops_with_inverse"] = (fl.value + ifl.value) / (ms.value * 1e-3) / 1e12
        return out

    def bench_precond(self, color, reps):
        """The exact preconditioner's forward / backward sweeps over colour class c: (ms_fwd, ms_bwd, stored panel
        bytes)."""
        f, b, p = C.c_double(), C.c_double(), C.c_double()
        _check(lib().dpgo_rbcd_bench_precond(self.h, int(color), int(reps), C.byref(f), C.byref(b), C.byref(p)))
        return f.value, b.value, p.value

    def exact_sweep_bytes(self, color):
        """(forward, backward) panel bytes one application over colour class c reads (wide nodes' tiles, narrow nodes'
        compact copies)."""
        f, b = C.c_double(), C.c_double()
        _check(lib().dpgo_rbcd_exact_sweep_bytes(self.h, int(color), C.byref(f), C.byref(b)))
        return f.value, b.value

    def comm_info(self):
        """(ncclCommCount, ncclCommUserRank) of the engine's own RCCL communicator, (-1, -1) without one."""
        n, r = C.c_int(), C.c_int()
        _check(lib().dpgo_rbcd_comm_info(self.h, C.byref(n), C.byref(r)))
        return n.value, r.value

    def exchange_color(self, color):
        """Per-colour halo by the engine's RCCL group (after pre_exchange(color)); pass the result to
        update_color()."""
        p = C.c_void_p()
        _check(lib().dpgo_rbcd_exchange_color(self.h, int(color), C.byref(p)))
        return p.value

    def pack_color(self, color, send_ptr):
        _check(lib().dpgo_rbcd_pack_color(self.h, int(color), C.c_void_p(send_ptr or 0)))

    def update_color(self, color, recv_ptr, want_results=False):
        if want_results:
            n = int(self.agents_per_color[color])
            res = (OptResult * max(n, 1))()
            _check(lib().dpgo_rbcd_update_color(self.h, int(color), C.c_void_p(recv_ptr or 0), res))
            return [res[i].as_dict() for i in range(n)]
        _check(lib().dpgo_rbcd_update_color(self.h, int(color), C.c_void_p(recv_ptr or 0), None))
        return None

    def exchange(self):
        """Pack + RCCL send/recv of the public poses (after pre_exchange); returns the device pointer of
        the engine-owned receive buffer for update()."""
        p = C.c_void_p()
        _check(lib().dpgo_rbcd_exchange(self.h, C.byref(p)))
        return p.value

    def mode_bytes(self, color):
        """{SpMM mode: algorithmic bytes of one launch over every agent of the colour}."""
        out = np.zeros(len(SPMM_MODES))
        _check(lib().dpgo_rbcd_mode_bytes(self.h, int(color), out.ctypes.data_as(_dp)))
        return {SPMM_MODES[m]: float(out[m]) for m in range(len(SPMM_MODES)) if out[m] > 0}

    def set_trace(self, capacity):
        _check(lib().dpgo_rbcd_set_trace(self.h, int(capacity)))
        self._trace_cap = int(capacity)

    def get_trace(self, agent):
        """Per-iteration records of one owned agent's updates: list of dicts (TRACE_FIELDS)."""
        cap = getattr(self, "_trace_cap", 0)
        buf = np.zeros(max(cap, 1) * TRACE_WIDTH)
        n = C.c_int()
        _check(lib().dpgo_rbcd_get_trace(self.h, int(agent), buf.ctypes.data_as(_dp), cap, C.byref(n)))
        return [dict(zip(TRACE_FIELDS, buf[i * TRACE_WIDTH:(i + 1) * TRACE_WIDTH].tolist()))
                for i in range(min(n.value, cap))]

    def set_kernel_timing(self, on):
        _check(lib().dpgo_rbcd_set_kernel_timing(self.h, int(on)))  # 0 off, k: every k-th launch per mode

    def set_tuning(self, key, value):
        """A tuning key on this engine's colour problems (A/B timing without rebuilding the engine)."""
        _check(lib().dpgo_rbcd_set_tuning(self.h, int(key), int(value)))

    def kernel_times(self, batch_equiv=False):
        """{mode: (ms summed, launches)} of the timed in-step X.Q launches since the last call; with batch_equiv,
        (ms, launches, full-batch launch equivalents) -- the divisor of mode_bytes for a per-launch rate."""
        ms = np.zeros(len(SPMM_MODES))
        n = np.zeros(len(SPMM_MODES), np.int64)
        fr = np.zeros(len(SPMM_MODES))
        _check(lib().dpgo_rbcd_kernel_times_ex(self.h, ms.ctypes.data_as(_dp), n.ctypes.data_as(_lp),
                                               fr.ctypes.data_as(_dp)))
        if batch_equiv:
            return {SPMM_MODES[m]: (float(ms[m]), int(n[m]), float(fr[m])) for m in range(len(SPMM_MODES)) if n[m] > 0}
        return {SPMM_MODES[m]: (float(ms[m]), int(n[m])) for m in range(len(SPMM_MODES)) if n[m] > 0}

    def pre_exchange(self, color):
        _check(lib().dpgo_rbcd_pre_exchange(self.h, int(color)))

    def pack(self, send_ptr):
        _check(lib().dpgo_rbcd_pack(self.h, C.c_void_p(send_ptr or 0)))

    def set_selected(self, agent_mask=None):
        """Optimise only these agents of the updated colour (None: all; the greedy schedule selects one)."""
        if agent_mask is None:
            _check(lib().dpgo_rbcd_set_selected(self.h, None))
            return
        m, mp = _i32(np.asarray(agent_mask) != 0)
        if m.size != self.num_agents:
            raise ValueError("agent_mask needs one entry per agent")
        _check(lib().dpgo_rbcd_set_selected(self.h, mp))

    def update(self, color, recv_ptr, want_results=False):
        if want_results:
            n = int(self.agents_per_color[color])
            res = (OptResult * max(n, 1))()
            _check(lib().dpgo_rbcd_update(self.h, int(color), C.c_void_p(recv_ptr or 0), res))
            return [res[i].as_dict() for i in range(n)]
        _check(lib().dpgo_rbcd_update(self.h, int(color), C.c_void_p(recv_ptr or 0), None))
        return None

    def bench_spmm(self, color, reps):
        b, ms = C.c_double(), C.c_double()
        _check(lib().dpgo_rbcd_bench_spmm(self.h, int(color), int(reps), C.byref(b), C.byref(ms)))
        return b.value, ms.value

    def spmm_bytes(self, color):
        """(SURVEY 8d B_spmm for explicit blocks, bytes of the stored form) of one X.Q SpMM."""
        bb, fb = C.c_double(), C.c_double()
        _check(lib().dpgo_rbcd_spmm_bytes(self.h, int(color), C.byref(bb), C.byref(fb)))
        return bb.value, fb.value

    def bench_hvp(self, color, reps):
        ms = C.c_double()
        _check(lib().dpgo_rbcd_bench_hvp(self.h, int(color), int(reps), C.byref(ms)))
        return ms.value

    def counters(self):
        a, i = C.c_longlong(), C.c_longlong()
        _check(lib().dpgo_rbcd_counters(self.h, C.byref(a), C.byref(i)))
        return a.value, i.value
