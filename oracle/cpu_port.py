"""ctypes driver of oracle/cpu/dpgo_cpu.cpp -- the timed CPU baseline ("kind": "port").

TEST / BASELINE INFRASTRUCTURE: used only by bench.py's cpu_baseline leg and tests/."""
import ctypes as C
import os
import platform

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_V3 = os.path.join(_HERE, "_build", "libdpgo_cpu.so")
LIB_V4 = os.path.join(_HERE, "_build", "libdpgo_cpu_v4.so")
_lib = None


def _host_flags():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                return set(line.split(":", 1)[1].split())
    except OSError:
        pass
    return set()


def _pick_lib():
    """The AVX-512 (x86-64-v4) build when the host has it (the GPU box's Zen 5 EPYC), else x86-64-v3."""
    f = _host_flags()
    if {"avx512f", "avx512bw", "avx512dq", "avx512vl", "avx512cd"} <= f and os.path.exists(LIB_V4):
        return LIB_V4, "x86-64-v4 (AVX-512)"
    return LIB_V3, "x86-64-v3 (AVX2/FMA)"


LIB, ISA = _pick_lib()


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run `make -C oracle`")
        L = C.CDLL(LIB)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int)
        L.dpgo_cpu_time_agent_step.argtypes = [C.c_int, C.c_int, C.c_int, ip, ip, dp, dp, dp, dp, C.c_int, ip,
                                               C.c_int, dp, C.c_int, C.c_int, C.c_int, dp]
        L.dpgo_cpu_time_agent_step.restype = C.c_double
        _lib = L
    return _lib


def time_agent_step(d, r, arrays, n, agent_of_pose, agent, X_dev_layout, accel, num_agents, reps):
    dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int)
    p1 = np.ascontiguousarray(arrays["p1"], np.int32)
    p2 = np.ascontiguousarray(arrays["p2"], np.int32)
    R = np.ascontiguousarray(arrays["R"], np.float64).ravel()
    t = np.ascontiguousarray(arrays["t"], np.float64).ravel()
    k = np.ascontiguousarray(arrays["kappa"], np.float64)
    ta = np.ascontiguousarray(arrays["tau"], np.float64)
    aop = np.ascontiguousarray(agent_of_pose, np.int32)
    X = np.ascontiguousarray(X_dev_layout, np.float64)
    f = C.c_double()
    sec = lib().dpgo_cpu_time_agent_step(d, r, len(p1), p1.ctypes.data_as(ip), p2.ctypes.data_as(ip),
                                         R.ctypes.data_as(dp), t.ctypes.data_as(dp), k.ctypes.data_as(dp),
                                         ta.ctypes.data_as(dp), n, aop.ctypes.data_as(ip), agent,
                                         X.ctypes.data_as(dp), int(accel), num_agents, reps, C.byref(f))
    return sec, f.value


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def baseline(graph, agent_of_pose, X_dev_layout, r, accel, num_agents, sample_updates):
    """Single-thread agent-update throughput on an interior agent (6 neighbours)."""
    arrays = graph.arrays()
    A = round(num_agents ** (1.0 / 3.0))
    mid = A // 2
    agent = mid + A * (mid + A * mid) if A ** 3 == num_agents else 0
    sec, f = time_agent_step(graph.d, r, arrays, graph.n, agent_of_pose, agent, X_dev_layout, accel,
                             num_agents, sample_updates)
    npose = int(np.sum(np.asarray(agent_of_pose) == agent))
    return {"value": 1.0 / sec, "unit": "RBCD agent-updates/s", "cores": 1, "kind": "port",
            "sample": f"{sample_updates} RBCD steps (iterate(true)+iterate(false), Nesterov={bool(accel)}) of "
                      f"interior agent {agent} ({npose} poses) on 1 host thread; a full step over all "
                      f"{num_agents} agents would take {num_agents * sec:.2f} s on this core",
            "seconds_per_agent_update": sec, "cpu_model": _cpu_model(), "nproc": os.cpu_count()}


# ---- multi-agent colour schedule on the host (dpgo_cpu_rbcd_*) -------------------------------
class CpuRbcd:
    """The engine's colour-class RBCD schedule restated on the host (L2, block-Jacobi, Nesterov with
    restart), OpenMP over the agents of a colour class.  TEST / BASELINE INFRASTRUCTURE."""

    def __init__(self, d, r, arrays, n, agent_of_pose, num_agents, accel, restart_interval=30, robust="L2",
                 robust_opt_inner_iters=30, precon="block_jacobi"):
        L = lib()
        dp, ip, vp = C.POINTER(C.c_double), C.POINTER(C.c_int), C.c_void_p
        if not hasattr(L, "_rbcd_bound"):
            L.dpgo_cpu_rbcd_create.argtypes = [C.c_int, C.c_int, C.c_int, ip, ip, dp, dp, dp, dp, C.c_long, ip, C.c_int,
                                               C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
            L.dpgo_cpu_rbcd_create.restype = vp
            L.dpgo_cpu_rbcd_destroy.argtypes = [vp]
            L.dpgo_cpu_rbcd_set_X.argtypes = [vp, dp]
            L.dpgo_cpu_rbcd_get_X.argtypes = [vp, dp]
            L.dpgo_cpu_rbcd_iterate.argtypes = [vp, C.c_int, dp, C.c_int]
            L.dpgo_cpu_rbcd_iterate.restype = C.c_double
            L.dpgo_cpu_rbcd_stats.argtypes = [vp, ip]
            L.dpgo_cpu_rbcd_status.argtypes = [vp, dp, ip]
            L.dpgo_cpu_rbcd_color.argtypes = [vp, C.c_int]
            L.dpgo_cpu_max_threads.restype = C.c_int
            L.dpgo_cpu_rbcd_time_sample.argtypes = [vp, ip, C.c_int, C.c_int, C.c_int, dp, dp]
            L.dpgo_cpu_rbcd_time_sample.restype = C.c_double
            L.dpgo_cpu_rbcd_factor_info.argtypes = [vp, ip, dp]
            L.dpgo_cpu_rbcd_perturb.argtypes = [vp, C.c_double, C.c_ulonglong]
            L._rbcd_bound = True
        self._keep = [np.ascontiguousarray(arrays["p1"], np.int32), np.ascontiguousarray(arrays["p2"], np.int32),
                      np.ascontiguousarray(arrays["R"], np.float64).ravel(),
                      np.ascontiguousarray(arrays["t"], np.float64).ravel(),
                      np.ascontiguousarray(arrays["kappa"], np.float64), np.ascontiguousarray(arrays["tau"], np.float64),
                      np.ascontiguousarray(agent_of_pose, np.int32)]
        p1, p2, R, t, k, ta, aop = self._keep
        self.n, self.r, self.d, self.K = int(n), r, d, int(num_agents)
        self.h = L.dpgo_cpu_rbcd_create(d, r, len(p1), p1.ctypes.data_as(ip), p2.ctypes.data_as(ip),
                                        R.ctypes.data_as(dp), t.ctypes.data_as(dp), k.ctypes.data_as(dp),
                                        ta.ctypes.data_as(dp), int(n), aop.ctypes.data_as(ip), int(num_agents),
                                        int(accel), int(restart_interval), {"L2": 0, "GNC_TLS": 1}[robust],
                                        int(robust_opt_inner_iters), {"block_jacobi": 0, "exact": 1}[precon])
        self.colors = [L.dpgo_cpu_rbcd_color(self.h, a) for a in range(self.K)]

    def close(self):
        if getattr(self, "h", None):
            lib().dpgo_cpu_rbcd_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def set_X(self, X_dev_layout):
        x = np.ascontiguousarray(X_dev_layout, np.float64)
        lib().dpgo_cpu_rbcd_set_X(self.h, x.ctypes.data_as(C.POINTER(C.c_double)))

    def perturb(self, eps, seed):
        """X, Y, V entries times (1 + eps u), u uniform in [-1, 1), Nesterov state kept (a rounding-noise model for
        parity bars: the port with this after every iteration differs from itself as another implementation's
        rounding would)."""
        lib().dpgo_cpu_rbcd_perturb(self.h, float(eps), int(seed))

    def get_X(self):
        x = np.empty(self.n * (self.d + 1) * self.r)
        lib().dpgo_cpu_rbcd_get_X(self.h, x.ctypes.data_as(C.POINTER(C.c_double)))
        return x

    def iterate(self, threads=1, timed_serial=0):
        """One colour iteration; returns (wall seconds, per-agent update seconds (nan = not selected))."""
        sec = np.full(self.K, np.nan)
        w = lib().dpgo_cpu_rbcd_iterate(self.h, int(threads), sec.ctypes.data_as(C.POINTER(C.c_double)),
                                        int(timed_serial))
        return w, sec

    def time_sample(self, agents, threads, reps):
        """Factorise (if needed) then update each listed agent `reps` times, OpenMP over them: (update-phase wall
        seconds, per-agent factor seconds, per-agent seconds per update)."""
        a = np.ascontiguousarray(agents, np.int32)
        fs, us = np.zeros(len(a)), np.zeros(len(a))
        w = lib().dpgo_cpu_rbcd_time_sample(self.h, a.ctypes.data_as(C.POINTER(C.c_int)), len(a), int(threads),
                                            int(reps), fs.ctypes.data_as(C.POINTER(C.c_double)),
                                            us.ctypes.data_as(C.POINTER(C.c_double)))
        return w, fs, us

    def factor_info(self):
        cnt = np.zeros(self.K, np.int32)
        sec = np.zeros(self.K)
        lib().dpgo_cpu_rbcd_factor_info(self.h, cnt.ctypes.data_as(C.POINTER(C.c_int)),
                                        sec.ctypes.data_as(C.POINTER(C.c_double)))
        return cnt, sec

    def stats(self):
        out = np.zeros(self.K * 10, np.int32)
        lib().dpgo_cpu_rbcd_stats(self.h, out.ctypes.data_as(C.POINTER(C.c_int)))
        return out.reshape(self.K, 10)

    def status(self):
        rc = np.zeros(self.K)
        rd = np.zeros(self.K, np.int32)
        lib().dpgo_cpu_rbcd_status(self.h, rc.ctypes.data_as(C.POINTER(C.c_double)), rd.ctypes.data_as(C.POINTER(C.c_int)))
        return rc, rd


def max_threads():
    return int(lib().dpgo_cpu_max_threads())


def host_cores():
    """(threads of the all-cores leg, CPUs this process may run on, OpenMP's default team).  SURVEY 8d(b): OpenMP
    over a colour's agents on all host cores, i.e. min(32 = the agents of a colour, CPUs in the affinity mask);
    the OpenMP team (OMP_NUM_THREADS: on the GPU box the pool's per-GPU host share, 16) is timed as a second leg."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    omp = max_threads()
    return max(1, min(avail, 32)), avail, omp


def engine_baseline(graph, agent_of_pose, X_start, r, accel, num_agents, warmup=3, rounds=20, robust="L2"):
    """The like-for-like host baseline: oracle/cpu runs the engine's colour schedule from the GPU's
    timed-region start X (fresh Nesterov, as after set_X), with the reference's preconditioner
    replaced by block-Jacobi on both sides (CHOLMOD is absent).  Protocol: warm-up 3, then
    the median over 20 rounds.
      single thread: a round = one agent update (iterate(true)) of the first colour, each timed alone;
      all cores:     a round = one colour iteration (every agent, OpenMP over the selected ones).
    Returns (result dict, the CPU's X after its iterations, its per-agent counters, iterations run)."""
    arrays = graph.arrays()
    E = CpuRbcd(graph.d, r, arrays, graph.n, agent_of_pose, num_agents, accel, robust=robust)
    E.set_X(X_start)
    T, avail, omp = host_cores()
    per_colour = min(sum(1 for c in E.colors if c == 0), sum(1 for c in E.colors if c == 1) or 10 ** 9)
    ns = min(warmup + rounds, per_colour)
    _, sec = E.iterate(threads=T, timed_serial=ns)  # iteration 0: ns updates serially, the rest in parallel
    serial = [sec[a] for a in range(num_agents) if E.colors[a] == 0 and not np.isnan(sec[a])][:ns]
    one = float(np.median(serial[warmup:])) if len(serial) > warmup else float("nan")
    def leg(threads):
        walls, sel_counts = [], []
        for it in range(warmup + rounds):
            w, s = E.iterate(threads=threads)
            walls.append(w)
            sel_counts.append(int(np.sum(~np.isnan(s))))
        return float(np.median(walls[warmup:])), float(np.median(sel_counts[warmup:]))
    med, upd = leg(T)
    T_share = max(1, min(omp, avail, 32))
    share = None
    if T_share != T:
        ms_, us_ = leg(T_share)
        share = {"value": us_ / ms_, "threads": T_share, "seconds_per_iteration": ms_,
                 "what": "the OpenMP team (OMP_NUM_THREADS: the GPU box's per-GPU host share)"}
    res = {"value": upd / med, "unit": "RBCD agent-updates/s", "cores": T, "kind": "port",
           "sample": (f"oracle/cpu colour-schedule RBCD ({robust}, Nesterov={bool(accel)}, block-Jacobi on both sides: "
                      f"CHOLMOD absent) from the GPU timed region's start X; {T} OpenMP threads (of {avail} CPUs in "
                      f"the affinity mask, capped at a colour's 32 agents; OMP team {omp} timed as omp_team_leg): median of {rounds} colour iterations ({upd:.0f} agent "
                      f"updates each, OpenMP over them) after {warmup} warm-up; one thread: median of "
                      f"{max(len(serial) - warmup, 0)} single agent updates after {warmup}"),
           "threads": T, "affinity_cpus": avail, "omp_max_threads": omp, "isa": ISA,
           "seconds_per_iteration_all_cores": med,
           "single_thread": {"value": 1.0 / one if one > 0 else None, "seconds_per_agent_update": one,
                             "cores": 1},
           "omp_team_leg": share,
           "cpu_model": _cpu_model(), "nproc": os.cpu_count()}
    iters = 1 + (warmup + rounds) * (2 if share is not None else 1)
    return res, E.get_X(), E.stats(), iters


def exact_sample_baseline(graph, agent_of_pose, X_start, r, accel, num_agents, robust="L2", reps=2, sample=None,
                          updates=None, agent_factorisations=0):
    """CPU baseline of the exact-preconditioner legs (bench.py --precon exact): oracle/cpu's exact mode (reverse
    Cuthill-McKee envelope Cholesky of Q + 0.1 I per agent, no code shared with the GPU library) on a BOUNDED sample of
    the workload: `sample` agents of colour 0 (default: as many as the OpenMP team has threads, at most a colour's),
    OpenMP over them, each factorised once and then updated `reps` times from the GPU timed region's start X.  The
    two measured rates -- agent factorisations / s and agent updates / s -- are combined for the GPU run's own mix:
    `updates` agent updates and `agent_factorisations` agent factorisations (the L2 leg refactorises nothing inside
    the timed steps; GNC_TLS refactorises every agent after each reweighting).  The reference itself refactorises at
    EVERY update under a robust cost (constructQMatrix -> setQ in PGOAgent::updateX, src/PGOAgent.cpp:1110-1112;
    src/QuadraticProblem.cpp:37-41), which this baseline does not charge."""
    import time as _time
    arrays = graph.arrays()
    t0 = _time.time()
    E = CpuRbcd(graph.d, r, arrays, graph.n, agent_of_pose, num_agents, accel, robust=robust, precon="exact")
    E.set_X(X_start)
    setup = _time.time() - t0
    T, avail, omp = host_cores()
    T = max(1, min(omp, avail, T))
    col0 = [a for a in range(num_agents) if E.colors[a] == 0]
    S = min(len(col0), sample or T)
    agents = col0[:S]
    wall_upd, fsec, usec = E.time_sample(agents, T, reps)
    # the factor phase's wall time: S factorisations over min(S, T) threads
    waves = -(-S // T)
    fac_wall = float(np.max(fsec)) * waves
    upd_rate = S * reps / wall_upd
    fac_rate = S / fac_wall
    U = updates if updates is not None else S * reps
    t_model = U / upd_rate + agent_factorisations / fac_rate
    E.close()
    return {"value": U / t_model, "unit": "RBCD agent-updates/s", "cores": T, "kind": "port",
            "sample": (f"oracle/cpu exact mode (RCM envelope Cholesky of Q + 0.1 I, {robust}, Nesterov={bool(accel)}) "
                       f"from the GPU timed region's start X: {S} agents of colour 0 on {T} OpenMP threads, each "
                       f"factorised once and updated {reps} times; combined for the GPU run's {U} agent updates and "
                       f"{agent_factorisations} agent factorisations"),
            "agent_updates_per_s": upd_rate, "seconds_per_update_median": float(np.median(usec)),
            "agent_factorisations_per_s": fac_rate, "seconds_per_factorisation_median": float(np.median(fsec)),
            "setup_s": setup, "threads": T, "affinity_cpus": avail, "omp_max_threads": omp, "isa": ISA,
            "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
            "note": "the reference refactorises at every update under a robust cost (src/PGOAgent.cpp:1110-1112); "
                    "not charged here"}
