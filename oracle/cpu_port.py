"""ctypes driver of oracle/cpu/dpgo_cpu.cpp -- the timed CPU baseline ("kind": "port").

TEST / BASELINE INFRASTRUCTURE: used only by bench.py's cpu_baseline leg and tests/."""
import ctypes as C
import os
import platform

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "libdpgo_cpu.so")
_lib = None


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
