#!/usr/bin/env python3
"""How far the device RTR trace is from an extended-precision (64-bit mantissa) Run of the same problem, per tCG
sequence: the float64 oracle, the classic five-launch sequence, the merged one over BSR Q (round-3 partials),
and over the edge-stream Q with the round-3 partials (v1) and with the round-4 kernels (v2, whose per-quantity
precision the loaded library was built with).
Same problems and measure as tests/test_gpu_status_trace.py::test_rtr_trace_extended_precision; one JSON line
per problem.  Run it once per variant library (tools/build_variant.py, DPGO_HIP_LIB) to choose the partials'
precision.

  DPGO_HIP_LIB=dpgo_amd/ab/dd60/libdpgo_hip.so python tools/trace_precision.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from dpgo_amd import hip as H
    from oracle import dpgo_oracle as O
    from tests._common import load_meas
    from tests.test_gpu_status_trace import _expected_records, _rtr_extended, _trace_deviation
    for name, r in (("tinyGrid3D", 3), ("smallGrid3D", 5)):
        meas = load_meas(name)
        d, n = meas.d, meas.num_poses
        Q = O.connection_laplacian(meas, n)
        P_ = O.QuadraticProblem(n, d, r)
        P_.set_Q(Q)
        P_.precon_mode = O.PRECON_BLOCK_JACOBI
        X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
        trace = []
        O.optimize(P_, X0, O.OptParams(tr_iterations=10, tr_tolerance=1e-1, tr_initial_radius=10.0,
                                       tr_max_inner=50), trace)
        ora = _expected_records(trace)
        ext = _rtr_extended(Q, X0, d, 1e-1, 10.0, 50.0, 10, 50)
        dev = {"oracle": _trace_deviation(ora, ext)}
        for label, classic, v2, edges in (("classic", 1, 0, 0), ("merged_bsr", 0, 0, 0), ("merged_edges_v1", 0, 0, 1),
                                          ("merged_edges_v2", 0, 1, 1)):
            H.set_tuning(5, classic)
            H.set_tuning(11, v2)
            try:
                h = H.Problem(n, d, r)
                if edges:
                    h.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
                else:
                    h.set_Q_scipy(0, Q)
                h.set_trace(4096)
                h.optimize(X0, H.default_params(tr_iterations=10, tr_tolerance=1e-1, tr_initial_radius=10.0,
                                                tr_max_inner=50, precon=H.PRECON_BLOCK_JACOBI))
                got = h.get_trace(0)
            finally:
                H.set_tuning(5, 0)
                H.set_tuning(11, 0)
            same = [int(g["op"]) for g in got] == [e["op"] for e in ext]
            dev[label] = _trace_deviation(got, ext) if same else float("inf")
        print(json.dumps({"lib": os.environ.get("DPGO_HIP_LIB", "tree"), "problem": name, "r": r,
                          "deviation_from_extended": dev}), flush=True)


if __name__ == "__main__":
    main()
