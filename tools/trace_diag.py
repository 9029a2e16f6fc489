#!/usr/bin/env python3
"""Per-record deviation of the device RTR trace from the oracle's (tinyGrid3D, block-Jacobi, the
localPoseGraphOptimization settings) for the merged and the classic tCG sequences: which record, which
outer iteration, how far (relative to the quantity's largest magnitude in its tCG)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import dpgo_oracle as O  # noqa: E402
from tests._common import load_meas  # noqa: E402
from tests.test_gpu_status_trace import _expected_records  # noqa: E402
from dpgo_amd import hip as H  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "tinyGrid3D"
r = int(sys.argv[2]) if len(sys.argv) > 2 else 3
meas = load_meas(name)
d, n = meas.d, meas.num_poses
Q = O.connection_laplacian(meas, n)
P = O.QuadraticProblem(n, d, r)
P.set_Q(Q)
P.precon_mode = O.PRECON_BLOCK_JACOBI
X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
trace = []
O.optimize(P, X0, O.OptParams(tr_iterations=10, tr_tolerance=1e-1, tr_initial_radius=10.0, tr_max_inner=50), trace)
exp = _expected_records(trace)
for classic in (0, 1):
    H.set_tuning(5, classic)
    h = H.Problem(n, d, r)
    h.set_Q_scipy(0, Q)
    h.set_trace(4096)
    h.optimize(X0, H.default_params(tr_iterations=10, tr_tolerance=1e-1, tr_initial_radius=10.0, tr_max_inner=50,
                                    precon=H.PRECON_BLOCK_JACOBI))
    got = h.get_trace(0)
    H.set_tuning(5, 0)
    print(f"== {'classic' if classic else 'merged'}: {len(got)} records (oracle {len(exp)})")
    outer, scale = 0, {}
    for i, (g, e) in enumerate(zip(got, exp)):
        if e["op"] == 5:
            outer += 1
            scale = {}
            continue
        for k in ("d_Hd", "norm_r", "z_r", "beta", "alpha"):
            if k in e:
                scale[k] = max(scale.get(k, 0.0), abs(e[k]))
        devs = {k: abs(g[k] - e[k]) / max(scale[k], 1e-300) for k in ("d_Hd", "norm_r", "z_r", "beta") if k in e}
        worst = max(devs.values()) if devs else 0.0
        if worst > 1e-12:
            print(f"  rec {i} outer {outer} op {e['op']} j {e['j']}: " + ", ".join(f"{k} {v:.1e}" for k, v in devs.items()))
