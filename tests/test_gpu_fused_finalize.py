"""Opt-in fused finalize (DPGO_FUSE_FINALIZE=1/2: the last-arriving SpMM block of each agent runs
k_finalize's work) must give bitwise the same RTR result as the separate k_finalize launch; both
restate the same 256-wide summation tree (kernels.hip finalize_agent / k_finalize)."""
import os

import numpy as np
import pytest

from tests._common import load_meas

pytestmark = pytest.mark.gpu


def _run(mode):
    from dpgo_amd import hip as H
    from oracle import dpgo_oracle as O

    meas = load_meas("smallGrid3D")
    d, n, r = meas.d, meas.num_poses, 5
    Q = O.connection_laplacian(meas, n)
    X0 = O.lifting_matrix(d, r) @ O.chordal_initialization(d, n, meas)
    old = os.environ.get("DPGO_FUSE_FINALIZE")
    os.environ["DPGO_FUSE_FINALIZE"] = str(mode)
    try:
        h = H.Problem(n, d, r)  # the mode is read when the handle is created
    finally:
        if old is None:
            del os.environ["DPGO_FUSE_FINALIZE"]
        else:
            os.environ["DPGO_FUSE_FINALIZE"] = old
    h.set_Q_scipy(0, Q)
    X, res = h.optimize(X0, H.default_params(tr_iterations=3, tr_tolerance=1e-6, tr_initial_radius=10.0,
                                             tr_max_inner=10))
    return np.asarray(X), res[0]


@pytest.mark.parametrize("mode", [1, 2])
def test_fused_finalize_bitwise(mode):
    X0, r0 = _run(0)
    X1, r1 = _run(mode)
    assert np.array_equal(X0, X1)
    assert r0["fOpt"] == r1["fOpt"] and r0["gradNormOpt"] == r1["gradNormOpt"]
    assert r1["fOpt"] < r1["fInit"]
