"""GPU chordal initialisation (chordalInitialization, src/DPGO_utils.cpp:377-476, as
examples/MultiRobotExample.cpp:158 uses it): both linear least-squares solves by Jacobi-PCG on the
device against the host direct solve (block Cholesky of the same normal equations, itself checked
against the oracle's scipy solve in tests/test_host_native.py) and the oracle."""
import numpy as np
import pytest

from oracle import dpgo_oracle as O
from tests._common import load_meas, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    from dpgo_amd import hip as H
    assert H.device_count() >= 1
    return H


@pytest.mark.parametrize("name", ["tinyGrid3D", "smallGrid3D", "sphere2500", "torus3D", "input_INTEL_g2o",
                                  "city10000", "kitti_00"])
def test_gpu_chordal_matches_direct_and_oracle(hip, name):
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    Tg, iters, rr = hip.chordal_initialization_gpu(d, n, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau,
                                                   rtol=1e-12)
    assert rr <= 1e-12 and iters > 0
    Th = hip.chordal_initialization(d, n, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau)
    To = O.chordal_initialization(d, n, meas)
    assert rel(Tg, Th) <= 1e-8
    assert rel(Tg, To) <= 1e-8
    b = d + 1
    for i in range(0, n, max(1, n // 50)):
        Ri = Tg[:, i * b:i * b + d]
        assert np.abs(Ri.T @ Ri - np.eye(d)).max() <= 1e-12
        assert np.linalg.det(Ri) > 0


def test_gpu_chordal_grid(hip):
    """A 20^3 synthetic grid (8000 poses, the BASELINE generator): PCG vs the direct factor."""
    g = hip.Graph.grid3d(20, seed=1)
    a = g.arrays()
    r = 5
    YL = O.lifting_matrix(3, r)
    Xg, iters, rr = g.chordal_init_gpu(r, YL, rtol=1e-12)
    Xh = g.chordal_init(r, YL)
    assert rel(Xg, Xh) <= 1e-8
    meas = O.Measurements(3, np.zeros(g.m, np.int64), np.zeros(g.m, np.int64), a["p1"].astype(np.int64),
                          a["p2"].astype(np.int64), a["R"], a["t"], a["kappa"], a["tau"], np.ones(g.m), g.n)
    assert O.central_cost(meas, Xg) < 1e-3 * O.central_cost(meas, g.chain_init(r, YL))


def test_gpu_chordal_reports_nonconvergence(hip):
    meas = load_meas("sphere2500")
    with pytest.raises(hip.DPGOHipError, match="PCG did not reach"):
        hip.chordal_initialization_gpu(meas.d, meas.num_poses, meas.p1, meas.p2, meas.R, meas.t, meas.kappa,
                                       meas.tau, rtol=1e-14, max_iters=3)


@pytest.mark.parametrize("name,agents", [("smallGrid3D", 5), ("city10000", 8)])
def test_gpu_distributed_init_matches_host_and_oracle(hip, name, agents):
    """Per-agent chordal (one block-diagonal PCG on the device) + frame alignment vs the host Cholesky
    path and the oracle restatement (PGOAgent::localInitialization + initializeInGlobalFrame)."""
    meas = load_meas(name)
    d, n, r = meas.d, meas.num_poses, 5
    aop = np.minimum(np.arange(n) // (n // agents), agents - 1).astype(np.int32)
    g = hip.Graph.from_arrays(d, n, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau)
    YL = O.lifting_matrix(d, r)
    Xg, iters, rr = g.distributed_init(aop, r, YL, gpu=True, rtol=1e-12)
    Xh, _, _ = g.distributed_init(aop, r, YL, gpu=False)
    assert rr <= 1e-12 and iters > 0
    assert rel(Xg, Xh) <= 1e-8
    assert rel(Xg, YL @ O.distributed_initialization(meas, aop, agents)) <= 1e-8


def test_gpu_distributed_init_grid_cubes(hip):
    """BASELINE's partition (cube agents) on a 24^3 grid: PCG vs host; far better than odometry."""
    g = hip.Graph.grid3d(24, seed=2)
    aop = g.grid_partition(4)
    r = 5
    YL = O.lifting_matrix(3, r)
    Xg, _, _ = g.distributed_init(aop, r, YL, gpu=True, rtol=1e-12)
    Xh, _, _ = g.distributed_init(aop, r, YL, gpu=False)
    assert rel(Xg, Xh) <= 1e-8
    e = hip.Rbcd(g, aop, np.zeros(64, np.int32), 0, 1, hip.rbcd_params(r=r))
    e.set_X(hip.to_dev_layout(Xg))
    f_dist, _ = e.central_eval()
    e.set_X(g.chain_init_dev_layout(r, YL))
    f_chain, _ = e.central_eval()
    assert f_dist < 1e-3 * f_chain
