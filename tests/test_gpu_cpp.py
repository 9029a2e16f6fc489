"""Runs the C++ drop-in tests (tests/cpp/test_dpgo.cpp, built by __graft_entry__.build()) on the
GPU: the reference's gtests restated against DPGO::PGOAgent / QuadraticProblem / LiftedSEManifold,
and the multi-robot example loop compared with the oracle's log."""
import os
import subprocess

import numpy as np
import pytest

from tests._common import GOLDEN

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "dpgo_amd", "cpp", "build", "test_dpgo")


@pytest.fixture(scope="module")
def cpp_output():
    assert os.path.exists(BIN), "C++ tests not built (run __graft_entry__.build())"
    p = subprocess.run([BIN, GOLDEN], capture_output=True, text=True, timeout=300)
    return p.returncode, p.stdout + p.stderr


@pytest.mark.parametrize("name", ["Chi2Inv", "RobustSingleRotationAveraging", "RobustSinglePoseAveraging",
                                  "MultiRobotInitialization", "Construction", "MemoryLayout", "Stiefel",
                                  "TriangleGraph", "LineGraph", "MultiRobotExample"])
def test_cpp_case(cpp_output, name):
    rc, out = cpp_output
    assert f"[PASS] {name}" in out, out[-3000:]


def test_cpp_multirobot_matches_oracle(cpp_output):
    """examples/MultiRobotExample.cpp loop (5 robots, Nesterov, GNC_TLS defaults, the reference's exact
    preconditioner) through the C++ drop-in on the GPU vs the oracle's restatement: same greedy robot
    sequence, same costs."""
    rc, out = cpp_output
    rows = [l.split() for l in out.splitlines() if l.startswith("ITER ")]
    got = np.array([[float(x) for x in r[1:]] for r in rows])
    ref = np.load(os.path.join(GOLDEN, "smallGrid3D.multirobot5.exact.npz"))["log"]
    assert got.shape == ref.shape
    assert np.array_equal(got[:, 1], ref[:, 1]), "greedy selection sequence differs"
    assert np.max(np.abs(got[:, 2] - ref[:, 2]) / ref[:, 2]) <= 1e-9
    assert np.max(np.abs(got[:, 3] - ref[:, 3]) / ref[:, 3]) <= 1e-7
