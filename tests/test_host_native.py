"""CPU checks of the native library's host side (no GPU): ABI exports, no-CPU-fallback
behaviour, graph inputs (reader, grid generator, Laplacian) and the CPU port."""
import os
import re
import subprocess

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import dpgo_oracle as O
from tests._common import GOLDEN, load_meas, rel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def H():
    from dpgo_amd import hip
    return hip


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?(?:int|void|double|const char\*)\s*\**\s*(dpgo_\w+)\s*\(", txt, re.M))


def test_library_exports_every_declared_symbol(H):
    lib = os.path.join(ROOT, "dpgo_amd", "libdpgo_hip.so")
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (dpgo_\w+)", out))
    declared = _declared("dpgo_hip.h") | _declared("dpgo_rbcd.h")
    assert len(declared) > 40
    missing = declared - exported
    assert not missing, missing
    H.lib()  # ctypes binds every symbol the Python binding uses
    assert set(H.EXPORTED_SYMBOLS) <= exported


def test_library_built_from_this_tree(H):
    """The loaded libdpgo_hip.so carries the sha256 of the sources it was compiled from; it must be
    this tree's (a stale binary shipped beside newer sources fails here, on the CPU and on the box)."""
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as G
    assert H.build_id() == G.source_hash()


def test_no_cpu_fallback_without_device(H):
    if H.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(H.DPGOHipError, match="no gfx950 device"):
        H.Problem(10, 3, 5)


def test_grid3d_bitwise_identical_to_oracle(H):
    for k, seed in [(3, 0), (4, 0), (5, 7)]:
        g = H.Graph.grid3d(k, seed=seed)
        o = O.grid3d(k, seed=seed)
        a = g.arrays()
        assert np.array_equal(a["p1"], o.p1) and np.array_equal(a["p2"], o.p2)
        assert np.array_equal(a["R"], o.R) and np.array_equal(a["t"], o.t)
        assert g.m == 3 * k * k * (k - 1)


def test_grid_partition_and_chain_init(H):
    g = H.Graph.grid3d(6, seed=1)
    aop = g.grid_partition(3)
    assert aop.min() == 0 and aop.max() == 26 and np.all(np.bincount(aop) == 8)
    o = O.grid3d(6, seed=1)
    Y = O.lifting_matrix(3, 5)
    X = g.chain_init(5, Y)
    Xo = Y @ O.chain_initialization(3, o.num_poses, o)
    assert rel(X, Xo) <= 1e-12


@pytest.mark.parametrize("name", ["smallGrid3D", "sphere2500", "input_INTEL_g2o", "kitti_00"])
def test_laplacian_matches_oracle(H, name):
    meas = load_meas(name)
    g = H.Graph.from_arrays(meas.d, meas.num_poses, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau)
    rp, col, blk = g.laplacian_bsr()
    b = meas.d + 1
    Q = O.connection_laplacian(meas, meas.num_poses)
    Qb = sp.bsr_matrix((blk.reshape(-1, b, b).transpose(0, 2, 1), col, rp), shape=Q.shape)
    assert abs(Qb - Q).max() <= 1e-12 * abs(Q).max()


@pytest.mark.parametrize("name", ["smallGrid3D", "sphere2500", "input_INTEL_g2o", "kitti_00", "CSAIL",
                                  "city10000"])
def test_g2o_reader_matches_oracle(H, name):
    path = f"/root/reference/data/{name}.g2o"
    if not os.path.exists(path):
        pytest.skip("reference data not mounted (GPU box)")
    g = H.Graph.read_g2o(path)
    o = O.read_g2o(path)
    a = g.arrays()
    assert g.n == o.num_poses and g.m == o.m and g.duplicates == o.duplicates
    assert np.array_equal(a["p1"], o.p1) and np.array_equal(a["p2"], o.p2)
    assert rel(a["R"], o.R) <= 1e-15 and rel(a["t"], o.t) <= 1e-15
    assert rel(a["kappa"], o.kappa) <= 1e-12 and rel(a["tau"], o.tau) <= 1e-12


def test_cpu_port_matches_oracle_agent_step():
    """oracle/cpu (the timed baseline) agrees with the numpy oracle on one RBCD update."""
    from oracle import cpu_port
    g = O.grid3d(6, seed=2)
    s = 3
    aop = np.array([(c[0] // s) + 2 * ((c[1] // s) + 2 * (c[2] // s)) for c in g.extra["coords"]], np.int32)
    X0 = O.lifting_matrix(3, 5) @ O.chain_initialization(3, g.num_poses, g)
    arrays = dict(p1=g.p1, p2=g.p2, R=g.R, t=g.t, kappa=g.kappa, tau=g.tau)
    sec, f = cpu_port.time_agent_step(3, 5, arrays, g.num_poses, aop, 0, O.to_dev(X0), False, 8, 1)
    # oracle: agent 0, non-accelerated update with neighbour poses from X0
    local = np.zeros(g.num_poses, np.int64)
    cnt = np.zeros(8, np.int64)
    for i in range(g.num_poses):
        local[i] = cnt[aop[i]]
        cnt[aop[i]] += 1
    parts = O._split(g, aop, local, 8)
    ag = O.Agent(0, O.AgentParams(3, 5, 8, robust="L2", precon=O.PRECON_BLOCK_JACOBI))
    ag.set_pose_graph(*parts[0], n=int(cnt[0]))
    glob = np.nonzero(aop == 0)[0]
    cols = np.concatenate([np.arange(p * 4, p * 4 + 4) for p in glob])
    ag.set_X(X0[:, cols])
    for pid in ag.neighbor_shared:
        gp = np.nonzero(aop == pid[0])[0][pid[1]]
        ag.neighbor_pose[pid] = X0[:, gp * 4:gp * 4 + 4]
    ag.iterate(True)
    assert abs(f - ag.last_result["fOpt"]) <= 1e-9 * abs(ag.last_result["fOpt"])


@pytest.mark.parametrize("name", ["tinyGrid3D", "smallGrid3D", "sphere2500", "input_INTEL_g2o", "city10000",
                                  "kitti_00"])
def test_chordal_initialization_matches_oracle(H, name):
    """chordalInitialization (src/DPGO_utils.cpp:377-424): native host block-Cholesky solve of the
    rotation / translation least squares vs the oracle's normal-equation solve (same minimiser)."""
    from oracle import dpgo_oracle as O
    from tests._common import load_meas, rel
    meas = load_meas(name)
    d, n = meas.d, meas.num_poses
    T = H.chordal_initialization(d, n, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau)
    To = O.chordal_initialization(d, n, meas)
    assert rel(T, To) <= 1e-8
    b = d + 1
    for i in range(0, n, max(1, n // 50)):  # rotations on SO(d)
        Ri = T[:, i * b:i * b + d]
        assert np.abs(Ri.T @ Ri - np.eye(d)).max() <= 1e-12
        assert np.linalg.det(Ri) > 0


def test_cpp_host_cases():
    """Host-only cases of the C++ drop-in tests (no GPU call): chi2inv and the robust single
    rotation / pose averages of the global-frame initialisation, restating tests/testUtils.cpp:55-190,
    and the connection-Laplacian construction (tests/testConstruction.cpp)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    binary = os.path.join(root, "dpgo_amd", "cpp", "build", "test_dpgo")
    assert os.path.exists(binary), "C++ tests not built (run __graft_entry__.build())"
    p = subprocess.run([binary, os.path.join(root, "tests", "golden"), "--host"], capture_output=True, text=True,
                       timeout=300)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-3000:]
    for name in ["Chi2Inv", "RobustSingleRotationAveraging", "RobustSinglePoseAveraging", "Construction"]:
        assert f"[PASS] {name}" in out, out[-3000:]


@pytest.mark.parametrize("name,agents", [("smallGrid3D", 5), ("input_INTEL_g2o", 4), ("city10000", 8)])
def test_distributed_initialization_matches_oracle(H, name, agents):
    """PGOAgent::localInitialization per agent + initializeInGlobalFrame (host Cholesky path) vs the
    oracle's restatement: contiguous agents as examples/MultiRobotExample.cpp:73-90."""
    from oracle import dpgo_oracle as O
    from tests._common import load_meas, rel
    meas = load_meas(name)
    d, n, r = meas.d, meas.num_poses, 5
    aop = np.minimum(np.arange(n) // (n // agents), agents - 1).astype(np.int32)
    g = H.Graph.from_arrays(d, n, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau)
    YL = O.lifting_matrix(d, r)
    X, _, _ = g.distributed_init(aop, r, YL, gpu=False)
    To = O.distributed_initialization(meas, aop, agents)
    assert rel(X, YL @ To) <= 1e-8
    # the init is a good start: far below the odometry chain's cost
    assert O.central_cost(meas, YL @ To) < O.central_cost(meas, YL @ O.chain_initialization(d, n, meas))


@pytest.mark.parametrize("accel", [False, True])
def test_cpu_engine_matches_oracle_colour_schedule(accel):
    """oracle/cpu's multi-agent colour schedule (the like-for-like CPU baseline, OpenMP over a colour's
    agents) vs the numpy PGOAgent restatement, through a Nesterov restart (iteration 29)."""
    from oracle import cpu_port
    k, A, r = 6, 2, 5
    g = O.grid3d(k, seed=3)
    s = k // A
    aop = np.array([(c[0] // s) + A * ((c[1] // s) + A * (c[2] // s)) for c in g.extra["coords"]], np.int32)
    X0 = O.lifting_matrix(3, r) @ O.chain_initialization(3, g.num_poses, g)
    arrays = dict(p1=g.p1, p2=g.p2, R=g.R, t=g.t, kappa=g.kappa, tau=g.tau)
    E = cpu_port.CpuRbcd(3, r, arrays, g.num_poses, aop, A ** 3, accel)
    E.set_X(O.to_dev(X0))
    iters = 31
    for _ in range(iters):
        E.iterate(threads=4)
    agents, trace = [], []
    Xo, cols = O.colour_rbcd(g, aop, A ** 3, X0, iters, r, acceleration=accel, agents_out=agents, trace=trace)
    assert E.colors == cols
    assert rel(O.from_dev(E.get_X(), r), Xo) <= 1e-10
    rc, rd = E.status()
    for a, ag in enumerate(agents):
        assert abs(rc[a] - ag.status_relative_change) <= 1e-9 * ag.status_relative_change
        assert bool(rd[a]) == bool(ag.ready_to_terminate)
    st = E.stats()
    runs = np.zeros(A ** 3, int)
    pending = []
    for t in trace:
        if isinstance(t, tuple):
            runs[t[1]] += len(pending)
            pending = []
        else:
            pending.append(t)
    assert list(st[:, 2]) == list(runs)


@pytest.mark.parametrize("accel", [False, True])
def test_cpu_engine_gnc_tls_matches_oracle(accel):
    """oracle/cpu's GNC_TLS (PGOAgent::updateLoopClosuresWeights, src/PGOAgent.cpp:1174-1289: reweighting every
    robust_opt_inner_iters iterations, shared edges by the lower-ID agent only, mu schedule, Nesterov restart
    on reweighting, converged-ratio readiness) vs the numpy PGOAgent restatement on a grid with outliers."""
    from oracle import cpu_port
    k, A, r, inner, iters = 6, 2, 5, 3, 8
    g = O.grid3d(k, seed=3)
    s = k // A
    aop = np.array([(c[0] // s) + A * ((c[1] // s) + A * (c[2] // s)) for c in g.extra["coords"]], np.int32)
    rng = np.random.default_rng(7)
    lc = np.nonzero(np.abs(g.p2 - g.p1) != 1)[0]
    bad = rng.choice(lc, size=max(1, len(lc) // 10), replace=False)
    g.t = g.t.copy()
    g.t[bad] += rng.normal(0.0, 5.0, size=(len(bad), 3))
    X0 = O.lifting_matrix(3, r) @ O.chain_initialization(3, g.num_poses, g)
    arrays = dict(p1=g.p1, p2=g.p2, R=g.R, t=g.t, kappa=g.kappa, tau=g.tau)
    E = cpu_port.CpuRbcd(3, r, arrays, g.num_poses, aop, A ** 3, accel, robust="GNC_TLS",
                         robust_opt_inner_iters=inner)
    E.set_X(O.to_dev(X0))
    for _ in range(iters):
        E.iterate(threads=4)
    agents = []
    Xo, _ = O.colour_rbcd(g, aop, A ** 3, X0, iters, r, acceleration=accel, robust="GNC_TLS",
                          robust_opt_inner_iters=inner, agents_out=agents)
    assert rel(O.from_dev(E.get_X(), r), Xo) <= 1e-9
    rc, rd = E.status()
    for a, ag in enumerate(agents):
        assert abs(rc[a] - ag.status_relative_change) <= 1e-8 * ag.status_relative_change
        assert bool(rd[a]) == bool(ag.ready_to_terminate)
    assert min(ag.converged_loop_closure_ratio() for ag in agents) < 1.0  # the reweighting decided some


def test_cpu_engine_gnc_dictionary_many_colours():
    """oracle/cpu's GNC_TLS reads a shared loop closure's other endpoint from the agent's own neighbour-pose dictionary
    (PGOAgent::neighborPoseDict, src/PGOAgent.cpp:1201-1235), filled only when the agent is selected
    (examples/MultiRobotExample.cpp:188-213), and keeps the weight of an edge whose neighbour pose it never received.
    A random 6-agent partition (>= 3 colours) reweighted every 2 iterations -- the first reweighting comes before
    some colours were ever selected, later ones read dictionaries older than the neighbours' current X -- against the
    numpy PGOAgent restatement at 1e-9."""
    from oracle import cpu_port
    k, K, r, inner, iters = 5, 6, 5, 2, 9
    g = O.grid3d(k, seed=4)
    aop = np.random.default_rng(11).integers(0, K, g.num_poses).astype(np.int32)
    assert max(O.greedy_colors(g, aop, K)) + 1 >= 3
    rng = np.random.default_rng(8)
    lc = np.nonzero(np.abs(g.p2 - g.p1) != 1)[0]
    bad = rng.choice(lc, size=max(1, len(lc) // 8), replace=False)
    g.t = g.t.copy()
    g.t[bad] += rng.normal(0.0, 5.0, size=(len(bad), 3))
    X0 = O.lifting_matrix(3, r) @ O.chain_initialization(3, g.num_poses, g)
    arrays = dict(p1=g.p1, p2=g.p2, R=g.R, t=g.t, kappa=g.kappa, tau=g.tau)
    E = cpu_port.CpuRbcd(3, r, arrays, g.num_poses, aop, K, True, robust="GNC_TLS", robust_opt_inner_iters=inner)
    E.set_X(O.to_dev(X0))
    for _ in range(iters):
        E.iterate(threads=4)
    agents = []
    Xo, _ = O.colour_rbcd(g, aop, K, X0, iters, r, acceleration=True, robust="GNC_TLS",
                          robust_opt_inner_iters=inner, agents_out=agents)
    assert rel(O.from_dev(E.get_X(), r), Xo) <= 1e-9
    assert min(ag.converged_loop_closure_ratio() for ag in agents) < 1.0


@pytest.mark.parametrize("accel,robust", [(False, "L2"), (True, "L2"), (True, "GNC_TLS")])
def test_cpu_engine_exact_precon_matches_oracle(accel, robust):
    """oracle/cpu's exact preconditioner (P = Q + 0.1 I factorised per Q, src/QuadraticProblem.cpp:31-42, 75-87;
    a reverse Cuthill-McKee envelope Cholesky that shares no code with the GPU library's supernodal factor) vs the
    numpy restatement's sparse LU inside the same colour schedule: X to 1e-10 over 12 iterations (L2; the trajectory
    from the odometry chain amplifies rounding ~10x per 4 iterations, so 31 iterations sit at 1e-9..1e-8 for either
    side's arithmetic), GNC_TLS with a refactorisation after every reweighting (every 3 iterations) to 1e-9."""
    from oracle import cpu_port
    k, A, r = 6, 2, 5
    g = O.grid3d(k, seed=3)
    s = k // A
    aop = np.array([(c[0] // s) + A * ((c[1] // s) + A * (c[2] // s)) for c in g.extra["coords"]], np.int32)
    if robust != "L2":
        rng = np.random.default_rng(7)
        lc = np.nonzero(np.abs(g.p2 - g.p1) != 1)[0]
        bad = rng.choice(lc, size=max(1, len(lc) // 10), replace=False)
        g.t = g.t.copy()
        g.t[bad] += rng.normal(0.0, 5.0, size=(len(bad), 3))
    X0 = O.lifting_matrix(3, r) @ O.chain_initialization(3, g.num_poses, g)
    arrays = dict(p1=g.p1, p2=g.p2, R=g.R, t=g.t, kappa=g.kappa, tau=g.tau)
    E = cpu_port.CpuRbcd(3, r, arrays, g.num_poses, aop, A ** 3, accel, robust=robust, robust_opt_inner_iters=3,
                         precon="exact")
    E.set_X(O.to_dev(X0))
    iters = 12 if robust == "L2" else 8
    for _ in range(iters):
        E.iterate(threads=4)
    agents, trace = [], []
    Xo, _ = O.colour_rbcd(g, aop, A ** 3, X0, iters, r, acceleration=accel, robust=robust, robust_opt_inner_iters=3,
                          agents_out=agents, trace=trace, precon=O.PRECON_EXACT)
    assert rel(O.from_dev(E.get_X(), r), Xo) <= (1e-10 if robust == "L2" else 1e-9)
    runs = np.zeros(A ** 3, int)
    pending = []
    for t in trace:
        if isinstance(t, tuple):
            runs[t[1]] += len(pending)
            pending = []
        else:
            pending.append(t)
    assert list(E.stats()[:, 2]) == list(runs)
    cnt, _ = E.factor_info()
    assert cnt.min() >= 1 and (robust == "L2") == (cnt.max() == 1)  # refactorised after the reweightings
    # the block-Jacobi schedule is a different trajectory: the exact factor is what ran
    Eb = cpu_port.CpuRbcd(3, r, arrays, g.num_poses, aop, A ** 3, accel, robust=robust, robust_opt_inner_iters=3)
    Eb.set_X(O.to_dev(X0))
    for _ in range(iters):
        Eb.iterate(threads=4)
    assert rel(Eb.get_X(), E.get_X()) > 1e-3


def build_abi_check(tmp_path):
    """tests/c/abi_check.c compiled against include/*.h and linked to the in-tree libdpgo_hip.so."""
    exe = str(tmp_path / "abi_check")
    libdir = os.path.join(ROOT, "dpgo_amd")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    "-I", "/opt/rocm/include", os.path.join(ROOT, "tests", "c", "abi_check.c"), "-o", exe,
                    "-L", libdir, "-ldpgo_hip", "-Wl,-rpath," + libdir], check=True)
    return exe


def test_c_header_constants_match_library(H, tmp_path):
    """A C caller sizes its per-mode / per-agent arrays from the header: the header's constants must be the
    library's (the Python binding's mode list is the library's kSpmmModes order)."""
    exe = build_abi_check(tmp_path)
    out = subprocess.run([exe, "consts"], capture_output=True, text=True, check=True).stdout
    vals = dict((k, int(v)) for k, v in (ln.split() for ln in out.strip().splitlines()))
    assert vals["DPGO_SPMM_MODES"] == len(H.SPMM_MODES) == 11
    assert vals["DPGO_STATS_INTS"] == H.STATS_INTS
    assert vals["DPGO_RCCL_ID_BYTES"] == 128
