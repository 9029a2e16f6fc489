"""BASELINE configs[3] and [4] at full size on the GPU: synthetic grids of
48^3 = 110,592 and 100^3 = 10^6 poses, r = 5, 64 cube agents, from the multi-robot initialisation.

The numpy oracle cannot run these sizes; parity is checked against oracle/cpu's multi-agent colour
schedule (itself pinned to the numpy oracle through a Nesterov restart in tests/test_host_native.py)
and through size-independent properties: the central cost never increases without acceleration
(block-coordinate descent), the result does not depend on the number of ranks (bitwise), the Nesterov
restart (iteration 29, src/PGOAgent.cpp:1033-1060) and the GNC reweighting at the default cadence
(every 30 iterations, :1174-1181) fire inside the run.  tests/ infrastructure only."""
import os
import socket

import numpy as np
import pytest

from oracle import dpgo_oracle as O
from tests._common import rel

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R = 5


@pytest.fixture(scope="module")
def hip():
    from dpgo_amd import hip as H
    assert H.device_count() >= 1
    return H


_CACHE = {}


def _setup(hip, k):
    """Graph, cube partition and the distributed initialisation (cached per size)."""
    if k not in _CACHE:
        g = hip.Graph.grid3d(k, seed=0)
        aop = g.grid_partition(4)
        YL = hip.lifting_matrix(3, R)
        X0, it, rr = g.distributed_init(aop, R, YL, gpu=True, rtol=1e-12, max_iters=50000, dev_layout=True)
        _CACHE[k] = (g, aop, X0)
    return _CACHE[k]


def _engine(hip, g, aop, accel, robust="L2", ranks=None, rank=0, world=1, exact=False):
    ranks = np.zeros(64, np.int32) if ranks is None else ranks
    return hip.Rbcd(g, aop, ranks, rank, world, hip.rbcd_params(
        r=R, acceleration=int(accel), robust_cost=hip.ROBUST[robust],
        precon=hip.PRECON_EXACT if exact else hip.PRECON_BLOCK_JACOBI))


def _cpu(g, aop, accel, robust="L2", exact=False):
    from oracle import cpu_port
    return cpu_port.CpuRbcd(3, R, g.arrays(), g.n, aop, 64, accel, robust=robust,
                            precon="exact" if exact else "block_jacobi")


@pytest.mark.parametrize("k", [48, 100])
def test_distributed_init_full_size(hip, k):
    """The initial iterate: every rotation on SO(3), and far below the odometry chain's cost."""
    g, aop, X0 = _setup(hip, k)
    X = X0.reshape(-1, 4, R)  # pose, column, row
    for j in range(0, g.n, g.n // 997):
        Y = X[j, :3, :].T
        assert np.abs(Y.T @ Y - np.eye(3)).max() <= 1e-12
    e = _engine(hip, g, aop, False)
    e.set_X(X0)
    f0, _ = e.central_eval()
    e.set_X(g.chain_init_dev_layout(R, hip.lifting_matrix(3, R)))
    f_chain, _ = e.central_eval()
    assert f0 < 1e-3 * f_chain


def test_c4_monotone_without_acceleration_and_cpu_parity(hip):
    """C4 (110,592 poses), 36 iterations without acceleration: the central cost never increases, and
    X, statuses and solver counters equal oracle/cpu's run of the same schedule."""
    g, aop, X0 = _setup(hip, 48)
    e = _engine(hip, g, aop, False)
    e.set_X(X0)
    f_prev, _ = e.central_eval()
    iters = 36
    for it in range(iters):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
        f, gn = e.central_eval()
        assert f <= f_prev * (1 + 1e-13), (it, f, f_prev)
        f_prev = f
    Xg = np.zeros(X0.size)
    e.get_X_into(Xg)
    cpu = _cpu(g, aop, False)
    cpu.set_X(X0)
    for _ in range(iters):
        cpu.iterate(threads=16)
    assert rel(Xg, cpu.get_X()) <= 1e-9
    st_g, st_c = e.stats()[:, :10], cpu.stats()
    assert np.array_equal(st_g[:, 2:4], st_c[:, 2:4])  # Runs and tCG iterations per agent
    rc_g, rd_g = e.status()
    rc_c, rd_c = cpu.status()
    assert np.allclose(rc_g, rc_c, rtol=1e-8, atol=0)
    assert np.array_equal(rd_g, rd_c)


def test_c4_nesterov_restart_cpu_parity(hip):
    """C4 with Nesterov: 36 iterations (the restart at iteration 29 fires), against oracle/cpu."""
    g, aop, X0 = _setup(hip, 48)
    e = _engine(hip, g, aop, True)
    e.set_X(X0)
    f0, _ = e.central_eval()
    iters = 36
    for it in range(iters):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
    f1, _ = e.central_eval()
    assert f1 < f0
    Xg = np.zeros(X0.size)
    e.get_X_into(Xg)
    cpu = _cpu(g, aop, True)
    cpu.set_X(X0)
    for _ in range(iters):
        cpu.iterate(threads=16)
    assert rel(Xg, cpu.get_X()) <= 1e-9
    assert np.array_equal(e.stats()[:, 2:4], cpu.stats()[:, 2:4])
    # the restart re-ran updateX from XPrev for the selected colour: one extra optimize call each
    calls = e.stats()[:, 0]
    assert calls.sum() == 32 * iters + 32


@pytest.mark.timeout(900)
@pytest.mark.parametrize("accel", [False, True])
def test_c4_exact_precon_cpu_parity(hip, accel):
    """C4 (110,592 poses, 64 agents of 12^3) with the reference's default preconditioner: the engine's supernodal
    factor of Q + 0.1 I (nested-dissection tree on the host, numeric factorisation and panel sweeps on the device)
    against oracle/cpu's independent exact mode (reverse Cuthill-McKee envelope Cholesky on the host,
    tests/test_host_native.py pins it to the numpy oracle's sparse LU), in lockstep over 36 colour iterations from the
    multi-robot initialisation (with Nesterov: through the restart at iteration 29).  Every agent's Run and tCG
    counters are equal after every iteration, and X agrees to 1e-12 through iteration 12.  Later the trajectory itself
    amplifies rounding (~1.75x per iteration without acceleration: a smooth geometric rise with identical solver
    decisions, profiles/r05b_exact_probe_c4.log), so the final bar is derived like the trace tests': max(1e-9, 2 x the
    largest distance between the port and three runs of itself with 1e-16 relative noise injected after every
    iteration -- a model of an implementation whose rounding differs in every step)."""
    g, aop, X0 = _setup(hip, 48)
    e = _engine(hip, g, aop, accel, exact=True)
    e.set_X(X0)
    cpu = _cpu(g, aop, accel, exact=True)
    cpu.set_X(X0)
    iters = 36
    Xg = np.zeros(X0.size)
    for it in range(iters):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
        cpu.iterate(threads=16)
        assert np.array_equal(e.stats()[:, 2:4], cpu.stats()[:, 2:4]), it  # Runs and tCG iterations per agent
        if it == 12:
            e.get_X_into(Xg)
            assert rel(Xg, cpu.get_X()) <= 1e-12, (it, rel(Xg, cpu.get_X()))
    e.get_X_into(Xg)
    Xc = cpu.get_X()
    err = rel(Xg, Xc)
    # the trajectory's own amplification of rounding: three twins of the port whose X, Y, V are multiplied by
    # (1 + 1e-16 u) after EVERY iteration (CpuRbcd.perturb, Nesterov state kept) -- the GPU's rounding differs from the
    # port's in every reduction of every step, which a single perturbation of the start under-represents (round 5's
    # twins: 3.4e-10 .. 9.1e-10 against the GPU's 2.75e-9 with acceleration)
    floors = []
    for seed in (1, 2, 3):
        twin = _cpu(g, aop, accel, exact=True)
        twin.set_X(X0)
        for it in range(iters):
            twin.iterate(threads=16)
            twin.perturb(1e-16, 1000 * seed + it)
        floors.append(rel(twin.get_X(), Xc))
    floor = max(floors)
    print(f"C4 exact accel={accel}: |X_gpu - X_cpu| / |X| = {err:.2e}, port vs its per-step 1e-16-noise twins "
          + ", ".join(f"{x:.2e}" for x in floors))
    assert err <= max(1e-9, 2.0 * floor)
    assert cpu.stats()[:, 3].sum() > cpu.stats()[:, 2].sum()  # CG steps beyond the first were taken
    bj = _cpu(g, aop, accel)  # and the preconditioner matters on this trajectory
    bj.set_X(X0)
    for _ in range(iters):
        bj.iterate(threads=16)
    assert rel(bj.get_X(), Xc) > 1e-6


@pytest.mark.timeout(900)
@pytest.mark.parametrize("robust", ["L2", "GNC_TLS"])
def test_exact_stop_rule_cost_parity(hip, robust):
    """north_star's quantities with the reference's default preconditioner: the engine (device supernodal factor of
    Q + 0.1 I, refactorised on the device after every GNC reweighting) and oracle/cpu's independent exact mode (RCM
    envelope Cholesky on the host) run the colour schedule with Nesterov in lockstep from the multi-robot
    initialisation until the example's stop rule, central |RieGrad| < 0.1 (examples/MultiRobotExample.cpp:229-241),
    on grid3d k = 24 with 8 agents of 12^3 poses (the C4 agent shape; C4 itself needs > 3,000 iterations to the stop
    rule, profiles/r06b_exact_stop_rule_c4_*.json).  Both stop at the same iteration; there the central cost agrees to
    1e-9 relative (measured ~1e-13) and the gradient norm to 1e-9 of the initial gradient norm; the gradient norm's
    own relative difference is bounded by 2x the port's distance from its twin started 1e-15 away (a residual of a
    trajectory whose tCG decisions amplify rounding: measured 2e-7 L2 / 5e-6 GNC_TLS against twins 2e-6 / 1.5e-5,
    profiles/r06c_stop_rule_k24_*.json).  The per-agent Run / tCG counters stay equal every iteration as long as the
    port's own twin keeps them (L2: to the stop; GNC_TLS: both lose lockstep after ~200 iterations).  The cost and
    gradient norm of the port's iterate are computed in numpy from the dataset's Q (tests/_common.py)."""
    from tests._common import central_cost_gradnorm, unit_laplacian
    g = hip.Graph.grid3d(24, seed=0)
    aop = g.grid_partition(2)
    X0, _, _ = g.distributed_init(aop, R, hip.lifting_matrix(3, R), gpu=True, rtol=1e-12, max_iters=50000,
                                  dev_layout=True)
    Q = unit_laplacian(g.arrays(), g.n)
    from oracle import cpu_port
    e = hip.Rbcd(g, aop, np.zeros(8, np.int32), 0, 1, hip.rbcd_params(
        r=R, acceleration=1, robust_cost=hip.ROBUST[robust], precon=hip.PRECON_EXACT))
    e.set_X(X0)
    ports = []
    for seed in (None, 1):
        c = cpu_port.CpuRbcd(3, R, g.arrays(), g.n, aop, 8, True, robust=robust, precon="exact")
        c.set_X(X0 if seed is None else X0 * (1.0 + 1e-15 * np.random.default_rng(seed).standard_normal(X0.size)))
        ports.append(c)
    cpu, twin = ports
    g0 = central_cost_gradnorm(Q, hip.from_dev_layout(X0, R), 3)[1]
    flip = twin_flip = None
    stop_gpu = stop_cpu = None
    Xg = np.zeros(X0.size)
    for it in range(1, 2001):
        e.pre_exchange((it - 1) % e.num_colors)
        e.update((it - 1) % e.num_colors, None)
        cpu.iterate(threads=16)
        twin.iterate(threads=16)
        sc = cpu.stats()[:, 2:4]
        if flip is None and not np.array_equal(e.stats()[:, 2:4], sc):
            flip = it
        if twin_flip is None and not np.array_equal(twin.stats()[:, 2:4], sc):
            twin_flip = it
        if it % 5:
            continue
        fg, gg = e.central_eval()
        gg = float(np.sqrt(gg.sum()))
        fc, gc = central_cost_gradnorm(Q, hip.from_dev_layout(cpu.get_X(), R), 3)
        if stop_gpu is None and gg < 0.1:
            stop_gpu = it
        if stop_cpu is None and gc < 0.1:
            stop_cpu = it
        if stop_gpu and stop_cpu:
            break
    assert stop_gpu is not None and stop_gpu == stop_cpu, (stop_gpu, stop_cpu)
    ft, gt = central_cost_gradnorm(Q, hip.from_dev_layout(twin.get_X(), R), 3)
    e.get_X_into(Xg)
    print(f"{robust} exact to the stop rule: iteration {stop_gpu}; f {fg:.10f} vs {fc:.10f} (rel {abs(fg - fc) / fc:.2e}, "
          f"twin {abs(ft - fc) / fc:.2e}); |RG| {gg:.8f} vs {gc:.8f} (rel {abs(gg - gc) / gc:.2e}, twin "
          f"{abs(gt - gc) / gc:.2e}, |RG_0| {g0:.1f}); X rel {rel(Xg, cpu.get_X()):.2e}; counters flip at {flip}, "
          f"twin at {twin_flip}")
    assert abs(fg - fc) <= 1e-9 * abs(fc)
    assert abs(gg - gc) <= 1e-9 * g0
    assert abs(gg - gc) <= max(1e-9 * gc, 2.0 * abs(gt - gc))
    if flip is not None:  # lockstep lost only where the port's own twin loses it too, and not earlier than it
        assert twin_flip is not None and flip >= twin_flip, (flip, twin_flip)
    if robust == "L2":
        assert flip is None


def test_c4_gnc_default_cadence(hip):
    """GNC_TLS (the reference default) at robust_opt_inner_iters = 30: the reweighting at iteration 29
    changes the solution (not the L2 trajectory) and the converged-ratio status reflects it."""
    g, aop, X0 = _setup(hip, 48)
    out = {}
    for robust in ("L2", "GNC_TLS"):
        e = _engine(hip, g, aop, True, robust)
        e.set_X(X0)
        for it in range(32):
            e.pre_exchange(it % e.num_colors)
            e.update(it % e.num_colors, None)
        X = np.zeros(X0.size)
        e.get_X_into(X)
        out[robust] = (X, e.central_eval()[0])
    assert rel(out["GNC_TLS"][0], out["L2"][0]) > 1e-9
    assert np.isfinite(out["GNC_TLS"][1])


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dpgo_amd import hip as H
        import bench
        g, aop, X0 = _setup(H, 48)
        e = _engine(H, g, aop, True, ranks=bench.super_cube_ranks(4, world), rank=rank, world=world)
        e.set_X(X0)
        dev = torch.device("cuda", 0)
        s = torch.cuda.Stream(dev)
        e.set_stream(s.cuda_stream)
        with torch.cuda.stream(s):
            send = torch.zeros(max(int(e.send_counts.sum()), 1), dtype=torch.float64, device=dev)
            recv = torch.zeros(max(int(e.recv_counts.sum()), 1), dtype=torch.float64, device=dev)
            for it in range(32):
                c = it % e.num_colors
                e.pre_exchange(c)
                e.pack(send.data_ptr())
                hr = torch.empty_like(recv, device="cpu")
                dist.all_to_all_single(hr, send.cpu(), [int(x) for x in e.recv_counts], [int(x) for x in e.send_counts])
                recv.copy_(hr)
                e.update(c, recv.data_ptr())
        X = np.zeros(X0.size)
        e.get_X_into(X)
        q.put((rank, X))
    finally:
        dist.destroy_process_group()


def test_c4_two_ranks_bitwise_one_rank(hip):
    """C4, Nesterov, 32 iterations over two ranks (one device, halo over gloo) == one rank, bitwise."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    X2 = outs[0][1] + outs[1][1]
    g, aop, X0 = _setup(hip, 48)
    e = _engine(hip, g, aop, True)
    e.set_X(X0)
    for it in range(32):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
    X1 = np.zeros(X0.size)
    e.get_X_into(X1)
    assert np.array_equal(X1, X2)


def test_c5_iterations_cpu_parity(hip):
    """C5 (10^6 poses, 64 agents of 15,625), Nesterov: the engine against oracle/cpu after 2 colour
    iterations (every agent updated once), after 30 (past the Nesterov restart at iteration 29,
    src/PGOAgent.cpp:1033-1060) and after 36: X to 1e-9 and the per-agent Run / tCG counters equal; the
    central cost decreases."""
    g, aop, X0 = _setup(hip, 100)
    e = _engine(hip, g, aop, True)
    e.set_X(X0)
    f0, gn0 = e.central_eval()
    cpu = _cpu(g, aop, True)
    cpu.set_X(X0)
    it = 0
    for stop in (2, 30, 36):
        for it in range(it, stop):
            e.pre_exchange(it % e.num_colors)
            e.update(it % e.num_colors, None)
            cpu.iterate(threads=16)
        it = stop
        Xg = np.zeros(X0.size)
        e.get_X_into(Xg)
        assert rel(Xg, cpu.get_X()) <= 1e-9, stop
        assert np.array_equal(e.stats()[:, 2:4], cpu.stats()[:, 2:4]), stop
    f1, gn1 = e.central_eval()
    assert f1 < f0 and np.isfinite(f1)


def test_c5_burnin_regime_cpu_parity(hip):
    """The regime bench.py times (C5, Nesterov, 300 untimed steps from the distributed initialisation, then
    set_X of the burnt-in iterate): from that X the engine and oracle/cpu run the same 24 colour iterations --
    every update 10 tCG iterations deep -- and end with X equal to 1e-9 and the per-agent Run / tCG counters
    equal (the bench's like_for_like replay, as a test)."""
    g, aop, X0 = _setup(hip, 100)
    e = _engine(hip, g, aop, True)
    e.set_X(X0)
    for it in range(600):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
    Xb = np.zeros(X0.size)
    e.get_X_into(Xb)
    e.set_X(Xb)  # PGOAgent::setX: Nesterov restarts from the burnt-in iterate
    s0 = e.stats()[:, :10].copy()
    iters = 24
    for it in range(iters):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
    Xg = np.zeros(X0.size)
    e.get_X_into(Xg)
    sg = e.stats()[:, :10] - s0
    cpu = _cpu(g, aop, True)
    cpu.set_X(Xb)
    for _ in range(iters):
        cpu.iterate(threads=16)
    sc = cpu.stats()
    assert rel(Xg, cpu.get_X()) <= 1e-9
    assert np.array_equal(sg[:, 2:4], sc[:, 2:4])
    assert sg[:, 3].sum() >= 9 * sg[:, 2].sum()  # the CG regime: (nearly) every Run takes 10 tCG iterations
