"""Multi-rank RBCD engine on the GPU: 2 processes (both on the one visible GPU) exchange public
poses with all_to_all_single (gloo over host copies here; bench.py uses RCCL).  The result must be
bitwise the one-rank engine's (the per-agent arithmetic does not depend on how agents are batched or
where neighbour poses come from) and match the oracle's PGOAgent colour schedule.

The engine runs on the torch current stream (dpgo_rbcd_set_stream) and the exchange is issued on that
same stream with no explicit device synchronisation between pack, exchange and update: stream order
alone must make the halo consistent."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import dpgo_oracle as O
from tests._common import rel

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K, A, R, ITERS = 8, 2, 5, 6


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _params(H, accel, robust):
    return H.rbcd_params(r=R, acceleration=int(accel), robust_cost=H.ROBUST[robust], robust_opt_inner_iters=3)


def _worker(rank, world, port, accel, robust, q, halo="full"):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dpgo_amd import hip as H
        g = H.Graph.grid3d(K, seed=5)
        aop = g.grid_partition(A)
        ranks = (np.arange(A ** 3) * world // A ** 3).astype(np.int32)
        e = H.Rbcd(g, aop, ranks, rank, world, _params(H, accel, robust))
        X0 = g.chain_init(R, O.lifting_matrix(3, R))
        e.set_X(X0)
        dev = torch.device("cuda", 0)
        s = torch.cuda.Stream(dev)
        e.set_stream(s.cuda_stream)
        with torch.cuda.stream(s):
            send = torch.zeros(max(int(e.send_counts.sum()), 1), dtype=torch.float64, device=dev)
            recv = torch.zeros(max(int(e.recv_counts.sum()), 1), dtype=torch.float64, device=dev)
            rsplit = [int(x) for x in e.recv_counts]
            ssplit = [int(x) for x in e.send_counts]
            for it in range(ITERS):
                c = it % e.num_colors
                e.pre_exchange(c)
                if halo == "color":  # per-colour halo: only the poses colour c's agents read
                    rs_c = [int(x) for x in e.recv_counts_color[c]]
                    ss_c = [int(x) for x in e.send_counts_color[c]]
                    e.pack_color(c, send.data_ptr())
                    hs = send[:sum(ss_c)].cpu()
                    hr = torch.empty(sum(rs_c), dtype=torch.float64)
                    dist.all_to_all_single(hr, hs, rs_c, ss_c)
                    recv[:sum(rs_c)].copy_(hr)
                    e.update_color(c, recv.data_ptr())
                    continue
                e.pack(send.data_ptr())
                hs = send.cpu()  # D2H on the current stream: ordered after the pack
                hr = torch.empty_like(recv, device="cpu")
                dist.all_to_all_single(hr, hs, rsplit, ssplit)
                recv.copy_(hr)  # H2D on the current stream: ordered before the update
                e.update(c, recv.data_ptr())
        out = np.zeros(X0.size)
        e.get_X_into(out)
        rc, rd = e.status()
        q.put((rank, out, rc, rd))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("robust,halo", [("L2", "full"), ("GNC_TLS", "full"), ("L2", "color"), ("GNC_TLS", "color")])
@pytest.mark.parametrize("accel", [False, True])
def test_two_ranks_bitwise_one_rank_and_oracle(accel, robust, halo):
    """GNC_TLS: shared loop closures across the two ranks are reweighted by the lower-ID agent from
    the received neighbour poses (robust_opt_inner_iters = 3: reweightings at iterations 2 and 5).
    halo "color": per-colour halos (dpgo_rbcd_pack_color / update_color), bitwise the full halo's result."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, accel, robust, q, halo)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(2)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
    Xflat = outs[0][1] + outs[1][1]  # each rank wrote only its own poses into zeros
    from dpgo_amd import hip as H
    g = H.Graph.grid3d(K, seed=5)
    aop = g.grid_partition(A)
    X0 = g.chain_init(R, O.lifting_matrix(3, R))
    # one rank, same schedule: bitwise the same poses and status
    e1 = H.Rbcd(g, aop, np.zeros(A ** 3, np.int32), 0, 1, _params(H, accel, robust))
    e1.set_X(X0)
    for it in range(ITERS):
        c = it % e1.num_colors
        e1.pre_exchange(c)
        e1.update(c, None)
    X1 = np.zeros(X0.size)
    e1.get_X_into(X1)
    assert np.array_equal(Xflat, X1)
    rc1, rd1 = e1.status()
    ranks = (np.arange(A ** 3) * 2 // A ** 3)
    for a in range(A ** 3):
        rc, rd = outs[ranks[a]][2], outs[ranks[a]][3]
        assert rc[a] == rc1[a] and rd[a] == rd1[a]
    a = g.arrays()
    meas = O.Measurements(3, np.zeros(g.m, np.int64), np.zeros(g.m, np.int64), a["p1"].astype(np.int64),
                          a["p2"].astype(np.int64), a["R"], a["t"], a["kappa"], a["tau"], np.ones(g.m), g.n)
    Xo, _ = O.colour_rbcd(meas, aop, A ** 3, X0, ITERS, R, acceleration=accel, robust=robust,
                          robust_opt_inner_iters=3)
    assert rel(H.from_dev_layout(Xflat, R), Xo) <= 1e-9


# a non-cyclic schedule: the example's greedy pattern (one robot per round, colours in any order; None = the whole
# colour) over 12 iterations, reweighting every 3 (GNC_TLS, robust_opt_inner_iters = 3)
ORDER = [(0, 0), (0, 3), (1, None), (1, 1), (0, 5), (1, 6), (1, 2), (0, None), (0, 3), (1, 7), (0, 0), (1, 4)]


def _run_order(H, e, world, rank, halo="color"):
    """Drive `e` through ORDER; on several ranks each iteration's halo goes over gloo through host copies, ordered
    with the engine's launches by running both on one stream."""
    s = torch.cuda.Stream()
    e.set_stream(s.cuda_stream)
    with torch.cuda.stream(s):
        _run_order_on(H, e, world, halo)
    torch.cuda.synchronize()


def _run_order_on(H, e, world, halo):
    send = torch.zeros(max(int(e.send_counts.sum()), 1), dtype=torch.float64, device="cuda")
    recv = torch.zeros(max(int(e.recv_counts.sum()), 1), dtype=torch.float64, device="cuda")
    for c, sel in ORDER:
        mask = None
        if sel is not None:
            mask = np.zeros(A ** 3, np.int32)
            mask[sel] = 1
            c = int(e.color_of_agent[sel])
        e.set_selected(mask)
        e.pre_exchange(c)
        if world == 1:
            e.update(c, None)
            continue
        if halo == "color":
            rs_c = [int(x) for x in e.recv_counts_color[c]]
            ss_c = [int(x) for x in e.send_counts_color[c]]
            e.pack_color(c, send.data_ptr())
            hr = torch.empty(sum(rs_c), dtype=torch.float64)
            dist.all_to_all_single(hr, send[:sum(ss_c)].cpu(), rs_c, ss_c)
            recv[:sum(rs_c)].copy_(hr)
            e.update_color(c, recv.data_ptr())
        else:
            e.pack(send.data_ptr())
            hr = torch.empty(recv.shape, dtype=torch.float64)
            dist.all_to_all_single(hr, send.cpu(), [int(x) for x in e.recv_counts], [int(x) for x in e.send_counts])
            recv.copy_(hr)
            e.update(c, recv.data_ptr())
    e.set_selected(None)


def _order_worker(rank, world, port, accel, halo, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dpgo_amd import hip as H
        g = H.Graph.grid3d(K, seed=5)
        aop = g.grid_partition(A)
        ranks = (np.arange(A ** 3) * world // A ** 3).astype(np.int32)
        e = H.Rbcd(g, aop, ranks, rank, world, _params(H, accel, "GNC_TLS"))
        X0 = g.chain_init(R, O.lifting_matrix(3, R))
        e.set_X(X0)
        _run_order(H, e, world, rank, halo=halo)
        out = np.zeros(X0.size)
        e.get_X_into(out)
        rc, rd = e.status()
        q.put((rank, out, rc, rd))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("halo", ["color", "full"])
@pytest.mark.parametrize("accel", [False, True])
def test_robust_cost_any_colour_order_across_ranks(accel, halo):
    """GNC_TLS (PGOAgent::updateLoopClosuresWeights, src/PGOAgent.cpp:1174-1244) under a non-cyclic schedule -- the
    example's greedy single-robot rounds (examples/MultiRobotExample.cpp:243-256) mixed with whole colours in any
    order -- on two ranks: every reweighting reads the agent's own X and its neighborPoseDict (the poses it received
    when last selected), never the halo's vintage, so the result is bitwise the one-rank engine's with either halo."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_order_worker, args=(r, 2, port, accel, halo, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(2)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
    from dpgo_amd import hip as H
    g = H.Graph.grid3d(K, seed=5)
    aop = g.grid_partition(A)
    X0 = g.chain_init(R, O.lifting_matrix(3, R))
    e1 = H.Rbcd(g, aop, np.zeros(A ** 3, np.int32), 0, 1, _params(H, accel, "GNC_TLS"))
    e1.set_X(X0)
    _run_order(H, e1, 1, 0)
    X1 = np.zeros(X0.size)
    e1.get_X_into(X1)
    assert np.array_equal(outs[0][1] + outs[1][1], X1)
    rc1, rd1 = e1.status()
    ranks = (np.arange(A ** 3) * 2 // A ** 3)
    for a in range(A ** 3):
        assert outs[ranks[a]][2][a] == rc1[a] and outs[ranks[a]][3][a] == rd1[a]
    assert not np.array_equal(X1, X0)


# a partition with three or more colours: 8 agents over the poses at random (seeded), so the agent adjacency graph is
# far from the cube partition's bipartite one
def _aop_many(g):
    return np.random.default_rng(21).integers(0, A ** 3, g.n).astype(np.int32)


def _order_many(e):
    """12 iterations over the colours out of cyclic order; every third one the example's single-robot round (the
    lowest-id agent of that colour)."""
    C = e.num_colors
    cols = [(2 * it + it // 3) % C for it in range(12)]
    out = []
    for it, c in enumerate(cols):
        sel = None
        if it % 3 == 2:
            sel = int(np.nonzero(e.color_of_agent == c)[0][0])
        out.append((c, sel))
    return out


def _run_many(H, e, world):
    s = torch.cuda.Stream()
    e.set_stream(s.cuda_stream)
    send = recv = None
    with torch.cuda.stream(s):
        send = torch.zeros(max(int(e.send_counts.sum()), 1), dtype=torch.float64, device="cuda")
        recv = torch.zeros(max(int(e.recv_counts.sum()), 1), dtype=torch.float64, device="cuda")
        for c, sel in _order_many(e):
            mask = None
            if sel is not None:
                mask = np.zeros(A ** 3, np.int32)
                mask[sel] = 1
            e.set_selected(mask)
            e.pre_exchange(c)
            if world == 1:
                e.update(c, None)
                continue
            rs_c = [int(x) for x in e.recv_counts_color[c]]
            ss_c = [int(x) for x in e.send_counts_color[c]]
            e.pack_color(c, send.data_ptr())
            hr = torch.empty(sum(rs_c), dtype=torch.float64)
            dist.all_to_all_single(hr, send[:sum(ss_c)].cpu(), rs_c, ss_c)
            recv[:sum(rs_c)].copy_(hr)
            e.update_color(c, recv.data_ptr())
        e.set_selected(None)
    torch.cuda.synchronize()


def _many_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dpgo_amd import hip as H
        g = H.Graph.grid3d(K, seed=5)
        ranks = (np.arange(A ** 3) * world // A ** 3).astype(np.int32)
        e = H.Rbcd(g, _aop_many(g), ranks, rank, world, _params(H, True, "GNC_TLS"))
        X0 = g.chain_init(R, O.lifting_matrix(3, R))
        e.set_X(X0)
        _run_many(H, e, world)
        out = np.zeros(X0.size)
        e.get_X_into(out)
        q.put((rank, out, int(e.num_colors)))
    finally:
        dist.destroy_process_group()


def test_robust_cost_many_colours_non_cyclic_across_ranks():
    """GNC_TLS on a partition with >= 3 colours (the per-colour halo once had a full-halo fallback for
    this case), per-colour halos, colours out of cyclic order mixed with single-robot rounds, two ranks: bitwise the
    one-rank engine (every reweighting reads the agent's own X and its neighbour-pose dictionary)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_many_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(2)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
    from dpgo_amd import hip as H
    g = H.Graph.grid3d(K, seed=5)
    X0 = g.chain_init(R, O.lifting_matrix(3, R))
    e1 = H.Rbcd(g, _aop_many(g), np.zeros(A ** 3, np.int32), 0, 1, _params(H, True, "GNC_TLS"))
    assert e1.num_colors >= 3 and outs[0][2] == e1.num_colors
    e1.set_X(X0)
    _run_many(H, e1, 1)
    X1 = np.zeros(X0.size)
    e1.get_X_into(X1)
    assert np.array_equal(outs[0][1] + outs[1][1], X1)
    assert not np.array_equal(X1, X0)


def test_gnc_many_colours_cyclic_matches_oracle():
    """The same >= 3-colour random partition under the cyclic colour schedule, GNC_TLS reweighting every 3 iterations
    (the first before the last colour was ever selected: its dictionaries are empty, its shared edges keep their
    weights): the one-rank engine against the numpy PGOAgent restatement at 1e-9."""
    from dpgo_amd import hip as H
    g = H.Graph.grid3d(K, seed=5)
    aop = _aop_many(g)
    X0 = g.chain_init(R, O.lifting_matrix(3, R))
    e = H.Rbcd(g, aop, np.zeros(A ** 3, np.int32), 0, 1, _params(H, True, "GNC_TLS"))
    assert e.num_colors >= 3
    e.set_X(X0)
    iters = 9
    for it in range(iters):
        e.pre_exchange(it % e.num_colors)
        e.update(it % e.num_colors, None)
    X1 = np.zeros(X0.size)
    e.get_X_into(X1)
    a = g.arrays()
    meas = O.Measurements(3, np.zeros(g.m, np.int64), np.zeros(g.m, np.int64), a["p1"].astype(np.int64),
                          a["p2"].astype(np.int64), a["R"], a["t"], a["kappa"], a["tau"], np.ones(g.m), g.n)
    Xo, colors = O.colour_rbcd(meas, aop, A ** 3, X0, iters, R, acceleration=True, robust="GNC_TLS",
                               robust_opt_inner_iters=3)
    assert max(colors) + 1 == e.num_colors
    assert rel(H.from_dev_layout(X1, R), Xo) <= 1e-9
