"""Multi-rank RBCD engine on the GPU: 2 processes (both on the one visible GPU) exchange public
poses with all_to_all_single (gloo over host copies here; bench.py uses RCCL), and the result must
equal the oracle's PGOAgent colour schedule."""
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


def _worker(rank, world, port, accel, robust, q):
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
        e = H.Rbcd(g, aop, ranks, rank, world, H.rbcd_params(r=R, acceleration=int(accel),
                                                             robust_cost=H.ROBUST[robust], robust_opt_inner_iters=3))
        X0 = g.chain_init(R, O.lifting_matrix(3, R))
        e.set_X(X0)
        dev = torch.device("cuda", 0)
        send = torch.zeros(max(int(e.send_counts.sum()), 1), dtype=torch.float64, device=dev)
        recv = torch.zeros(max(int(e.recv_counts.sum()), 1), dtype=torch.float64, device=dev)
        for it in range(ITERS):
            c = it % e.num_colors
            e.pre_exchange(c)
            e.pack(send.data_ptr())
            torch.cuda.synchronize()
            hs, hr = send.cpu(), torch.empty_like(recv, device="cpu")
            dist.all_to_all_single(hr, hs, [int(x) for x in e.recv_counts], [int(x) for x in e.send_counts])
            recv.copy_(hr)
            torch.cuda.synchronize()
            e.update(c, recv.data_ptr())
        out = np.zeros(X0.size)
        e.get_X_into(out)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("robust", ["L2", "GNC_TLS"])
@pytest.mark.parametrize("accel", [False, True])
def test_two_ranks_match_oracle(accel, robust):
    """GNC_TLS: shared loop closures across the two ranks are reweighted by the lower-ID agent from
    the received neighbour poses (robust_opt_inner_iters = 3: reweightings at iterations 2 and 5)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, accel, robust, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    Xflat = outs[0][1] + outs[1][1]  # each rank wrote only its own poses into zeros
    from dpgo_amd import hip as H
    g = H.Graph.grid3d(K, seed=5)
    a = g.arrays()
    meas = O.Measurements(3, np.zeros(g.m, np.int64), np.zeros(g.m, np.int64), a["p1"].astype(np.int64),
                          a["p2"].astype(np.int64), a["R"], a["t"], a["kappa"], a["tau"], np.ones(g.m), g.n)
    X0 = g.chain_init(R, O.lifting_matrix(3, R))
    Xo, _ = O.colour_rbcd(meas, g.grid_partition(A), A ** 3, X0, ITERS, R, acceleration=accel, robust=robust,
                          robust_opt_inner_iters=3)
    assert rel(H.from_dev_layout(Xflat, R), Xo) <= 1e-9
