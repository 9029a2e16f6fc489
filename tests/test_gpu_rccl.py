"""Native halo exchange through the library's own RCCL calls (dpgo_rbcd_comm_init / dpgo_rbcd_exchange,
examples/MultiRobotExample.cpp:188-213), without torch.distributed.

On a one-GPU box only the one-rank communicator can be built (RCCL refuses two ranks on one device):
that case checks RCCL loading, communicator creation, the grouped (empty) exchange on the engine
stream and that the update is unchanged.  The two-rank case (one device per rank, unique id shared
through a queue) runs where two GPUs are visible and must be bitwise the one-rank engine."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K, A, R, ITERS = 8, 2, 5, 8


@pytest.fixture(scope="module")
def hip():
    from dpgo_amd import hip as H
    assert H.device_count() >= 1
    return H


def _run(H, ranks, rank, world, native, uid=None):
    g = H.Graph.grid3d(K, seed=5)
    aop = g.grid_partition(A)
    e = H.Rbcd(g, aop, ranks, rank, world, H.rbcd_params(r=R, acceleration=1))
    X0 = g.chain_init_dev_layout(R, H.lifting_matrix(3, R))
    e.set_X(X0)
    if native:
        e.comm_init(uid)
    for it in range(ITERS):
        c = it % e.num_colors
        e.pre_exchange(c)
        e.update(c, e.exchange() if native else None)
    X = np.zeros(X0.size)
    e.get_X_into(X)
    return X


def test_native_exchange_one_rank(hip):
    ranks = np.zeros(A ** 3, np.int32)
    uid = hip.rccl_unique_id()
    assert len(uid) == 128
    X_native = _run(hip, ranks, 0, 1, True, uid)
    X_plain = _run(hip, ranks, 0, 1, False)
    assert np.array_equal(X_native, X_plain)


def _rank_worker(rank, world, uid, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["HIP_VISIBLE_DEVICES"] = str(rank)
    from dpgo_amd import hip as H
    ranks = (np.arange(A ** 3) * world // A ** 3).astype(np.int32)
    q.put((rank, _run(H, ranks, rank, world, True, uid)))


def test_native_exchange_two_ranks(hip):
    if hip.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = hip.rccl_unique_id()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, uid, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    X1 = _run(hip, np.zeros(A ** 3, np.int32), 0, 1, False)
    assert np.array_equal(outs[0] + outs[1], X1)
