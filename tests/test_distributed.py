"""Multi-rank exchange plan over torch.distributed (gloo, CPU, world_size 2 and 4).

Each rank computes its public-pose exchange plan with the native library (host-only
dpgo_rbcd_plan, the same code dpgo_rbcd_create uses), packs pose blocks of a known global X in
plan order, runs all_to_all_single exactly as bench.py does over RCCL, and checks that every rank
received the true poses of the neighbours its agents need."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, k, A, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dpgo_amd import hip as H
        import bench
        g = H.Graph.grid3d(k, seed=0)
        aop = g.grid_partition(A)
        ranks = bench.super_cube_ranks(A, world)
        send, recv = H.exchange_plan(g, aop, ranks, rank, world)
        rb = 20
        Xg = np.arange(g.n * rb, dtype=np.float64).reshape(g.n, rb) * 1e-3 + 7.0  # known pose blocks
        sbuf = torch.from_numpy(np.concatenate([Xg[s].ravel() for s in send]) if sum(len(s) for s in send)
                                else np.zeros(0))
        rbuf = torch.empty(sum(len(r) for r in recv) * rb, dtype=torch.float64)
        dist.all_to_all_single(rbuf, sbuf, [len(r) * rb for r in recv], [len(s) * rb for s in send])
        got = rbuf.numpy().reshape(-1, rb)
        want = np.concatenate([Xg[r] for r in recv]) if len(got) else np.zeros((0, rb))
        ok = np.array_equal(got, want)
        # every received pose is the endpoint of an edge into an agent this rank owns
        a = g.arrays()
        owner = ranks[aop]
        need = set()
        for i, j in zip(a["p1"], a["p2"]):
            if owner[i] == rank and owner[j] != rank:
                need.add(int(j))
            if owner[j] == rank and owner[i] != rank:
                need.add(int(i))
        ok = ok and need == set(int(x) for r in recv for x in r)
        q.put((rank, bool(ok), int(sum(len(r) for r in recv))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_exchange_plan_all_to_all(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 8, 4, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert all(ok for _, ok, _ in res), res
    assert all(n > 0 for _, _, n in res)


@pytest.mark.parametrize("world", [2, 4])
def test_bench_spawns_ranks_without_launcher(world):
    """`python bench.py --gpus N` with no WORLD_SIZE starts N rank processes itself (the parent makes no GPU call)
    and relays rank 0's single JSON line: the launch path the driver's SCALE run uses when it does not wrap the
    command in torchrun."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--spawn-selftest"],
                         env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d == {"world": world, "rank_sum": float(world * (world - 1) // 2), "spawned": True}


def test_super_cube_assignment():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    for world in (1, 2, 4, 8):
        r = bench.super_cube_ranks(4, world)
        assert sorted(np.bincount(r)) == [64 // world] * world
    # at 8 GPUs each rank owns one 2x2x2 super-cube
    r = bench.super_cube_ranks(4, 8)
    assert r[0] == r[1] == r[4] == r[5] == r[16] == r[17] == r[20] == r[21] == 0


def _worker_color(rank, world, port, k, A, q):
    """Per-colour halos: each colour's plan delivers the true poses over all_to_all_single; with two colours
    the colour plans partition the full plan (every received pose is read by exactly one colour)."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dpgo_amd import hip as H
        import bench
        g = H.Graph.grid3d(k, seed=0)
        aop = g.grid_partition(A)
        ranks = bench.super_cube_ranks(A, world)
        full_send, full_recv = H.exchange_plan(g, aop, ranks, rank, world)
        rb = 20
        Xg = np.arange(g.n * rb, dtype=np.float64).reshape(g.n, rb) * 1e-3 + 7.0
        ok, total = True, 0
        got_sets = []
        for c in range(2):
            send, recv = H.exchange_plan_color(g, aop, ranks, c, rank, world)
            sbuf = torch.from_numpy(np.concatenate([Xg[s].ravel() for s in send]) if sum(len(s) for s in send)
                                    else np.zeros(0))
            rbuf = torch.empty(sum(len(r) for r in recv) * rb, dtype=torch.float64)
            dist.all_to_all_single(rbuf, sbuf, [len(r) * rb for r in recv], [len(s) * rb for s in send])
            got = rbuf.numpy().reshape(-1, rb)
            want = np.concatenate([Xg[r] for r in recv]) if len(got) else np.zeros((0, rb))
            ok = ok and np.array_equal(got, want)
            for p in range(world):  # ascending ids, a subset of the full plan's
                ok = ok and list(recv[p]) == sorted(recv[p]) and set(recv[p]) <= set(full_recv[p])
                ok = ok and set(send[p]) <= set(full_send[p])
            got_sets.append(set(int(x) for r in recv for x in r))
            total += sum(len(r) for r in recv)
        ok = ok and not (got_sets[0] & got_sets[1])
        ok = ok and (got_sets[0] | got_sets[1]) == set(int(x) for r in full_recv for x in r)
        q.put((rank, bool(ok), total))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_exchange_plan_per_color(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_color, args=(r, world, port, 8, 4, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert all(ok for _, ok, _ in res), res
    assert all(n > 0 for _, _, n in res)
