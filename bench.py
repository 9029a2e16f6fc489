#!/usr/bin/env python3
"""bench.py -- RBCD throughput + X.Q SpMM HBM roofline on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[4] / SURVEY 8d C5): synthetic 3D grid, k^3 = 10^6 poses, r = 5,
64 agents (4 x 4 x 4 sub-cubes of 25^3 poses), Nesterov-accelerated RBCD (as
examples/MultiRobotExample.cpp) with the L2 cost, colour-class schedule (2 colours).
One *step* = one sweep over both colours = every agent updated once (64 agent updates, each an
RTR(1 outer, 10 tCG) solve as PGOAgent::updateX configures it) plus the public-pose exchange.

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "RBCD iters/sec + X·Q SpMM HBM GB/s, 1M-pose synth grid r=5, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def measured_traffic():
    """HBM bytes per launch of the edge-stream X.Q SpMM from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, produced by tools/pmc_traffic.py), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            t = json.load(f)
        t["source"] = os.path.relpath(files[-1], ROOT)
        return t
    except (OSError, ValueError):
        return None


def super_cube_ranks(A, world):
    """Agents -> ranks: 2x2x2 super-cubes of agents (8 groups), merged for world < 8."""
    ranks = np.zeros(A ** 3, np.int32)
    h = max(A // 2, 1)
    for az in range(A):
        for ay in range(A):
            for ax in range(A):
                sup = (ax // h) + 2 * ((ay // h) + 2 * (az // h))
                ranks[ax + A * (ay + A * az)] = (sup * world) // 8 if A >= 2 else 0
    return ranks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=100, help="grid side (k^3 poses)")
    ap.add_argument("--agents-per-axis", type=int, default=4)
    ap.add_argument("--r", type=int, default=5)
    ap.add_argument("--accel", type=int, default=1)
    ap.add_argument("--spmm-reps", type=int, default=20)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-sample-updates", type=int, default=40)
    ap.add_argument("--verify", type=int, default=0, help="central cost before/after (slow)")
    ap.add_argument("--robust", default="L2", choices=["L2", "GNC_TLS", "TLS", "Huber", "GM", "L1"],
                    help="robust cost (L2: throughput setting; GNC_TLS: the reference default, "
                         "reweighting every 30 iterations on the device)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from dpgo_amd import hip as H

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal on a one-GPU box: every rank on device 0 and the exchange over gloo through host
    # copies, since RCCL refuses two ranks on one device (DPGO_BENCH_ONE_DEVICE=1; never the default)
    one_device = os.environ.get("DPGO_BENCH_ONE_DEVICE") == "1"
    if one_device:
        local_rank = 0
    if world != args.gpus:
        world = max(world, 1)
    torch.cuda.set_device(local_rank)
    if world > 1:
        if one_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)

    t_setup = time.time()
    g = H.Graph.grid3d(args.k, seed=0)
    A = args.agents_per_axis
    aop = g.grid_partition(A)
    num_agents = A ** 3
    agent_rank = super_cube_ranks(A, world)
    params = H.rbcd_params(r=args.r, acceleration=args.accel, robust_cost=H.ROBUST[args.robust])
    eng = H.Rbcd(g, aop, agent_rank, rank, world, params)
    stream = torch.cuda.current_stream(dev)
    eng.set_stream(stream.cuda_stream)
    YLift = H.lifting_matrix(3, args.r)
    X0 = g.chain_init_dev_layout(args.r, YLift)
    eng.set_X(X0)
    send = torch.empty(max(int(eng.send_counts.sum()), 1), dtype=torch.float64, device=dev)
    recv = torch.empty(max(int(eng.recv_counts.sum()), 1), dtype=torch.float64, device=dev)
    in_splits = [int(x) for x in eng.send_counts]
    out_splits = [int(x) for x in eng.recv_counts]
    setup_s = time.time() - t_setup

    def step():
        for c in range(eng.num_colors):
            eng.pre_exchange(c)
            if world > 1:
                eng.pack(send.data_ptr())
                if one_device:
                    recv_h = torch.empty(recv.shape, dtype=recv.dtype)
                    dist.all_to_all_single(recv_h, send.cpu(), out_splits, in_splits)
                    recv.copy_(recv_h)
                else:
                    dist.all_to_all_single(recv, send, out_splits, in_splits)
            eng.update(c, recv.data_ptr() if world > 1 else None)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if one_device else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # ---- roofline of the X.Q SpMM over one colour class (HIP events on the engine stream)
    fmt_bytes, spmm_ms = eng.bench_spmm(0, args.spmm_reps)
    bsr_bytes, _ = eng.spmm_bytes(0)
    achieved = bsr_bytes / (spmm_ms * 1e-3) / 1e9 if spmm_ms > 0 else 0.0
    hvp_ms = eng.bench_hvp(0, args.spmm_reps)
    traffic = measured_traffic()

    agent_updates = num_agents * args.steps
    value = agent_updates / elapsed
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "RBCD agent-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (repo-defined grid3d, SplitMix64 seed 0; no reference data at this size)",
        "config": {"workload": f"grid3d k={args.k} ({args.k ** 3} poses), r={args.r}, "
                               f"{num_agents} agents ({A}^3 sub-cubes), Nesterov={bool(args.accel)}, "
                               f"{args.robust} cost, colour schedule ({eng.num_colors} colours), "
                               f"RTR 1x10 tCG, block-Jacobi precond",
                   "poses": g.n, "edges": g.m, "agents": num_agents,
                   "parallelism": f"agents over {world} GPU(s), RCCL all_to_all halo"},
        "rounds_per_s": args.steps / elapsed,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic["traffic_bytes_per_launch"] if traffic else None,
                     "kernel": "k_spmm<5,4,MODE_XQ,edge-stream> (X.Q over colour class 0 on rank 0)",
                     "algorithmic_bytes_per_launch": bsr_bytes,
                     "algorithmic_bytes_definition": "SURVEY 8d B_spmm = nnzb(b^2 8 + 4) + (n+1) 4 + 2 r b n 8",
                     "avg_launch_ms": spmm_ms,
                     "format_bytes_per_launch": fmt_bytes,
                     "format_GBps": fmt_bytes / (spmm_ms * 1e-3) / 1e9 if spmm_ms > 0 else 0.0,
                     "traffic_source": traffic["source"] if traffic else None},
        "hvp": {"per_s": 1e3 / hvp_ms if hvp_ms > 0 else 0.0, "avg_launch_ms": hvp_ms,
                "agents": int(eng.agents_per_color[0]),
                "what": "Riemannian HVP (EucHessianEta + EucHvToHv, tangent-projected) over colour class 0"},
        "setup_s": setup_s,
    }
    if args.verify:
        # central cost 1/2 tr(X Q X^T) of the whole graph before and after (outside the timed region):
        # the schedule is deterministic, so the final cost must not depend on the number of ranks
        Xf = np.zeros(X0.size)
        eng.get_X_into(Xf)
        if world > 1:
            tx = torch.from_numpy(Xf) if one_device else torch.from_numpy(Xf).to(dev)
            dist.all_reduce(tx)
            Xf = tx.cpu().numpy()
        if rank == 0:
            import scipy.sparse as sp
            rp, col, blk = g.laplacian_bsr()
            b = g.d + 1
            Q = sp.bsr_matrix((np.ascontiguousarray(blk.reshape(-1, b, b).transpose(0, 2, 1)), col, rp),
                              shape=(g.n * b, g.n * b)).tocsr()

            def central(flat):
                X = H.from_dev_layout(flat, args.r)
                return 0.5 * float(np.sum(np.asarray(Q @ X.T).T * X))
            out["verify"] = {"f_init": central(X0), "f_final": central(Xf),
                             "steps_run": args.warmup + args.steps}
    if rank == 0 and world == 1 and args.cpu_baseline:
        try:
            from oracle import cpu_port
            out["cpu_baseline"] = cpu_port.baseline(g, aop, X0, args.r, bool(args.accel),
                                                    num_agents, args.cpu_sample_updates)
        except Exception as exc:  # reported, never silently replaced
            out["cpu_baseline"] = {"error": repr(exc)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
