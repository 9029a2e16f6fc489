#!/usr/bin/env python3
"""bench.py -- RBCD throughput + X.Q SpMM HBM roofline on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[4] / SURVEY 8d C5): synthetic 3D grid, k^3 = 10^6 poses, r = 5,
64 agents (4 x 4 x 4 sub-cubes of 25^3 poses), Nesterov-accelerated RBCD (as
examples/MultiRobotExample.cpp) with the L2 cost, colour-class schedule (2 colours).
One *step* = one sweep over both colours = every agent updated once (64 agent updates, each an
RTR(1 outer, 10 tCG) solve as PGOAgent::updateX configures it, plus the agent status) plus the
public-pose exchange.

Initial X (`--init`): the multi-robot initialisation (every agent's local chordal initialisation aligned
into one frame over the shared loop closures, PCG on the GPU).  `--burnin` untimed steps then bring the
solve into its converging phase, where every update's truncated CG runs its 10 iterations (the RTR
inner loop: Hessian-vector products, preconditioner, CG recurrences); the iterate re-enters set_X
(PGOAgent::setX: Nesterov restarts from it), then `--warmup` untimed steps and the timed steps.

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
# HIP hardware queues per process (HIP's default: 4), read when the runtime initialises: a stream takes its queue at
# its first command, and a run with N > 1 has more live streams than 4 -- the launch stream, one second-half stream per
# colour problem (TUNE_SPLIT_STREAMS), the halo side stream, the collective's stream.  Two of them sharing a queue
# serialise (the 8-GPU share measured 1.38 instead of 1.10 ms/step with its two halves on one queue).
# Spawned ranks inherit the value.  Not for the one-device rehearsal (DPGO_BENCH_ONE_DEVICE=1): N processes x 8
# queues on one device oversubscribe its hardware queue slots (k = 48 rehearsal: N = 4 4.5 -> 43 ms/step, N = 8 23.6 ->
# 79, profiles/r06fin_spawn_rehearsal_q8_*); one process per device, as the driver's runs are, holds 8 on its own device.
try:
    _hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
except ValueError:
    _hwq = 4
if _hwq < 8 and os.environ.get("DPGO_BENCH_ONE_DEVICE") != "1":
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

METRIC = "RBCD iters/sec + X·Q SpMM HBM GB/s, 1M-pose synth grid r=5, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
STATS = ["calls", "early", "runs", "tcg_iters", "NEGCURVTURE", "EXCREGION", "LCON", "SCON", "MAXITER",
         "gave_up", "cg_steps", "implicit", "first_full"]


def measured_traffic(build_id):
    """HBM bytes per launch from a committed PMC summary of THIS library build (profiles/*_pmc_traffic.json, written
    by tools/pmc_step.py, which records the profiled library's dpgo_hip_build_id): the newest file whose build id
    equals the loaded library's.  (None, reason) when there is none -- a summary of other kernels is never reported
    as this build's traffic."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    stale = []
    for path in reversed(files):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if t.get("build_id") == build_id and t.get("kernels"):
            t["source"] = os.path.relpath(path, ROOT)
            return t, None
        stale.append(os.path.relpath(path, ROOT))
    return None, ("no PMC summary of this build (" + build_id[:12] + "); newest of another build: " +
                  (stale[0] if stale else "none"))


def fp64_peak():
    """The fp64 ceilings measured on this pool (tools/fp64_peak.hip), newest committed profiles/*_fp64_peak.json."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_fp64_peak.json")))
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


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`python bench.py --gpus N` with no WORLD_SIZE in the environment: start N rank processes of this same
    command (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1) and relay rank 0's JSON line.
    This parent makes no GPU call (it does not even import torch) and starts the ranks as child processes, so the
    command runs the same whether or not a launcher wraps it."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, DPGO_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      text=True, start_new_session=True))
    import threading

    def watchdog():  # a rank that fails leaves the others blocked in a collective: end the whole job
        while procs[0].poll() is None:
            if any(p.poll() not in (None, 0) for p in procs[1:]):
                for p in procs:
                    if p.poll() is None:
                        os.killpg(p.pid, signal.SIGKILL)
                return
            time.sleep(1.0)
    threading.Thread(target=watchdog, daemon=True).start()
    line = None
    for ln in procs[0].stdout:  # rank 0 prints exactly one JSON line; anything else goes to stderr
        if ln.lstrip().startswith("{"):
            line = ln.strip()
        else:
            sys.stderr.write(ln)
    rcs = [p.wait() for p in procs[:1]]
    # rank 0 is done: the others have passed the final barrier or failed; never leave one behind
    for p in procs[1:]:
        try:
            rcs.append(p.wait(timeout=120))
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            rcs.append(p.wait())
    bad = [(r, rc) for r, rc in enumerate(rcs) if rc != 0]
    if bad or line is None:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
        raise SystemExit(f"bench.py: spawned ranks failed {bad or 'without a JSON line'}")
    print(line, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--init", default="distributed", choices=["distributed", "chordal", "odometry"],
                    help="initial X: distributed = every agent's local chordal initialisation aligned into one "
                         "frame over the shared loop closures (PGOAgent::localInitialization + "
                         "initializeInGlobalFrame; PCG on the GPU); chordal = one chordalInitialization of the "
                         "whole graph (examples/MultiRobotExample.cpp:158; its unconstrained rotation relaxation "
                         "shrinks below fp64 resolution far from the anchor on a 10^6-pose noisy grid); odometry "
                         "= the odometry chain")
    ap.add_argument("--burnin", type=int, default=300,
                    help="untimed steps from the initialisation before the timed run's set_X: from the distributed "
                         "init, ~200 steps bring every agent into the regime where tCG runs its 10 iterations")
    ap.add_argument("--k", type=int, default=100, help="grid side (k^3 poses)")
    ap.add_argument("--agents-per-axis", type=int, default=4)
    ap.add_argument("--r", type=int, default=5)
    ap.add_argument("--accel", type=int, default=1)
    ap.add_argument("--spmm-reps", type=int, default=20)
    ap.add_argument("--kernel-timing", type=int, default=4,
                    help="HIP events around every k-th in-step X.Q launch of each mode (0 off; 1 every launch: an "
                         "event pair costs a dispatch gap, +1.2%% ms/step at 1M and +7.5%% at the 125k share; "
                         "every 4th: +0.3%% / +2%%)")
    ap.add_argument("--exchange", default="torch", choices=["torch", "native"],
                    help="N > 1 halo exchange: torch.distributed all_to_all_single (RCCL), or the library's own "
                         "RCCL group send/recv (dpgo_rbcd_comm_init / dpgo_rbcd_exchange)")
    ap.add_argument("--halo", default="color", choices=["color", "full"],
                    help="N > 1: color = per-colour halo (only the poses the selected colour's agents read, "
                         "dpgo_rbcd_pack_color / update_color); full = every public pose every iteration")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--boundary-leg", type=int, default=1,
                    help="also time the same steps from the odometry chain initialisation (round 1's regime: every "
                         "tCG ends at its first step on the trust-region boundary), reported as boundary_regime")
    ap.add_argument("--certify-iters", type=int, default=0,
                    help="> 0: certified gap of the final iterate over the whole graph (dpgo_graph_certify_ex: "
                         "thick-restarted Lanczos steps with X's near-null block locked, a lower bound on lambda_min "
                         "of the central certificate matrix, SE(d) rounding, both costs)")
    ap.add_argument("--pmc-calib-mb", type=int, default=0,
                    help="tools/pmc_step.py: one device copy of this many MiB before the timed region (a launch of "
                         "known read/write bytes for the FETCH_SIZE calibration)")
    ap.add_argument("--precon", default="block_jacobi", choices=["block_jacobi", "exact"],
                    help="block_jacobi: per-pose (Q_jj + 0.1 I)^-1 (throughput setting, CPU baseline too); exact: the "
                         "reference's factor of Q + 0.1 I (nested-dissection tree on the host once per pattern, "
                         "supernodal numeric factorisation and panel sweeps on the device)")
    ap.add_argument("--robust", default="L2", choices=["L2", "GNC_TLS", "TLS", "Huber", "GM", "L1"],
                    help="robust cost (L2: throughput setting; GNC_TLS: the reference default, "
                         "reweighting every 30 iterations on the device)")
    ap.add_argument("--exact-leg", type=int, default=1,
                    help="one GPU: also time the reference's default configuration (GNC_TLS + the exact factor of "
                         "Q + 0.1 I, refactorised on the device after every reweighting) on the C4 grid, reported as "
                         "exact_leg with its factor TFLOP/s, sweep roofline and the CPU port's exact-mode baseline")
    ap.add_argument("--exact-leg-k", type=int, default=48)
    ap.add_argument("--exact-leg-burnin", type=int, default=60)
    ap.add_argument("--spawn-selftest", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)  # before torch is imported: this process never touches the GPU

    import torch
    import torch.distributed as dist
    if args.spawn_selftest:  # the launch path alone, on the CPU (tests/test_distributed.py): gloo, no device
        dist.init_process_group("gloo")
        t = torch.tensor([float(dist.get_rank())])
        dist.all_reduce(t)
        if dist.get_rank() == 0:
            print(json.dumps({"world": dist.get_world_size(), "rank_sum": float(t.item()),
                              "spawned": os.environ.get("DPGO_BENCH_SPAWNED") == "1"}), flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return None
    from dpgo_amd import hip as H

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal on a one-GPU box: every rank on device 0 and the exchange over gloo through host
    # copies, since RCCL refuses two ranks on one device (DPGO_BENCH_ONE_DEVICE=1; never the default)
    one_device = os.environ.get("DPGO_BENCH_ONE_DEVICE") == "1"
    if one_device:
        local_rank = 0
    world = max(world, 1)
    if world != args.gpus:  # the driver's SCALE runs must measure the world they name
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
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
    params = H.rbcd_params(r=args.r, acceleration=args.accel, robust_cost=H.ROBUST[args.robust],
                           precon=H.PRECON_EXACT if args.precon == "exact" else H.PRECON_BLOCK_JACOBI)
    eng = H.Rbcd(g, aop, agent_rank, rank, world, params)
    # every engine launch and the exchange run on one dedicated stream (stream order = halo order)
    stream = torch.cuda.Stream(dev)
    eng.set_stream(stream.cuda_stream)
    YLift = H.lifting_matrix(3, args.r)
    t_init = time.time()
    init_info = {"kind": args.init}
    if args.init == "distributed":
        X0, it, rr = g.distributed_init(aop, args.r, YLift, gpu=True, rtol=1e-12, max_iters=50000, dev_layout=True)
        init_info.update(pcg_iterations=it, pcg_relres=rr)
    elif args.init == "chordal":
        X0, it, rr = g.chordal_init_gpu(args.r, YLift, rtol=1e-10, max_iters=50000, dev_layout=True)
        init_info.update(pcg_iterations=it, pcg_relres=rr)
    else:
        X0 = g.chain_init_dev_layout(args.r, YLift)
    init_info["seconds"] = time.time() - t_init
    eng.set_X(X0)
    send = torch.empty(max(int(eng.send_counts.sum()), 1), dtype=torch.float64, device=dev)
    recv = torch.empty(max(int(eng.recv_counts.sum()), 1), dtype=torch.float64, device=dev)
    in_splits = [int(x) for x in eng.send_counts]
    out_splits = [int(x) for x in eng.recv_counts]
    setup_s = time.time() - t_setup

    native = args.exchange == "native" and world > 1
    if native:
        uid = [H.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(uid[0])

    def exchange():
        if world == 1:
            return None
        if native:
            return eng.exchange()
        eng.pack(send.data_ptr())
        if one_device:
            recv_h = torch.empty(recv.shape, dtype=recv.dtype)
            dist.all_to_all_single(recv_h, send.cpu(), out_splits, in_splits)
            recv.copy_(recv_h)
        else:
            dist.all_to_all_single(recv, send, out_splits, in_splits)
        return recv.data_ptr()

    # per-colour halos: splits and views per colour (the buffers are sized by the full plan)
    c_in = [[int(x) for x in v] for v in eng.send_counts_color]
    c_out = [[int(x) for x in v] for v in eng.recv_counts_color]

    def exchange_color(c):
        if world == 1:
            return None
        if native:
            return eng.exchange_color(c)
        eng.pack_color(c, send.data_ptr())
        ns, nr = sum(c_in[c]), sum(c_out[c])
        if one_device:
            recv_h = torch.empty(nr, dtype=recv.dtype)
            dist.all_to_all_single(recv_h, send[:ns].cpu(), c_out[c], c_in[c])
            recv[:nr].copy_(recv_h)
        else:
            dist.all_to_all_single(recv[:nr], send[:ns], c_out[c], c_in[c])
        return recv.data_ptr()

    def step():
        for c in range(eng.num_colors):
            eng.pre_exchange(c)
            if args.halo == "color":
                eng.update_color(c, exchange_color(c))
            else:
                eng.update(c, exchange())

    def central():
        """Central cost and |RieGrad| of the whole graph (examples/MultiRobotExample.cpp:229-235)."""
        f, gn = eng.central_eval(exchange())
        if world > 1:
            t = torch.tensor(np.concatenate([[f], gn]), dtype=torch.float64, device="cpu" if one_device else dev)
            dist.all_reduce(t)
            v = t.cpu().numpy()
            f, gn = float(v[0]), v[1:]
        return f, float(np.sqrt(np.sum(gn)))

    def like_for_like(X_start, Xc, stc, iters):
        """The GPU replays the host baseline's iterations from the same start: same solver decisions, same
        tCG work, same iterate."""
        with torch.cuda.stream(stream):
            eng.set_X(X_start)
            sg0 = eng.stats().copy()
            for it in range(iters):
                eng.pre_exchange(it % eng.num_colors)
                eng.update(it % eng.num_colors, None)
            sg = eng.stats() - sg0
            Xg = np.zeros(X_start.size)
            eng.get_X_into(Xg)

        def hist(st):
            t = st.sum(axis=0)
            return {"updates": int(t[0]), "runs": int(t[2]), "tcg_iters": int(t[3]),
                    "exits": dict(zip(STATS[4:9], (int(v) for v in t[4:9])))}
        return {"iterations": iters, "cpu": hist(stc), "gpu": hist(sg[:, :10]),
                "same_counters_per_agent": bool(np.array_equal(stc[:, :10], sg[:, :10])),
                "X_rel_diff": float(np.linalg.norm(Xg - Xc) / np.linalg.norm(Xc))}

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    with torch.cuda.stream(stream):
        for _ in range(args.burnin):
            step()
        if args.burnin:
            Xb = np.zeros(X0.size)
            eng.get_X_into(Xb)
            if world > 1:
                tx = torch.from_numpy(Xb) if one_device else torch.from_numpy(Xb).to(dev)
                dist.all_reduce(tx)  # every rank wrote only its own poses into zeros
                Xb = tx.cpu().numpy()
            eng.set_X(Xb)  # PGOAgent::setX: Nesterov restarts from the burnt-in iterate
        X_start = None
        if rank == 0 and world == 1 and args.cpu_baseline and args.robust in ("L2", "GNC_TLS"):
            X_start = np.zeros(X0.size)
            eng.get_X_into(X_start)
        f_start, gn_start = central()
        for _ in range(args.warmup):
            step()
        if args.pmc_calib_mb:
            cx = torch.ones(args.pmc_calib_mb * (1 << 17), dtype=torch.float64, device=dev)
            torch.empty_like(cx).copy_(cx)
        st0 = eng.stats().copy()
        b0, _ = eng.bytes()
        fc0 = sum(eng.exact_factor_info(c)["factor_count"] for c in range(eng.num_colors)) if args.precon == "exact" else 0
        eng.kernel_times()  # drop anything recorded so far
        eng.set_kernel_timing(args.kernel_timing)
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        sync()
        elapsed = time.perf_counter() - t0
        eng.set_kernel_timing(0)
        refactor_in_timed = (sum(eng.exact_factor_info(c)["factor_count"] for c in range(eng.num_colors)) - fc0
                             if args.precon == "exact" else 0)
        ktimes = eng.kernel_times(batch_equiv=True)
        st1 = eng.stats().copy()
        b1, _ = eng.bytes()
        f_end, gn_end = central()
    ready, owned = eng.ready_votes()
    if world > 1:
        tv = torch.tensor([ready, owned], dtype=torch.int64, device="cpu" if one_device else dev)
        dist.all_reduce(tv)
        ready, owned = (int(v) for v in tv.cpu().numpy())
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if one_device else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # ---- solver statistics over the timed region (all ranks)
    dst = (st1 - st0).astype(np.int64)
    sums = dst.sum(axis=0)
    if world > 1:
        ts = torch.tensor(sums, dtype=torch.int64, device="cpu" if one_device else dev)
        dist.all_reduce(ts)
        sums = ts.cpu().numpy()
    tot = dict(zip(STATS, (int(v) for v in sums)))
    upd = max(tot["calls"], 1)
    tcg = {"per_update": {"runs": tot["runs"] / upd, "tcg_iters": tot["tcg_iters"] / upd,
                          "cg_steps": tot["cg_steps"] / upd, "early_return": tot["early"] / upd},
           "exits": {k: tot[k] for k in ("NEGCURVTURE", "EXCREGION", "LCON", "SCON", "MAXITER")},
           "first_step_boundary_runs": tot["implicit"], "runs": tot["runs"], "updates": tot["calls"],
           "gave_up": tot["gave_up"]}

    # ---- roofline: the in-step X.Q launches timed with HIP events on the engine stream; bytes per launch =
    # the SURVEY 8d model over every agent of the colour (both colours' launches averaged)
    mb = [eng.mode_bytes(c) for c in range(eng.num_colors)]
    step_ms = 1e3 * elapsed / args.steps
    # the committed PMC figures are per launch of the 1M-pose, 64-agent, one-GPU workload only
    traffic, traffic_note = (measured_traffic(H.build_id()) if (args.k == 100 and A == 4 and world == 1)
                             else (None, "PMC summaries cover the one-GPU 1M-pose, 64-agent workload only"))
    per_mode = {}
    for m, v in ktimes.items():
        # per full-batch launch equivalent: a half-batch launch of the split merged tCG (small batches, tuning
        # key 10) moves about half the colour's bytes and counts 0.5 (dpgo_rbcd_kernel_times_ex)
        avg = v[0] / max(v[2], 1e-12)
        byt = float(np.mean([x.get(m, 0.0) for x in mb]))
        e = {"ms_total": v[0], "launches": v[1], "batch_equivalents": v[2], "avg_ms": avg,
             "algorithmic_bytes_per_launch": byt, "GBps": byt / (avg * 1e-3) / 1e9 if avg > 0 else 0.0}
        e["frac"] = e["GBps"] / HBM_PEAK_GBS
        tb = (traffic or {}).get("kernels", {}).get(m, {}).get("traffic_bytes_per_launch")
        if tb:
            e["traffic_bytes_per_launch"] = tb
            e["traffic_GBps"] = tb / (avg * 1e-3) / 1e9
        per_mode[m] = e
    dominant = max(per_mode, key=lambda m: per_mode[m]["ms_total"]) if per_mode else None
    dm = per_mode.get(dominant, {})
    step_bytes = (b1 - b0) / args.steps
    if world > 1:
        tb = torch.tensor([step_bytes], dtype=torch.float64, device="cpu" if one_device else dev)
        dist.all_reduce(tb)
        step_bytes = float(tb.item())
    # the events time every k-th launch of each mode (--kernel-timing k): per-step SpMM time ~ k x the sample's
    spmm_ms_step = max(args.kernel_timing, 1) * sum(v["ms_total"] for v in per_mode.values()) / args.steps

    # ---- what the multi-GPU run actually was (the driver's SCALE runs verify themselves): the collective's world as
    # the communicator reports it, ranks sharing a device, and per colour this rank's halo bytes and exchange time
    comm = {"world_size": world, "gpus_arg": args.gpus, "backend": dist.get_backend() if world > 1 else None,
            "torch_world": dist.get_world_size() if world > 1 else 1,
            "hip_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "0")),
            "launcher": ("bench.py spawn (one child process per rank)" if os.environ.get("DPGO_BENCH_SPAWNED")
                         else "external (torchrun or equivalent)" if world > 1 else None)}
    if native:
        comm["rccl_comm_count"], comm["rccl_comm_rank"] = eng.comm_info()
        if comm["rccl_comm_count"] != world:
            raise SystemExit(f"bench.py: RCCL communicator has {comm['rccl_comm_count']} ranks, WORLD_SIZE={world}")
    if world > 1:
        import socket
        who = [None] * world
        dist.all_gather_object(who, (socket.gethostname(), torch.cuda.current_device()))
        comm["ranks_per_device"] = max(who.count(w) for w in who)
        comm["devices"] = len(set(who))
        xt = []
        with torch.cuda.stream(stream):
            for c in range(eng.num_colors):
                reps = 10
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                sync()
                ev0.record(stream)
                for _ in range(reps):
                    if args.halo == "color":
                        exchange_color(c)
                    else:
                        exchange()
                ev1.record(stream)
                sync()
                xt.append(ev0.elapsed_time(ev1) / reps)
        tx = torch.tensor(xt, dtype=torch.float64, device="cpu" if one_device else dev)
        dist.all_reduce(tx, op=dist.ReduceOp.MAX)
        comm["exchange_per_color"] = [
            {"color": c, "bytes_sent_this_rank": 8.0 * (sum(c_in[c]) if args.halo == "color" else int(eng.send_counts.sum())),
             "bytes_received_this_rank": 8.0 * (sum(c_out[c]) if args.halo == "color" else int(eng.recv_counts.sum())),
             "ms_max_over_ranks": float(tx[c]), "what": "pack + all_to_all (or the RCCL group) on the engine stream, "
                                                          "mean of 10, outside the timed steps"}
            for c in range(eng.num_colors)]
    else:
        comm["ranks_per_device"] = 1
        comm["devices"] = 1

    # ---- the standalone X.Q SpMM over one colour class (the metric's "X.Q SpMM HBM GB/s")
    fmt_bytes, spmm_ms = eng.bench_spmm(0, args.spmm_reps)
    bsr_bytes, _ = eng.spmm_bytes(0)
    hvp_ms = eng.bench_hvp(0, args.spmm_reps)

    agent_updates = num_agents * args.steps
    value = agent_updates / elapsed
    if world == 1:
        par = f"1 GPU, all {num_agents} agents on it (no exchange)"
    elif one_device:
        par = f"{world} ranks on ONE device (rehearsal), halo all_to_all over gloo through host copies"
    elif native:
        par = (f"agents over {world} GPUs (2x2x2 super-cubes), {args.halo} halo by the library's RCCL group "
               f"send/recv over xGMI")
    else:
        par = f"agents over {world} GPUs (2x2x2 super-cubes), {args.halo} halo all_to_all_single over RCCL/xGMI"
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "RBCD agent-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (repo-defined grid3d, SplitMix64 seed 0; no reference data at this size)",
        "config": {"workload": f"grid3d k={args.k} ({args.k ** 3} poses), r={args.r}, "
                               f"{num_agents} agents ({A}^3 sub-cubes), Nesterov={bool(args.accel)}, "
                               f"{args.robust} cost, colour schedule ({eng.num_colors} colours), "
                               f"RTR 1x10 tCG, {args.precon} precond, agent status on, {args.init} init, "
                               f"burn-in {args.burnin} steps",
                   "poses": g.n, "edges": g.m, "agents": num_agents, "parallelism": par},
        "rounds_per_s": args.steps / elapsed,
        "roofline": {"bound": "hbm", "achieved": dm.get("GBps", 0.0), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": dm.get("frac", 0.0),
                     "traffic": dm.get("traffic_bytes_per_launch"),
                     "kernel": f"k_spmm<5,4,MODE_{dominant},edge-stream>: the in-step kernel with the most time "
                               "(every agent of a colour per launch)",
                     "algorithmic_bytes_per_launch": dm.get("algorithmic_bytes_per_launch"),
                     "algorithmic_bytes_definition": "SURVEY 8d per agent: Q as b x b blocks (n + 2 m_in)(b^2 8 + 4) "
                                                     "+ (n+1) 4 + pose vector 160 n, + per mode: HESS eta 160 n + S "
                                                     "48 n + out 160 n; EVAL_TCG S 48 n + Minv 80 n + out 160 n + G; "
                                                     "QF half pass + S; F half pass + G (dpgo_rbcd_mode_bytes)",
                     "avg_launch_ms": dm.get("avg_ms"),
                     "launches_timed": dm.get("launches", 0),
                     "timing_sample_period": args.kernel_timing,
                     "traffic_frac": (dm["traffic_GBps"] / HBM_PEAK_GBS) if "traffic_GBps" in dm else None,
                     "in_step_spmm": per_mode,
                     "spmm_ms_per_step": spmm_ms_step,
                     "step_level": {"algorithmic_bytes_per_step": step_bytes,
                                    "GBps": step_bytes / (step_ms * 1e-3) / 1e9,
                                    "frac": step_bytes / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                    "definition": "all in-step kernels: SURVEY 8d bytes x exact per-agent launch "
                                                  "counts (dpgo_rbcd_bytes)"},
                     "traffic_source": traffic["source"] if traffic else None,
                     "traffic_build_id": traffic.get("build_id") if traffic else None,
                     "traffic_note": traffic_note},
        "xq_spmm": {"kernel": "k_spmm<5,4,MODE_XQ,edge-stream> over colour class 0 (standalone reps)",
                    "avg_launch_ms": spmm_ms, "algorithmic_bytes_per_launch": bsr_bytes,
                    "GBps": bsr_bytes / (spmm_ms * 1e-3) / 1e9 if spmm_ms > 0 else 0.0,
                    "frac": bsr_bytes / (spmm_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if spmm_ms > 0 else 0.0,
                    "format_bytes_per_launch": fmt_bytes,
                    "traffic_bytes_per_launch": (traffic or {}).get("kernels", {}).get("XQ", {}).get(
                        "traffic_bytes_per_launch")},
        # guard: the X.Q-only pass does strictly less work than the HVP over the same colour, so a slower
        # X.Q launch means the measurement (not the kernel) is off -- reported, never hidden
        "xq_guard": {"xq_ms": spmm_ms, "hvp_ms": hvp_ms, "warning": bool(spmm_ms > hvp_ms),
                     "note": "X.Q slower than the HVP over the same colour" if spmm_ms > hvp_ms else "ok"},
        "hvp": {"per_s": 1e3 / hvp_ms if hvp_ms > 0 else 0.0, "avg_launch_ms": hvp_ms,
                "agents": int(eng.agents_per_color[0]),
                "what": "Riemannian HVP (EucHessianEta + EucHvToHv, tangent-projected) over colour class 0"},
        "tcg": tcg,
        "central": {"f_start": f_start, "gradnorm_start": gn_start, "f_end": f_end, "gradnorm_end": gn_end,
                    "steps_between": args.warmup + args.steps,
                    "agents_ready_to_terminate": ready, "agents": owned, "should_terminate": ready == owned},
        "setup_s": setup_s,
        "init": init_info,
    }
    out["comm"] = comm
    if args.precon == "exact":
        # the factor of Q + 0.1 I per colour batch: tree, size, and the device numeric factorisation (it re-runs after
        # every GNC reweighting, inside the timed steps when one falls there), its flops and TFLOP/s against the
        # measured fp64 matrix-core ceiling (tools/fp64_peak.hip, profiles/*_fp64_peak.json)
        out["exact_factor"] = {f"color{c}": eng.exact_factor_info(c) for c in range(eng.num_colors)}
        out["exact_factor"]["refactorisations_in_timed_steps"] = refactor_in_timed
        peak = fp64_peak()
        if peak:
            out["exact_factor"]["fp64_ceiling"] = peak
            for c in range(eng.num_colors):
                fi = out["exact_factor"][f"color{c}"]
                if fi.get("factor_tflops"):
                    fi["factor_frac_of_mfma_f64"] = fi["factor_tflops"] / peak["mfma_f64_16x16x4_tflops"]
        # the solves' roofline: each sweep streams every stored panel once (HBM-bound; HIP events around the sweeps of
        # standalone applications over colour 0, outside the timed steps)
        with torch.cuda.stream(stream):
            out["exact_roofline"] = sweep_roofline(eng)
    out["halo"] = {"kind": args.halo if world > 1 else "none (one rank)",
                   "bytes_sent_per_step_this_rank": 8.0 * (sum(sum(v) for v in c_in) if args.halo == "color"
                                                           else eng.num_colors * int(eng.send_counts.sum())),
                   "full_plan_bytes_per_exchange": 8.0 * int(eng.send_counts.sum())}
    if X_start is not None and args.precon == "exact":
        try:
            from oracle import cpu_port
            # the GPU timed region's mix: every agent update, and every agent factorisation its refactorisations ran
            per_color = max(int(eng.agents_per_color[0]), 1)
            cb = cpu_port.exact_sample_baseline(g, aop, X_start, args.r, bool(args.accel), num_agents,
                                                robust=args.robust, updates=agent_updates,
                                                agent_factorisations=refactor_in_timed * per_color)
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu_baseline"] = value / cb["value"]
        except Exception as exc:  # reported, never silently replaced
            out["cpu_baseline"] = {"error": repr(exc)}
    elif X_start is not None:
        try:
            from oracle import cpu_port
            cb, Xc, stc, iters = cpu_port.engine_baseline(g, aop, X_start, args.r, bool(args.accel), num_agents,
                                                          robust=args.robust)
            if args.robust == "L2":
                cb["like_for_like"] = like_for_like(X_start, Xc, stc, iters)
            else:
                # the host port starts GNC afresh (unit weights, initial mu) while the engine carries the
                # burn-in's weights and mu: the same kind of work per iteration (RTR + reweighting every 30),
                # not the same iterates, so no like-for-like replay
                cb["like_for_like"] = None
                cb["note"] = ("GNC_TLS from fresh weights / initial mu on the host (the engine's burn-in weights "
                              "are not transferred): timing of the same work kind, not the same iterates")
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu_baseline"] = value / cb["value"]
        except Exception as exc:  # reported, never silently replaced
            out["cpu_baseline"] = {"error": repr(exc)}
    if args.certify_iters > 0:
        with torch.cuda.stream(stream):
            Xc = np.zeros(X0.size)
            eng.get_X_into(Xc)
        if world > 1:
            tx = torch.from_numpy(Xc) if one_device else torch.from_numpy(Xc).to(dev)
            dist.all_reduce(tx)
            Xc = tx.cpu().numpy()
        if rank == 0:
            t_c = time.time()
            # thick-restarted Lanczos with X's near-null block locked (dpgo_graph_certify_ex): a lower bound on
            # lambda_min(S(X)), not only a Ritz value (tools/certify_c4.py runs it on converged iterates)
            c = g.certify(Xc, args.r, max_iters=args.certify_iters, tol=1e-8, basis=500 if args.certify_iters > 500 else 0,
                          seed_x=True)
            c["seconds"] = time.time() - t_c
            eta = 1e-6 * abs(c["f_relax"]) / max(g.n, 1)
            c["eta"] = eta
            c["certified"] = bool(c["lower_bound"] >= -eta)
            # the bound takes theta_C as the complement's lowest eigenvalue (Ritz value minus its
            # residual); a thick-restarted Lanczos from one random start could in principle miss a lower one
            c["certified_assumes"] = ("theta_C (thick-restarted Lanczos, one seeded random start) is the lowest "
                                      "eigenvalue of the complement block; a missed lower eigenvalue voids the bound")
            out["certificate"] = c
    if args.boundary_leg:
        # The same engine and step from the odometry chain (no burn-in): every update's tCG stops at its
        # first step on the Delta = 100 boundary, ~4 passes per update -- the regime round 1's headline was
        # measured in, timed the same way (barrier + synchronize, max over ranks).
        with torch.cuda.stream(stream):
            eng.set_X(g.chain_init_dev_layout(args.r, YLift))
            for _ in range(args.warmup):
                step()
            sb0 = eng.stats().copy()
            sync()
            tb0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            sync()
            eb = time.perf_counter() - tb0
            sb = (eng.stats() - sb0).astype(np.int64).sum(axis=0)
        if world > 1:
            tt = torch.tensor([eb], dtype=torch.float64, device="cpu" if one_device else dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            eb = float(tt.item())
            ts = torch.tensor(sb, dtype=torch.int64, device="cpu" if one_device else dev)
            dist.all_reduce(ts)
            sb = ts.cpu().numpy()
        bt = dict(zip(STATS, (int(v) for v in sb)))
        bu = max(bt["calls"], 1)
        out["boundary_regime"] = {
            "value": agent_updates / eb, "unit": "RBCD agent-updates/s", "ms_per_step": 1e3 * eb / args.steps,
            "init": "odometry chain, no burn-in", "steps": args.steps, "warmup": args.warmup,
            "tcg_per_update": {"runs": bt["runs"] / bu, "tcg_iters": bt["tcg_iters"] / bu,
                               "cg_steps": bt["cg_steps"] / bu, "first_step_boundary_runs": bt["implicit"] / bu}}
    if args.exact_leg and world == 1 and args.precon != "exact":
        out["exact_leg"] = exact_leg(args, H, torch, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def sweep_roofline(eng):
    """The exact preconditioner's solves as an HBM roofline: one full application over every agent of colour 0 timed
    sweep by sweep (dpgo_rbcd_bench_precond, HIP events, mean of 5 after 3 untimed), against the panel bytes each
    sweep reads once (dpgo_rbcd_exact_sweep_bytes: wide supernodes' 64 x 64 tiles, narrow ones' compact copies)."""
    mf, mb, stored = eng.bench_precond(0, 5)
    bf, bb = eng.exact_sweep_bytes(0)

    def leg(ms, byt, kernels):
        gbps = byt / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        return {"ms": ms, "bytes": byt, "GBps": gbps, "frac": gbps / HBM_PEAK_GBS, "kernels": kernels}
    return {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "stored_panel_bytes": stored,
            "forward": leg(mf, bf, "every level's k_sn_assemble + k_sn_fwd_small / k_sn_fwd"),
            "backward": leg(mb, bb, "every level's k_sn_bwd"),
            "what": "one full application over every agent of colour 0 (no tCG skip), mean of 5 after 3 untimed; "
                    "bytes = the panels each sweep reads once: wide supernodes' 64 x 64 tiles (padding included), "
                    "narrow ones' compact copies (k_sn_fwd on mixed levels reads their tiles)"}


def exact_leg(args, H, torch, dev):
    """The reference's default configuration -- GNC_TLS robust cost and the exact preconditioner (the factor of
    Q + 0.1 I, src/QuadraticProblem.cpp:37-41, refactorised after every GNC reweighting, src/PGOAgent.cpp:1110-1112) --
    on the C4 grid (k^3 poses, 64 agents), timed like the headline: distributed initialisation, burn-in, set_X, warm-up,
    then `steps` steps between synchronisations.  Reports ms/step, agent-updates/s, the device factorisation's flops
    and TFLOP/s against the measured fp64 ceiling, the sweeps' HBM roofline, and oracle/cpu's exact mode as the CPU
    baseline for the same mix of updates and factorisations.  One GPU only (it runs after the headline)."""
    k, A = args.exact_leg_k, 4
    num_agents = A ** 3
    g = H.Graph.grid3d(k, seed=0)
    aop = g.grid_partition(A)
    eng = H.Rbcd(g, aop, np.zeros(num_agents, np.int32), 0, 1,
                 H.rbcd_params(r=args.r, acceleration=args.accel, robust_cost=H.ROBUST["GNC_TLS"],
                               precon=H.PRECON_EXACT))
    stream = torch.cuda.Stream(dev)
    eng.set_stream(stream.cuda_stream)
    YLift = H.lifting_matrix(3, args.r)
    X0, _, _ = g.distributed_init(aop, args.r, YLift, gpu=True, rtol=1e-12, max_iters=50000, dev_layout=True)

    def step():
        for c in range(eng.num_colors):
            eng.pre_exchange(c)
            eng.update(c, None)

    def factors():
        return sum(eng.exact_factor_info(c)["factor_count"] for c in range(eng.num_colors))

    with torch.cuda.stream(stream):
        eng.set_X(X0)
        for _ in range(args.exact_leg_burnin):
            step()
        X_start = np.zeros(X0.size)
        eng.get_X_into(X_start)
        eng.set_X(X_start)
        for _ in range(args.warmup):
            step()
        st0, fc0 = eng.stats().copy(), factors()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        refac = factors() - fc0
        st = (eng.stats() - st0).astype(np.int64).sum(axis=0)
        roof = sweep_roofline(eng)
    updates = num_agents * args.steps
    tot = dict(zip(STATS, (int(v) for v in st)))
    leg = {"workload": f"grid3d k={k} ({g.n} poses), r={args.r}, {num_agents} agents, Nesterov={bool(args.accel)}, "
                       f"GNC_TLS (reweighting every 30 iterations on the device), exact preconditioner (device "
                       f"refactorisation after each reweighting), distributed init, burn-in {args.exact_leg_burnin}",
           "value": updates / el, "unit": "RBCD agent-updates/s", "ms_per_step": 1e3 * el / args.steps,
           "steps": args.steps, "warmup": args.warmup, "refactorisations_in_timed_steps": refac,
           "tcg": {"updates": tot["calls"], "runs": tot["runs"], "tcg_iters": tot["tcg_iters"],
                   "per_update": tot["tcg_iters"] / max(tot["calls"], 1)}}
    fac = {f"color{c}": eng.exact_factor_info(c) for c in range(eng.num_colors)}
    peak = fp64_peak()
    if peak:
        fac["fp64_ceiling"] = peak
        for c in range(eng.num_colors):
            fi = fac[f"color{c}"]
            if fi.get("factor_tflops"):
                fi["factor_frac_of_mfma_f64"] = fi["factor_tflops"] / peak["mfma_f64_16x16x4_tflops"]
                fi["factor_frac_of_valu_f64"] = fi["factor_tflops"] / peak.get("valu_fma_f64_tflops", float("nan"))
    leg["exact_factor"] = fac
    leg["exact_roofline"] = roof
    if args.cpu_baseline:
        try:
            from oracle import cpu_port
            per_color = max(int(eng.agents_per_color[0]), 1)
            cb = cpu_port.exact_sample_baseline(g, aop, X_start, args.r, bool(args.accel), num_agents,
                                                robust="GNC_TLS", updates=updates,
                                                agent_factorisations=refac * per_color)
            leg["cpu_baseline"] = cb
            leg["speedup_vs_cpu_baseline"] = leg["value"] / cb["value"]
        except Exception as exc:  # reported, never silently replaced
            leg["cpu_baseline"] = {"error": repr(exc)}
    del eng
    return leg


if __name__ == "__main__":
    main()
