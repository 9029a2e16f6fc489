#!/usr/bin/env python3
"""Where the merged tCG finalize (k_finalize<8, OP_TCG_STEP_CHECK>) spends its time: wall-clock marks in agent 0's
block of a DPGO_FIN_PROBE build (python tools/build_variant.py finprobe --units kernels.hip,capi.cpp
-DDPGO_FIN_PROBE; run with DPGO_HIP_LIB=dpgo_amd/ab/finprobe/libdpgo_hip.so).  Marks: 0 entry, 1 partials
summed, 2 first barrier, 3 totals reduced, 4 scalar logic done, 5 state stored; medians over the last 256
launches in 10 ns ticks.

  python tools/fin_probe.py [--k 50 --agents-per-axis 2] [--burnin 300 --steps 20]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--agents-per-axis", type=int, default=2)
    ap.add_argument("--burnin", type=int, default=300)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from dpgo_amd import hip as H
    torch.cuda.set_device(0)
    g = H.Graph.grid3d(a.k, seed=0)
    aop = g.grid_partition(a.agents_per_axis)
    eng = H.Rbcd(g, aop, np.zeros(a.agents_per_axis ** 3, np.int32), 0, 1, H.rbcd_params(r=5, acceleration=1))
    stream = torch.cuda.Stream()
    eng.set_stream(stream.cuda_stream)
    X0, _, _ = g.distributed_init(aop, 5, H.lifting_matrix(3, 5), gpu=True, rtol=1e-12, max_iters=50000,
                                  dev_layout=True)
    eng.set_X(X0)
    with torch.cuda.stream(stream):
        for _ in range(a.burnin + a.steps):
            for c in range(eng.num_colors):
                eng.pre_exchange(c)
                eng.update(c, None)
        torch.cuda.synchronize()
    fn = H.lib().dpgo_hip_debug_fin_probe
    buf = (C.c_longlong * (256 * 6))()
    n = C.c_int()
    assert fn(buf, C.byref(n)) == 0
    t = np.array(buf[:], dtype=np.int64).reshape(256, 6)
    t = t[t[:, 0] > 0]
    d = np.diff(t, axis=1)
    names = ["partials", "barrier1", "reduce+barrier2", "scalar", "store+wait"]
    print(f"launches probed {n.value}; median ticks (10 ns) per phase:",
          {nm: float(np.median(d[:, i])) for i, nm in enumerate(names)},
          "total", float(np.median(t[:, 5] - t[:, 0])))


if __name__ == "__main__":
    main()
