#!/usr/bin/env python3
"""Probe: does a large device buffer stream slower when it was allocated first?  Allocates --n buffers of --gb GiB
(torch, hipMalloc underneath), fills them, then times a full read of each (torch.sum, HIP events) in alternating
rounds and prints the median per buffer.  Probe only."""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3)
    ap.add_argument("--gb", type=float, default=12.0)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    bufs = []
    for _ in range(a.n):
        x = torch.empty(int(a.gb * (1 << 30)) // 8, dtype=torch.float64, device="cuda")
        x.fill_(1.0)
        bufs.append(x)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = [[] for _ in bufs]
    for _ in range(a.rounds):
        for i, x in enumerate(bufs):
            ev[0].record()
            s = x.sum()
            ev[1].record()
            ev[1].synchronize()
            res[i].append(ev[0].elapsed_time(ev[1]))
    out = {f"buf{i}": {"ms": sorted(r)[len(r) // 2], "GBps": bufs[i].numel() * 8 / (sorted(r)[len(r) // 2] * 1e-3) / 1e9}
           for i, r in enumerate(res)}
    print(json.dumps({"gb": a.gb, "n": a.n, "sum_check": float(s), "buffers": out}), flush=True)


if __name__ == "__main__":
    main()
