#!/usr/bin/env python3
"""GPU idle gaps of a rocprofv3 run recorded with --kernel-trace --hip-trace, and what the host did meanwhile.

Usage (on the GPU box, next to the database: the HIP API trace of a bench run is too large to copy back):
    python tools/gap_probe.py <rocprof outdir or .db> [--last-ms 1500] [--min-gap-us 500]
Over the last `--last-ms` of kernel activity: every idle gap above `--min-gap-us`, the kernels either side,
when the kernel after the gap was enqueued (its launch call's host time relative to the gap start: ≈ gap means
the host was late) and the HIP API calls that overlap the gap for more than 100 µs."""
import argparse
import glob
import re
import sqlite3
from collections import Counter


def short(n):
    m = re.search(r"k_spmm<(\d+), (\d+), (\d+),", n)
    if m:
        return "spmm" + m.group(3)
    return n.split("(")[0].replace("void dpgo::", "")[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last-ms", type=float, default=1500.0)
    ap.add_argument("--min-gap-us", type=float, default=500.0)
    a = ap.parse_args()
    db = a.path if a.path.endswith(".db") else glob.glob(f"{a.path}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    ks = c.execute("select name, start, end, corr_id, grid_x, scratch_size, queue_id from kernels order by start").fetchall()
    t_end = ks[-1][2]
    W = [k for k in ks if k[1] > t_end - a.last_ms * 1e6]
    busy = sum(k[2] - k[1] for k in W)
    span = W[-1][2] - W[0][1]
    print(f"# window {span / 1e6:.1f} ms, kernels busy {busy / 1e6:.1f} ms ({100 * busy / span:.1f} %), {len(W)} kernels")
    launch = {}
    for nm, st, en, corr in c.execute("select name, start, end, corr_id from regions where name like '%Launch%'"):
        launch[corr] = (st, en)
    if not launch:  # schema / naming check: what the regions table holds
        cols = [r[1] for r in c.execute("pragma table_info(regions)")]
        names = Counter(nm for (nm,) in c.execute("select name from regions limit 200000"))
        print("# no launch regions matched; regions columns:", cols, "top names:", names.most_common(12))
        kc = [r[1] for r in c.execute("pragma table_info(kernels)")]
        print("# kernels columns:", kc)
    gaps = []
    for x, y in zip(W, W[1:]):
        g = y[1] - x[2]
        if g > a.min_gap_us * 1e3:
            gaps.append((x, y, g))
    print(f"# gaps > {a.min_gap_us:.0f} us: {len(gaps)}, {sum(g for _, _, g in gaps) / 1e6:.1f} ms")
    pairs = Counter()
    for x, y, g in gaps:
        pairs[(short(x[0]), short(y[0]))] += g
    for k, v in pairs.most_common(12):
        print(f"#   {v / 1e6:8.2f} ms  {k[0]} -> {k[1]}")
    step = 100e6
    b0 = W[0][1]
    nb = int((W[-1][2] - b0) // step) + 1
    fill = [0.0] * nb
    for k in W:
        fill[int((k[1] - b0) // step)] += k[2] - k[1]
    print("# busy per 100 ms bucket:", " ".join(f"{100 * f / step:.0f}" for f in fill))
    for x, y, g in sorted(gaps, key=lambda t: -t[2])[:25]:
        l = launch.get(y[3])
        enq = f"{(l[0] - x[2]) / 1e3:9.1f}" if l else "        ?"
        print(f"gap {g / 1e3:9.1f} us at {(x[2] - b0) / 1e6:8.1f} ms  {short(x[0]):>28s} -> {short(y[0]):<28s} next enqueued at +{enq} us "
              f"(grid {y[4]}, scratch {y[5]}, queue {x[6]}->{y[6]}, dur {(y[2] - y[1]) / 1e3:.1f} us)")
        calls = c.execute("select name, start, end from regions where end > ? and start < ? and end - start > 100000 "
                          "order by start", (x[2], y[1])).fetchall()
        for nm, st, en in calls[:8]:
            print(f"      {nm[:60]:60s} {(st - x[2]) / 1e3:10.1f} .. {(en - x[2]) / 1e3:10.1f} us")
        cnt = Counter(nm for (nm,) in c.execute("select name from regions where start > ? and start < ?",
                                                (x[2], y[1])))
        print("      api calls in gap:", dict(cnt.most_common(6)))


if __name__ == "__main__":
    main()
