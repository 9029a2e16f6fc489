#!/usr/bin/env python3
"""Summarise rocprofv3 PMC databases (run_results.db) per kernel: mean counter value per dispatch
and mean duration.  Usage: python tools/pmc_summary.py <dir-with-*/run_results.db> [kernel-substring]"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else "k_spmm"
    rows = []
    for db in sorted(glob.glob(os.path.join(root, "*", "run_results.db"))):
        c = sqlite3.connect(db)
        acc = defaultdict(list)
        for name, ctr, val, dur in c.execute(
                "select kernel_name, counter_name, value, duration from counters_collection"):
            if filt in name:
                acc[(name, ctr)].append((val, dur))
        for (name, ctr), v in sorted(acc.items()):
            n = len(v)
            rows.append((os.path.basename(os.path.dirname(db)), name[:60], ctr, n,
                         sum(x for x, _ in v) / n, sum(d for _, d in v) / n / 1e3))
    print(f"{'pass':45s} {'kernel':60s} {'counter':22s} {'n':>3s} {'mean value':>16s} {'dur_us':>8s}")
    for r in rows:
        print(f"{r[0]:45s} {r[1]:60s} {r[2]:22s} {r[3]:3d} {r[4]:16.4f} {r[5]:8.1f}")


if __name__ == "__main__":
    main()
