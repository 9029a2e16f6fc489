#!/usr/bin/env python3
"""Per-level launch durations of the exact preconditioner's last full application in a rocprofv3 rocpd database
(k_sn_assemble / k_sn_fwd per level, deepest first, then k_sn_bwd per level, root first).  Probe only."""
import glob
import sqlite3
import sys


def main():
    path = sys.argv[1]
    db = path if path.endswith(".db") else glob.glob(f"{path}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name}, start, end from kernels where {name} like '%k_sn_%' order by start").fetchall()
    # the last application: from the last k_sn_assemble that follows a k_sn_bwd (or the first) to the end
    starts = [i for i in range(len(rows)) if "k_sn_assemble" in rows[i][0] and (i == 0 or "k_sn_bwd" in rows[i - 1][0])]
    last = rows[starts[-1]:] if starts else rows
    t0 = last[0][1]
    for nm, s, e in last:
        short = nm.split("(")[0].replace("void dpgo::", "")
        print(f"{short:24s} start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us")
    print(f"application: {(last[-1][2] - t0) / 1e3:.1f} us, kernels {sum(e - s for _, s, e in last) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
