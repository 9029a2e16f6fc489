"""Per-kernel summary (calls, total / average ns) from a rocprofv3 rocpd database.

--timed-steps K: only the kernels of bench.py's timed region, located in the trace as the window from
the start of the 2K-th last tCG-start evaluation launch (k_spmm mode 5, one per colour per step) to the
start of the first central evaluation (k_spmm mode 2) after the last one; the first timed step's
pre-exchange kernels fall outside the window (a few microseconds)."""
import argparse
import glob
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--timed-steps", type=int, default=0)
    ap.add_argument("--colors", type=int, default=2)
    a = ap.parse_args()
    db = a.path if a.path.endswith(".db") else glob.glob(f"{a.path}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    where = ""
    if a.timed_steps:
        ev = [r[0] for r in c.execute(f"select start from kernels where {name} like '%k_spmm<5, 4, 5,%' "
                                      f"order by start")]
        n = a.timed_steps * a.colors
        t0 = ev[-n]
        t1 = c.execute(f"select min(start) from kernels where {name} like '%k_spmm<5, 4, 2,%' and start > ?",
                       (ev[-1],)).fetchone()[0]
        where = f"where start >= {t0} and start < {t1}"
        print(f"# timed window: {(t1 - t0) / 1e6:.3f} ms over {a.timed_steps} steps "
              f"({(t1 - t0) / 1e6 / a.timed_steps:.3f} ms/step wall, kernels only below)")
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels {where} "
                     f"group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage"')
    for nm, k, t, av in rows:
        print(f'"{nm}",{k},{t},{av:.1f},{100.0 * t / tot:.2f}')
    print(f"# kernel time total {tot / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
