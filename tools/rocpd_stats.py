"""Per-kernel summary (calls, total / average ns) from a rocprofv3 rocpd database."""
import glob
import sqlite3
import sys


def main(path):
    db = path if path.endswith(".db") else glob.glob(f"{path}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels group by {name} "
                     f"order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage"')
    for n, k, t, a in rows:
        print(f'"{n}",{k},{t},{a:.1f},{100.0 * t / tot:.2f}')


if __name__ == "__main__":
    main(sys.argv[1])
