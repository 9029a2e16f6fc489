#!/usr/bin/env python3
"""HBM traffic per launch of the in-step X.Q kernels of bench.py's RBCD step (MI355X_MICROARCH.md, HBM
section): two separate rocprofv3 PMC passes (FETCH_SIZE, then WRITE_SIZE) over a short bench run in the
CG regime (burn-in as the default bench), each with a device copy of known size as the read calibration
(FETCH_SIZE on gfx950 under-counts wide reads; factor = copy read bytes / FETCH_SIZE(copy), same pass).

Per SpMM mode the median over the mode's last launches (all in the CG regime, every agent active) is
reported; bench.py folds profiles/*_pmc_traffic.json "kernels" into its roofline "traffic".

Usage on the GPU box:  python tools/pmc_step.py run <outdir>
                       python tools/pmc_step.py summarize <outdir> > profiles/rNN_pmc_traffic.json
"""
import glob
import json
import os
import re
import sqlite3
import subprocess
import sys

MODES = ["XQ", "XQ_G", "EVAL", "HESS", "F", "EVAL_TCG", "CERT", "QF", "HESS_QF", "HESS_M", "HESS_QF_M"]
CALIB_MB = 512


def run(outdir):
    os.makedirs(outdir, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        cmd = ["timeout", "-s", "KILL", "300", "rocprofv3", "--kernel-trace", "--pmc", ctr, "-d",
               os.path.join(outdir, ctr), "-o", "run", "--", sys.executable, "bench.py", "--steps", "3", "--warmup",
               "1", "--cpu-baseline", "0", "--kernel-timing", "0", "--spmm-reps", "3",
               "--pmc-calib-mb", str(CALIB_MB), "--exact-leg", "0", "--boundary-leg", "0"]
        with open(os.path.join(outdir, ctr + ".log"), "w") as f:
            rc = subprocess.call(cmd, stdout=f, stderr=subprocess.STDOUT, env=env)
        if rc != 0:
            raise SystemExit(f"pass {ctr} failed rc={rc}")


def _db(outdir, ctr):
    found = glob.glob(os.path.join(outdir, ctr, "**", "run_results.db"), recursive=True)
    if not found:
        raise SystemExit(f"no database for {ctr} under {outdir}")
    return found[0]


def per_kernel(db, ctr, last=200):
    """{kernel name: median of the last `last` launches' counter value}, in dispatch order."""
    c = sqlite3.connect(db)
    acc = {}
    for name, val in c.execute("select kernel_name, value from counters_collection where counter_name=? "
                               "order by dispatch_id", (ctr,)):
        acc.setdefault(name, []).append(val)
    out = {}
    for k, v in acc.items():
        t = sorted(v[-last:])
        out[k] = (t[len(t) // 2], len(v), max(v))
    return out


def summarize(outdir):
    fetch = per_kernel(_db(outdir, "FETCH_SIZE"), "FETCH_SIZE")
    write = per_kernel(_db(outdir, "WRITE_SIZE"), "WRITE_SIZE")
    copies = [k for k in fetch if "copyBuffer" in k]
    if not copies:
        raise SystemExit(f"calibration copy not found: {list(fetch)[:20]}")
    copy = max(copies, key=lambda k: fetch[k][2])
    copy_bytes = CALIB_MB * (1 << 20)
    factor = copy_bytes / (fetch[copy][2] * 1024.0)
    kernels = {}
    for name in fetch:
        m = re.search(r"k_spmm<(\d+), (\d+), (\d+),", name)
        if not m:
            continue
        mode = MODES[int(m.group(3))]
        rd = fetch[name][0] * 1024.0 * factor
        wr = write.get(name, (0.0, 0, 0.0))[0] * 1024.0
        kernels[mode] = {"kernel": name, "launches_profiled": fetch[name][1], "fetch_size_kb": fetch[name][0],
                         "write_size_kb": wr / 1024.0, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                         "traffic_bytes_per_launch": rd + wr}
    others = {}
    for name in fetch:
        if "k_spmm<" in name or "copyBuffer" in name:
            continue
        rd = fetch[name][0] * 1024.0 * factor
        wr = write.get(name, (0.0, 0, 0.0))[0] * 1024.0
        others[name.split("(")[0]] = {"read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                                      "launches_profiled": fetch[name][1]}
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dpgo_amd import hip as H  # the library the profiled bench loaded (no GPU call: the id is a constant)
    out = {"workload": "bench.py defaults (1M-pose grid, 64 agents, distributed init + burn-in, CG regime), "
                       "--steps 3 --warmup 1; median over each kernel's last 200 launches",
           "build_id": H.build_id(),
           "calibration_kernel": copy, "calibration_read_bytes": copy_bytes,
           "calibration_fetch_size_kb": fetch[copy][2], "read_factor": factor,
           "kernels": kernels, "other_kernels": others}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        summarize(sys.argv[2])
