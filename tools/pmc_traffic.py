#!/usr/bin/env python3
"""HBM traffic per launch of the X.Q SpMM from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section).

Two separate passes (rocprofv3 does not split counters): FETCH_SIZE, then WRITE_SIZE, each over
tools/spmm_ab.py (X.Q over one colour class of the 1M-pose grid + a device copy of known size).
FETCH_SIZE on gfx950 under-counts wide reads (the guide: exactly 1/2 for 16-B/lane streams; other
widths uncalibrated), so the read side is calibrated in the SAME pass against the copy kernel, whose
read bytes are known: factor = copy_read_bytes / FETCH_SIZE(copy).  WRITE_SIZE is exact for 16-B
stores (our Y stores are 8-40 B per lane and are reported raw).

Usage on the GPU box:  python tools/pmc_traffic.py run <outdir> [--qfmt edges]
                       python tools/pmc_traffic.py summarize <outdir>  -> JSON on stdout
"""
import glob
import json
import os
import sqlite3
import subprocess
import sys


def run(outdir, qfmt):
    os.makedirs(outdir, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    var = "1" if qfmt == "edges" else "0"
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--kernel-trace", "--pmc", ctr, "-d",
               os.path.join(outdir, ctr), "-o", "run", "--", sys.executable, "tools/spmm_ab.py", "--qfmt", qfmt,
               "--variants", var, "--rounds", "1", "--reps", "5"]
        with open(os.path.join(outdir, ctr + ".log"), "w") as f:
            rc = subprocess.call(cmd, stdout=f, stderr=subprocess.STDOUT, env=env)
        if rc != 0:
            raise SystemExit(f"pass {ctr} failed rc={rc}")
    with open(os.path.join(outdir, "FETCH_SIZE.log")) as f:
        last = [l for l in f if l.startswith("{")][-1]
    json.dump(json.loads(last), open(os.path.join(outdir, "ab.json"), "w"))


def per_kernel(db, ctr, how="mean"):
    c = sqlite3.connect(db)
    acc = {}
    for name, val in c.execute("select kernel_name, value from counters_collection where counter_name=?", (ctr,)):
        acc.setdefault(name, []).append(val)
    if how == "max":
        return {k: max(v) for k, v in acc.items()}
    return {k: sum(v) / len(v) for k, v in acc.items()}


def summarize(outdir):
    ab = json.load(open(os.path.join(outdir, "ab.json")))
    fetch = per_kernel(glob.glob(os.path.join(outdir, "FETCH_SIZE", "*", "run_results.db"))[0]
                       if glob.glob(os.path.join(outdir, "FETCH_SIZE", "*", "run_results.db"))
                       else os.path.join(outdir, "FETCH_SIZE", "run_results.db"), "FETCH_SIZE")
    write = per_kernel(glob.glob(os.path.join(outdir, "WRITE_SIZE", "*", "run_results.db"))[0]
                       if glob.glob(os.path.join(outdir, "WRITE_SIZE", "*", "run_results.db"))
                       else os.path.join(outdir, "WRITE_SIZE", "run_results.db"), "WRITE_SIZE")
    spmm = [k for k in fetch if "k_spmm<5, 4, 0," in k]
    fdb = glob.glob(os.path.join(outdir, "FETCH_SIZE", "*", "run_results.db")) or \
        [os.path.join(outdir, "FETCH_SIZE", "run_results.db")]
    fmax = per_kernel(fdb[0], "FETCH_SIZE", "max")
    copies = [k for k in fmax if "copyBuffer" in k]  # the D2D calibration copies (largest dispatch)
    if not spmm or not copies:
        raise SystemExit(f"kernels not found: {list(fetch)}")
    kname = spmm[0]
    copy = copies[0]
    fetch = dict(fetch, **{copy: fmax[copy]})
    # spmm_ab's calibration copy: n = bytes // 16 doubles read and written
    copy_bytes = (int(ab["bytes"]) // 16) * 8
    factor = copy_bytes / (fetch[copy] * 1024.0)
    rd = fetch[kname] * 1024.0 * factor
    wr = write[kname] * 1024.0
    out = {"kernel": kname, "qfmt": ab.get("qfmt"), "fetch_size_kb": fetch[kname], "write_size_kb": write[kname],
           "calibration_kernel": copy, "calibration_read_bytes": copy_bytes,
           "calibration_fetch_size_kb": fetch[copy], "read_factor": factor,
           "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "traffic_bytes_per_launch": rd + wr,
           "algorithmic_bytes_per_launch_bsr": ab.get("bsr_bytes"), "format_bytes_per_launch": ab.get("format_bytes")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        q = sys.argv[sys.argv.index("--qfmt") + 1] if "--qfmt" in sys.argv else "edges"
        run(sys.argv[2], q)
    else:
        summarize(sys.argv[2])
