#!/usr/bin/env python3
"""HBM traffic of the exact preconditioner's sweeps (k_sn_fwd / k_sn_bwd) per application against the supernodal
panels' size: two rocprofv3 PMC passes (FETCH_SIZE, then WRITE_SIZE) over a short C5 bench run with the exact
preconditioner, the read side calibrated against a 512 MiB device copy in the same pass (MI355X_MICROARCH.md).

Usage on the GPU box:  python tools/pmc_exact.py run <outdir>
                       python tools/pmc_exact.py summarize <outdir> > profiles/rNN_pmc_exact.json
"""
import glob
import json
import os
import sqlite3
import subprocess
import sys

CALIB_MB = 512
LEVELS = 13  # C5 agents' tree depth (one launch per level and sweep)


def run(outdir):
    os.makedirs(outdir, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp", DPGO_VERBOSE_CHOL="1")
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        cmd = ["timeout", "-s", "KILL", "400", "rocprofv3", "--kernel-trace", "--pmc", ctr, "-d",
               os.path.join(outdir, ctr), "-o", "run", "--", sys.executable, "bench.py", "--precon", "exact",
               "--steps", "2", "--warmup", "0", "--burnin", "5", "--cpu-baseline", "0", "--boundary-leg", "0",
               "--kernel-timing", "0", "--spmm-reps", "2", "--pmc-calib-mb", str(CALIB_MB)]
        with open(os.path.join(outdir, ctr + ".log"), "w") as f:
            rc = subprocess.call(cmd, stdout=f, stderr=subprocess.STDOUT, env=env)
        if rc != 0:
            raise SystemExit(f"pass {ctr} failed rc={rc}")


def per_launch(outdir, ctr):
    """{kernel: [counter value per launch, in dispatch order]}"""
    db = glob.glob(os.path.join(outdir, ctr, "**", "run_results.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    acc = {}
    for name, val in c.execute("select kernel_name, value from counters_collection where counter_name=? "
                               "order by dispatch_id", (ctr,)):
        acc.setdefault(name.split("(")[0].replace("void dpgo::", ""), []).append(val)
    return acc


def totals(outdir, ctr):
    return {k: (sum(v), len(v)) for k, v in per_launch(outdir, ctr).items()}


def summarize(outdir):
    f, w = totals(outdir, "FETCH_SIZE"), totals(outdir, "WRITE_SIZE")
    # the calibration copy: the largest single copyBuffer launch (bench.py --pmc-calib-mb; the others are small)
    copies = [x for k, v in per_launch(outdir, "FETCH_SIZE").items() if "copyBuffer" in k for x in v]
    calib = CALIB_MB * 1024 * 1024 / (max(copies) * 1024.0) if copies else None
    panel_gib = None
    with open(os.path.join(outdir, "FETCH_SIZE.log")) as fh:
        for line in fh:
            if "GiB of supernodal panels" in line:
                panel_gib = float(line.split(",")[1].split("GiB")[0])
    out = {"read_factor": calib, "panel_bytes_per_colour": panel_gib * 2 ** 30 if panel_gib else None,
           "kernels": {}}
    fl = per_launch(outdir, "FETCH_SIZE")
    for k in ("k_sn_fwd<5>", "k_sn_bwd<5>", "k_sn_assemble<5>"):
        if k not in fl:
            continue
        v = fl[k]
        apps = [sum(v[i:i + LEVELS]) for i in range(0, len(v) - LEVELS + 1, LEVELS)]
        # the largest application: every agent of the colour still in tCG (later ones skip stopped agents' nodes)
        rd = max(apps) * 1024.0 * (calib or 1.0)
        out["kernels"][k] = {"launches": len(v), "applications": len(apps),
                             "read_bytes_full_application": rd,
                             "read_bytes_mean_application": sum(apps) / len(apps) * 1024.0 * (calib or 1.0),
                             "write_bytes_per_launch_mean": w.get(k, (0.0, 1))[0] * 1024.0 / max(w.get(k, (0, 1))[1], 1),
                             "read_full_over_panel": rd / out["panel_bytes_per_colour"]
                             if out["panel_bytes_per_colour"] else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    run(sys.argv[2]) if sys.argv[1] == "run" else summarize(sys.argv[2])
