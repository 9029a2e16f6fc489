#!/usr/bin/env python3
"""Per-kernel PMC counters over bench.py's RBCD step in the CG regime (1M-pose grid, 64 agents): one
rocprofv3 pass per counter group (rocprofv3 does not split counters over passes; at most 8 SQ counters per
pass), the median of each counter over a kernel's last launches.

Usage on the GPU box:  python tools/pmc_kernel.py run <outdir> [group ...]
                       python tools/pmc_kernel.py summarize <outdir>
A group is a space-separated counter list, e.g. "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY".
"""
import glob
import json
import os
import re
import sqlite3
import subprocess
import sys

GROUPS = [
    "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT "
    "SQ_LDS_IDX_ACTIVE",
    "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum",
]
MODES = ["XQ", "XQ_G", "EVAL", "HESS", "F", "EVAL_TCG", "CERT", "QF", "HESS_QF", "HESS_M", "HESS_QF_M"]


def run(outdir, groups):
    os.makedirs(outdir, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    for i, grp in enumerate(groups):
        d = os.path.join(outdir, f"g{i}")
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--kernel-trace", "--pmc"] + grp.split() + [
            "-d", d, "-o", "run", "--", sys.executable, "bench.py", "--steps", "2", "--warmup", "0",
            "--cpu-baseline", "0", "--boundary-leg", "0", "--exact-leg", "0", "--kernel-timing", "0", "--spmm-reps",
            "2"]
        with open(d + ".log", "w") as f:
            rc = subprocess.call(cmd, stdout=f, stderr=subprocess.STDOUT, env=env)
        if rc != 0:
            raise SystemExit(f"pass {i} ({grp}) failed rc={rc}")


def short(name):
    m = re.search(r"k_spmm<(\d+), (\d+), (\d+),", name)
    if m:
        return "k_spmm " + MODES[int(m.group(3))]
    return name.split("(")[0].replace("void dpgo::", "")


def summarize(outdir, last=40):
    acc = {}
    for db in sorted(glob.glob(os.path.join(outdir, "g*", "**", "run_results.db"), recursive=True)):
        c = sqlite3.connect(db)
        for name, ctr, val in c.execute("select kernel_name, counter_name, value from counters_collection "
                                        "order by dispatch_id"):
            acc.setdefault(short(name), {}).setdefault(ctr, []).append(val)
    out = {}
    for k, ctrs in acc.items():
        if not any(s in k for s in ("k_spmm", "k_tcg_updir", "k_finalize", "k_retract")):
            continue
        row = {}
        for ctr, v in ctrs.items():
            t = sorted(v[-last:])
            row[ctr] = t[len(t) // 2]
        w = row.get("SQ_WAVE_CYCLES")
        if w:
            for s in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if s in row:
                    row[s + "_frac"] = row[s] / w
        if row.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_conflict_frac"] = row.get("SQ_LDS_BANK_CONFLICT", 0.0) / row["SQ_LDS_IDX_ACTIVE"]
        if "TCC_HIT_sum" in row and "TCC_MISS_sum" in row:
            row["l2_hit_rate"] = row["TCC_HIT_sum"] / max(row["TCC_HIT_sum"] + row["TCC_MISS_sum"], 1.0)
        out[k] = row
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dpgo_amd import hip as H  # the profiled library's build (a constant: no GPU call)
    out["build_id"] = H.build_id()
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3:] or GROUPS)
    else:
        summarize(sys.argv[2])
