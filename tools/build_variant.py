#!/usr/bin/env python3
"""Build a variant of libdpgo_hip.so for same-box A/B runs (loaded through DPGO_HIP_LIB): the units that read the
given -D flags are recompiled into dpgo_amd/ab/<name>/, the others are the tree's own objects (build() first).

  python tools/build_variant.py <name> [--units capi.cpp,spmm5] -DDPGO_MERGED_DD_SLOTS=0x60 ...

Units: a source file name, or spmmK for the K-th SpMM translation unit of kernels.hip.  Default: every unit."""
import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--units", default="")
    a, flags = ap.parse_known_args()
    G.build()
    obj_dir = os.path.join(ROOT, "dpgo_amd", "build")
    out_dir = os.path.join(ROOT, "dpgo_amd", "ab", a.name)
    os.makedirs(out_dir, exist_ok=True)
    units = [(s, os.path.join(G.CSRC, s), []) for s in G.SOURCES]
    units += [(f"spmm{k}", os.path.join(G.CSRC, "kernels.hip"), [f"-DDPGO_SPMM_TU={k}"])
              for k in range(1, G.SPMM_TUS + 1)]
    want = set(a.units.split(",")) if a.units else {u[0] for u in units}
    base = [G.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall"]
    objs, jobs = [], []
    for name, src, extra in units:
        main_obj = os.path.join(obj_dir, (os.path.basename(src) if not extra else f"kernels_{name}") + ".o")
        if name in want:
            o = os.path.join(out_dir, name + ".o")
            if name == "capi.cpp":
                extra = extra + [f'-DDPGO_SOURCE_HASH="variant-{a.name}"']
            jobs.append(base + extra + flags + ["-c", src, "-o", o])
            objs.append(o)
        else:
            objs.append(main_obj)

    def run(cmd):
        print("+", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    with ThreadPoolExecutor(max_workers=min(8, len(jobs) or 1)) as ex:
        list(ex.map(run, jobs))
    run([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out_dir, "libdpgo_hip.so")] + objs)


if __name__ == "__main__":
    main()
