#!/usr/bin/env python3
"""Exact-preconditioner outputs of the loaded library (DPGO_HIP_LIB selects another build) on the reference datasets,
both Q formats, written to one .npz: two builds' files compare bitwise (A/B of a kernel change that claims the same
products in the same order).  Measurement / A/B tool only.

  python tools/precond_dump.py OUT.npz            then   python tools/precond_dump.py --compare A.npz B.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        same = [k for k in a.files if np.array_equal(a[k], b[k])]
        diff = [k for k in a.files if k not in same]
        print({"arrays": len(a.files), "bitwise_equal": len(same), "different": diff})
        return 0 if not diff and set(a.files) == set(b.files) else 1
    from _common import load_meas, random_point, random_tangent
    from dpgo_amd import hip as H
    out = {}
    for name, r in [("smallGrid3D", 5), ("sphere2500", 3), ("input_INTEL_g2o", 5), ("torus3D", 5)]:
        meas = load_meas(name)
        d, n = meas.d, meas.num_poses
        X = random_point(r, d, n, 51)
        P = H.Problem(n, d, r)
        P.set_Q_edges(0, meas.p1, meas.p2, meas.R, meas.t, meas.kappa, meas.tau, meas.weight)
        P.set_precon(H.PRECON_EXACT)
        for k in range(3):
            out[f"{name}_{r}_{k}"] = P.precondition(X, random_tangent(X, d, 60 + k))
    np.savez(sys.argv[1], **out)
    print(f"{len(out)} outputs -> {sys.argv[1]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
