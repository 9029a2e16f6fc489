"""Shared test helpers: fixture loading and oracle setup (test infrastructure)."""
import os

import numpy as np

from oracle import dpgo_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_meas(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.meas.npz"))
    return O.Measurements(int(z["d"]), z["r1"], z["r2"], z["p1"], z["p2"], z["R"], z["t"],
                          z["kappa"], z["tau"], np.ones(len(z["p1"])), int(z["n"]),
                          int(z["duplicates"]))


def random_point(r, d, n, seed):
    rng = O.SplitMix64(seed)
    M = np.array([[rng.normal() for _ in range((d + 1) * n)] for _ in range(r)])
    return O.lifted_project(M, d)


def random_tangent(X, d, seed):
    rng = O.SplitMix64(seed)
    V = np.array([[rng.normal() for _ in range(X.shape[1])] for _ in range(X.shape[0])])
    return O.tangent_project(X, V, d)


def seeded_G(X, d, r, n, seed):
    G = np.zeros_like(X)
    rng = O.SplitMix64(seed)
    for j in range(0, n, max(1, n // 7)):
        for c in range(d + 1):
            for a in range(r):
                G[a, j * (d + 1) + c] = rng.normal()
    return G


def rel(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    den = max(np.linalg.norm(b), 1e-300)
    return float(np.linalg.norm(a - b) / den)
