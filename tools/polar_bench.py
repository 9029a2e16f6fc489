"""Microbenchmark of k_polar_comb on 500k poses (r=5, d=3): Y = project(0.9 X + 0.1 V) with V at
growing distance from X, to separate the Newton-Schulz path from the Jacobi fallback."""
import torch

from dpgo_amd import hip as H

n, d, r = 500_000, 3, 5
b = d + 1
P = H.Problem(n, d, r)
g = torch.Generator(device="cuda").manual_seed(0)
dev = torch.device("cuda")


def on_manifold(M):
    out = torch.empty_like(M)
    P.polar_combine_dev(M.data_ptr(), None, [1.0], [0.0], out.data_ptr())
    return out


X = on_manifold(torch.randn(n * r * b, dtype=torch.float64, device=dev, generator=g))
out = torch.empty_like(X)
for sigma in [0.0, 0.01, 0.1, 0.5, 2.0]:
    V = on_manifold(X + sigma * torch.randn(X.shape, dtype=torch.float64, device=dev, generator=g))
    Yv = V.view(n, b, r)[:, :d, :]  # pose-major, column-major r x b: rows of Yv are Y columns
    err = (Yv @ Yv.transpose(1, 2) - torch.eye(d, dtype=torch.float64, device=dev)).abs().amax().item()
    print(f"  V orthonormality error {err:.2e}")
    for _ in range(3):
        P.polar_combine_dev(X.data_ptr(), V.data_ptr(), [0.9], [0.1], out.data_ptr())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    reps = 20
    for _ in range(reps):
        P.polar_combine_dev(X.data_ptr(), V.data_ptr(), [0.9], [0.1], out.data_ptr())
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / reps
    print(f"sigma {sigma:5.2f}: {us:8.1f} us  ({3 * n * r * b * 8 / us / 1e3:.0f} GB/s)", flush=True)
