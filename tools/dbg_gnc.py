import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from dpgo_amd import hip as H
from oracle import dpgo_oracle as O
from tests._common import rel
from tests.test_gpu_rbcd import _grid_with_outliers, _run_engine
k, A, r = 6, 2, 5
g, g0, meas = _grid_with_outliers(H, k, 3, 0.1, 7)
aop = g0.grid_partition(A)
X0 = g0.chain_init(r, O.lifting_matrix(3, r))
for accel in (False, True):
    for iters in (2, 3, 4, 6, 9):
        Xh, e = _run_engine(H, g, aop, A ** 3, X0, iters, accel, r, robust_cost=H.ROBUST["GNC_TLS"], robust_opt_inner_iters=3)
        Xo, _ = O.colour_rbcd(meas, aop, A ** 3, X0, iters, r, acceleration=accel, robust="GNC_TLS", robust_opt_inner_iters=3)
        Xl, _ = O.colour_rbcd(meas, aop, A ** 3, X0, iters, r, acceleration=accel, robust="L2")
        Xhl, _ = _run_engine(H, g, aop, A ** 3, X0, iters, accel, r)
        print(accel, iters, "eng-gnc vs orc-gnc", rel(Xh, Xo), "eng-gnc vs orc-l2", rel(Xh, Xl), "eng-l2 vs orc-l2", rel(Xhl, Xl), flush=True)
