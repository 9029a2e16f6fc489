"""Positive control of the debug poisoning (DPGO_POISON=1, problem_internal.h DevBuf::ensure): a fresh device
allocation reads back as NaN, so a suite run with the variable set proves every kernel result it checks was computed
from written memory only (a read of a never-written entry would turn the result NaN)."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_PROBE = ("import ctypes as C, numpy as np, sys; sys.path.insert(0, %r); from dpgo_amd import hip as H; "
          "o = np.zeros(4); f = H.lib().dpgo_hip_debug_poison_probe; f.argtypes = [C.c_void_p]; f.restype = C.c_int; "
          "assert f(o.ctypes.data) == 0; print(int(np.isnan(o).all()))" % ROOT)


def test_poison_fills_fresh_allocations():
    env = dict(os.environ, DPGO_POISON="1")
    out = subprocess.run([sys.executable, "-c", _PROBE], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "1"
    if os.environ.get("DPGO_POISON", "0") not in ("", "0"):  # this process runs poisoned too
        from dpgo_amd import hip as H
        o = np.zeros(4)
        f = H.lib().dpgo_hip_debug_poison_probe
        f.argtypes = [C.c_void_p]
        f.restype = C.c_int
        assert f(o.ctypes.data) == 0 and np.isnan(o).all()
