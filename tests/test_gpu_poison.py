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


def test_panel_guard_gaps_untouched():
    """DPGO_PANEL_GUARD=1: a NaN gap after every supernode's panel (and after the last).  The exact preconditioner's
    single-application, dirty-reuse and per-agent-fallback tests run in a child process with it set: every
    application reports its gaps, none may change (no factor or sweep kernel writes past a node's panel), and the
    tests themselves pass (a gap read into a product would turn the compared output NaN)."""
    import re
    env = dict(os.environ, DPGO_PANEL_GUARD="1")
    out = subprocess.run([sys.executable, "-m", "pytest", "-q", "-s", "-p", "no:cacheprovider", "-m", "gpu",
                          os.path.join(ROOT, "tests", "test_gpu_precon_exact.py"), "-k",
                          "test_exact_precondition or dirty_reuse or fallback_per_agent"],
                         env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    rows = re.findall(r"panel guard: (\d+) of (\d+) guard doubles in (\d+) gaps changed", out.stderr)
    assert len(rows) >= 12, out.stderr[-2000:]
    assert all(int(bad) == 0 and int(gaps) >= 2 for bad, _, gaps in rows), rows[:5]
    print(f"{len(rows)} applications checked, {max(int(g) for _, _, g in rows)} gaps at most, none changed")
