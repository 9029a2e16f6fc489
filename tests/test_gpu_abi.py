"""The C ABI from a plain C caller on the GPU: arrays sized by include/*.h with canary words after them
survive dpgo_rbcd_kernel_times / dpgo_rbcd_mode_bytes / dpgo_rbcd_stats (no out-of-bounds writes)."""
import subprocess

import pytest

from tests.test_host_native import build_abi_check

pytestmark = pytest.mark.gpu


def test_c_caller_header_sized_arrays_keep_canaries(tmp_path):
    exe = build_abi_check(tmp_path)
    p = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.returncode, p.stdout, p.stderr)
    assert "canaries ok" in p.stdout
