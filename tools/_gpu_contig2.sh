# Contiguous panels (default) with the host factor's panels staged through pinned memory: the exact tests, then the
# same tests with the direct pageable copies (DPGO_PANEL_UPLOAD_DIRECT=1, the round-5 / round-6 failure expected),
# then poisoned.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06z}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -x -q --timeout 500 --timeout-method thread \
  > gpurun_out/${T}_exact_tests.log 2>&1 || { tail -5 gpurun_out/${T}_exact_tests.log; exit 1; }
tail -1 gpurun_out/${T}_exact_tests.log
DPGO_PANEL_UPLOAD_DIRECT=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -q \
  --timeout 500 --timeout-method thread > gpurun_out/${T}_exact_direct.log 2>&1
echo "direct rc=$?"
grep -E '^FAILED|passed|failed' gpurun_out/${T}_exact_direct.log | tail -8
DPGO_POISON=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -x -q --timeout 500 \
  --timeout-method thread > gpurun_out/${T}_exact_poison.log 2>&1 || { tail -5 gpurun_out/${T}_exact_poison.log; exit 1; }
tail -1 gpurun_out/${T}_exact_poison.log
