# Which contiguous buffer turns test_exact_precondition[sphere2500-3-bsr] wrong: the exact tests up to it with
# DPGO_PANEL_CONTIG = 1 (tile panels) / 2 (compact copies) / 3 (both), compact copies on and off, and the test alone.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06za}
K="test_exact_precondition"
for cfg in "1 1" "2 1" "3 1" "3 0" "0 1"; do
  set -- $cfg
  DPGO_PANEL_CONTIG=$1 DPGO_SN_COMPACT=$2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -q \
    -k "$K" --timeout 250 --timeout-method thread > gpurun_out/${T}_c$1_s$2.log 2>&1
  echo "contig=$1 compact=$2 rc=$? $(grep -E 'passed|failed' gpurun_out/${T}_c$1_s$2.log | tail -1) $(grep -E '^FAILED' gpurun_out/${T}_c$1_s$2.log | head -3 | tr '\n' ' ')"
done
DPGO_PANEL_CONTIG=3 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -q \
  -k "test_exact_precondition and sphere2500-3-bsr" --timeout 250 --timeout-method thread > gpurun_out/${T}_alone.log 2>&1
echo "alone rc=$? $(tail -1 gpurun_out/${T}_alone.log)"
