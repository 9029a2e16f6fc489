# The exact preconditioner's panels in physically contiguous memory (DPGO_PANEL_CONTIG, default on) against plain
# hipMalloc: sweep timings at C5 colour 0 (tools/sweep_ab.py), one engine per process and two per process in both
# orders; then the exact tests once with the default (contiguous) and once poisoned.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06y}
for o in 0 1; do
  SWEEP_ENV=DPGO_PANEL_CONTIG SWEEP_ORDERS=$o timeout -k 10 300 python3 -u tools/sweep_ab.py --rounds 3 --reps 5 \
    > gpurun_out/${T}_single_$o.json 2> gpurun_out/${T}_single_$o.err || exit 1
  cat gpurun_out/${T}_single_$o.json
done
for oo in 0,1 1,0; do
  SWEEP_ENV=DPGO_PANEL_CONTIG SWEEP_ORDERS=$oo timeout -k 10 400 python3 -u tools/sweep_ab.py --rounds 3 --reps 5 \
    > gpurun_out/${T}_pair_${oo/,/}.json 2> gpurun_out/${T}_pair_${oo/,/}.err || exit 1
  cat gpurun_out/${T}_pair_${oo/,/}.json
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -x -q --timeout 500 --timeout-method thread \
  > gpurun_out/${T}_exact_tests.log 2>&1 || { tail -30 gpurun_out/${T}_exact_tests.log; exit 1; }
tail -1 gpurun_out/${T}_exact_tests.log
DPGO_POISON=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -x -q --timeout 500 \
  --timeout-method thread > gpurun_out/${T}_exact_poison.log 2>&1 || { tail -30 gpurun_out/${T}_exact_poison.log; exit 1; }
tail -1 gpurun_out/${T}_exact_poison.log
