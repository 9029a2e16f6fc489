# Sweep item records (SnView::desc, DPGO_SN_DESC=1, default) against the per-node arrays (0): C5 colour-0 sweeps, one
# engine per process, alternated twice; then the exact tests.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06zc}
for i in 1 2; do
  for o in 1 0; do
    SWEEP_ENV=DPGO_SN_DESC SWEEP_ORDERS=$o timeout -k 10 300 python3 -u tools/sweep_ab.py --rounds 3 --reps 5 \
      > gpurun_out/${T}_desc${o}_$i.json 2> gpurun_out/${T}_desc${o}_$i.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/${T}_desc${o}_$i.json')); m=list(d['ms'].values())[0]; print('desc=$o', round(m['fwd'],3), round(m['bwd'],3))"
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -x -q --timeout 500 --timeout-method thread \
  > gpurun_out/${T}_exact_tests.log 2>&1 || { tail -5 gpurun_out/${T}_exact_tests.log; exit 1; }
tail -1 gpurun_out/${T}_exact_tests.log
