# Round-end verification on the final tree: the GPU suite and smoke exactly as the driver runs them, the exact
# preconditioner's tests once more under DPGO_POISON=1 (the compact panels included), and the 8-GPU share.
#   bash tools/_gpu_final.sh TAG
set -o pipefail
TAG=${1:-r06}
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_smoke.log
DPGO_POISON=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -x -q --timeout 500 \
  --timeout-method thread > gpurun_out/${TAG}_exact_poison.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_exact_poison.log
timeout -k 10 300 python3 -u bench.py --k 50 --agents-per-axis 2 --steps 50 --cpu-baseline 0 --boundary-leg 0 \
  --exact-leg 0 > gpurun_out/${TAG}_share_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/${TAG}_share_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('share', d['ms_per_step'], d['value'])"
