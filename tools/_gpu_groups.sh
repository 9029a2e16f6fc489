# The 8-GPU share (k = 50, 8 agents: four per colour) with the merged tCG's agents in 2 / 4 / per-agent stream
# groups (TUNE_SPLIT_STREAMS = 1 / 3 / 4), at 4 and 8 HIP hardware queues per process; then the split's bitwise test.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06t}
run() {  # run NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --k 50 --agents-per-axis 2 --steps 200 --cpu-baseline 0 \
     --boundary-leg 0 --exact-leg 0 > gpurun_out/${T}_$name.log 2>&1 || exit 1
  grep '^{' gpurun_out/${T}_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'])"
}
for i in a b; do
  for q in 4 8; do
    for s in 1 3 4; do run s${s}_q${q}_$i GPU_MAX_HW_QUEUES=$q DPGO_TUNE=10=$s; done
  done
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_status_trace.py -m gpu -x -q -k split_streams --timeout 200 \
  --timeout-method thread > gpurun_out/${T}_split_test.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_split_test.log
