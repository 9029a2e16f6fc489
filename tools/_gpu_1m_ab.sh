# Same-box A/B of the one-GPU headline workload (1M poses, 64 agents) between this tree and the round-5 tree in
# ab_r05/ (temporary), alternated twice; plus the barrier probe (tools/barrier_probe.hip).
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06v}
timeout -k 10 120 ./tools/barrier_probe > gpurun_out/${T}_barrier_probe.json 2>&1 || exit 1
for i in 1 2; do
  (cd ab_r05 && timeout -k 10 400 python3 -u bench.py --cpu-baseline 0 --boundary-leg 0 \
     > ../gpurun_out/${T}_1m_r05_$i.log 2>&1) || exit 1
  grep '^{' gpurun_out/${T}_1m_r05_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('r05', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  timeout -k 10 400 python3 -u bench.py --cpu-baseline 0 --boundary-leg 0 --exact-leg 0 \
     > gpurun_out/${T}_1m_head_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/${T}_1m_head_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('head', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
