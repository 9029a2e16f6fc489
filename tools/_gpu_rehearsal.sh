# N > 1 path rehearsed on one device (gloo through host copies; bench.py spawns its ranks) and the 8-GPU share.
#   bash tools/_gpu_rehearsal.sh TAG
set -o pipefail
TAG=${1:-r06}
mkdir -p gpurun_out
for n in 2 4 8; do
  DPGO_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 -u bench.py --gpus $n --k 48 --steps 10 --warmup 2 --burnin 30 \
    --cpu-baseline 0 --boundary-leg 0 > gpurun_out/${TAG}_spawn_rehearsal_k48_n$n.log 2>&1 || exit 1
  grep '^{' gpurun_out/${TAG}_spawn_rehearsal_k48_n$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['ms_per_step'], d['comm']['world_size'], d['comm']['torch_world'], d['central']['f_end'])"
done
timeout -k 10 300 python3 -u bench.py --k 50 --agents-per-axis 2 --cpu-baseline 0 --boundary-leg 0 --exact-leg 0 \
  > gpurun_out/${TAG}_share_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/${TAG}_share_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('share', d['ms_per_step'], d['value'])"
