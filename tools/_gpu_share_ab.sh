# Same-box A/B of the 8-GPU share (k = 50, 8 agents) between this tree and the round-5 tree in ab_r05/ (temporary).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  (cd ab_r05 && timeout -k 10 300 python3 -u bench.py --k 50 --agents-per-axis 2 --steps 50 --cpu-baseline 0 \
     --boundary-leg 0 > ../gpurun_out/r06p_share_r05_$i.log 2>&1) || exit 1
  grep '^{' gpurun_out/r06p_share_r05_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('r05', d['ms_per_step'])"
  timeout -k 10 300 python3 -u bench.py --k 50 --agents-per-axis 2 --steps 50 --cpu-baseline 0 --boundary-leg 0 \
     --exact-leg 0 > gpurun_out/r06p_share_r06_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/r06p_share_r06_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('r06', d['ms_per_step'])"
done
