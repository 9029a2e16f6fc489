# The 8-GPU share (k = 50, 8 agents) against the number of HIP hardware queues per process (GPU_MAX_HW_QUEUES):
# whether the two-stream split of small batches lands on one hardware queue (serialised halves) depends on how
# many streams share the queues.  This tree and the round-5 tree in ab_r05/ (temporary), plus the fused finalize.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06s}
run() {  # run NAME DIR ENV...
  local name=$1 dir=$2; shift 2
  X="--exact-leg 0"; [ $dir = ab_r05 ] && X=""
  (cd $dir && env "$@" timeout -k 10 300 python3 -u bench.py --k 50 --agents-per-axis 2 --steps 50 --cpu-baseline 0 \
     --boundary-leg 0 $X > $OLDPWD/gpurun_out/${T}_$name.log 2>&1) || exit 1
  grep '^{' gpurun_out/${T}_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'])"
}
run head_q4_a . GPU_MAX_HW_QUEUES=4
run head_q8_a . GPU_MAX_HW_QUEUES=8
run head_q4_b . GPU_MAX_HW_QUEUES=4
run head_q8_b . GPU_MAX_HW_QUEUES=8
run head_q4_c . GPU_MAX_HW_QUEUES=4
run r05_q8_a ab_r05 GPU_MAX_HW_QUEUES=8
run r05_q8_b ab_r05 GPU_MAX_HW_QUEUES=8
run r05_q4_a ab_r05 GPU_MAX_HW_QUEUES=4
run head_q8_fuse2 . GPU_MAX_HW_QUEUES=8 DPGO_FUSE_FINALIZE=2
run head_q4_fuse2 . GPU_MAX_HW_QUEUES=4 DPGO_FUSE_FINALIZE=2
