# Kernel traces of the 8-GPU share (k = 50, 8 agents) for this tree and the round-5 tree in ab_r05/ (temporary).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd ab_r05 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_s05 -o run -- python3 bench.py \
   --k 50 --agents-per-axis 2 --cpu-baseline 0 --boundary-leg 0 > ../gpurun_out/r06q_kt_r05.log 2>&1) || exit 1
python3 tools/rocpd_stats.py gpurun_out/prof_s05 --timed-steps 20 > gpurun_out/r06q_share_kt_r05.csv 2>&1 || exit 1
rm -rf gpurun_out/prof_s05
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s06 -o run -- python3 bench.py \
   --k 50 --agents-per-axis 2 --cpu-baseline 0 --boundary-leg 0 --exact-leg 0 > gpurun_out/r06q_kt_r06.log 2>&1 || exit 1
python3 tools/rocpd_stats.py gpurun_out/prof_s06 --timed-steps 20 > gpurun_out/r06q_share_kt_r06.csv 2>&1 || exit 1
rm -rf gpurun_out/prof_s06
head -12 gpurun_out/r06q_share_kt_r05.csv gpurun_out/r06q_share_kt_r06.csv
