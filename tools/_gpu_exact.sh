# Exact-preconditioner legs at C5 (the reference's default configuration): the bench line and a rocprofv3 kernel
# trace of the same run restricted to the timed steps.  bash tools/_gpu_exact.sh TAG
set -o pipefail
TAG=${1:-r06}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py --precon exact --robust GNC_TLS --burnin 60 --boundary-leg 0 --exact-leg 0 \
  > gpurun_out/${TAG}_bench_exact_gnc.log 2>&1 || exit 1
tail -c 400 gpurun_out/${TAG}_bench_exact_gnc.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_exact -o run -- python3 bench.py --precon exact \
  --robust GNC_TLS --burnin 60 --cpu-baseline 0 --boundary-leg 0 --exact-leg 0 > gpurun_out/${TAG}_exact_kt.log 2>&1 || exit 1
python3 tools/rocpd_stats.py gpurun_out/prof_${TAG}_exact > gpurun_out/${TAG}_exact_kernel_stats.csv 2>&1 || exit 1
head -12 gpurun_out/${TAG}_exact_kernel_stats.csv
python3 tools/sweep_levels.py gpurun_out/prof_${TAG}_exact > gpurun_out/${TAG}_sweep_levels.txt 2>&1
rm -rf gpurun_out/prof_${TAG}_exact  # the database exceeds what gpurun copies back
