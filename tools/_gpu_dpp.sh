# The sweeps' cross-lane sums by DPP / permlane swaps (tree) against ds_bpermute shuffles (dpgo_amd/ab/shfl, built with
# -DDPGO_SN_DPP_SUMS=0): outputs compared bitwise, C5 colour-0 sweeps alternated twice, then the exact tests.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06zd}
timeout -k 10 300 python3 -u tools/precond_dump.py gpurun_out/${T}_dpp.npz || exit 1
DPGO_HIP_LIB=$PWD/dpgo_amd/ab/shfl/libdpgo_hip.so timeout -k 10 300 python3 -u tools/precond_dump.py gpurun_out/${T}_shfl.npz || exit 1
python3 tools/precond_dump.py --compare gpurun_out/${T}_dpp.npz gpurun_out/${T}_shfl.npz || exit 1
for i in 1 2; do
  for v in dpp shfl; do
    L=""; [ $v = shfl ] && L="DPGO_HIP_LIB=$PWD/dpgo_amd/ab/shfl/libdpgo_hip.so"
    env $L timeout -k 10 300 python3 -u tools/sweep_ab.py --rounds 3 --reps 5 > gpurun_out/${T}_${v}_$i.json \
      2> gpurun_out/${T}_${v}_$i.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/${T}_${v}_$i.json')); m=list(d['ms'].values())[0]; print('$v', round(m['fwd'],3), round(m['bwd'],3))"
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -x -q --timeout 500 --timeout-method thread \
  > gpurun_out/${T}_exact_tests.log 2>&1 || { tail -5 gpurun_out/${T}_exact_tests.log; exit 1; }
tail -1 gpurun_out/${T}_exact_tests.log
