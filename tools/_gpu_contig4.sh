# Contiguous panels (DPGO_PANEL_CONTIG=3) with and without an agent-scope acquire (L2 invalidate) at the start of
# every supernodal kernel (the -DDPGO_SN_ACQUIRE_TEST build in dpgo_amd/ab/acq), twice each.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06zb}
K="test_exact_precondition"
for i in 1 2; do
  for v in base acq; do
    L=""; [ $v = acq ] && L="DPGO_HIP_LIB=$PWD/dpgo_amd/ab/acq/libdpgo_hip.so"
    env $L DPGO_PANEL_CONTIG=3 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_precon_exact.py -m gpu -q \
      -k "$K" --timeout 250 --timeout-method thread > gpurun_out/${T}_${v}_$i.log 2>&1
    echo "$v run $i rc=$? $(grep -E 'passed|failed' gpurun_out/${T}_${v}_$i.log | tail -1) $(grep -E '^FAILED' gpurun_out/${T}_${v}_$i.log | head -3 | tr '\n' ' ')"
  done
done
