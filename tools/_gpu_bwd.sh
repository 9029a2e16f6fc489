# k_sn_bwd with the gather's pose ids one tile ahead (tree: natural registers; ab/pidw3: a 3-wave budget) against the
# one-step gather (ab/old, -DDPGO_SNB_PID_AHEAD=0): outputs bitwise, C5 colour-0 sweeps alternated twice, exact tests.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06ze}
lib() { [ $1 = tree ] && echo "" || echo "DPGO_HIP_LIB=$PWD/dpgo_amd/ab/$1/libdpgo_hip.so"; }
for v in tree pidw3 old; do
  env $(lib $v) timeout -k 10 300 python3 -u tools/precond_dump.py gpurun_out/${T}_$v.npz > /dev/null 2>&1 || exit 1
done
python3 tools/precond_dump.py --compare gpurun_out/${T}_tree.npz gpurun_out/${T}_old.npz || exit 1
python3 tools/precond_dump.py --compare gpurun_out/${T}_pidw3.npz gpurun_out/${T}_old.npz || exit 1
for i in 1 2; do
  for v in tree pidw3 old; do
    env $(lib $v) timeout -k 10 300 python3 -u tools/sweep_ab.py --rounds 3 --reps 5 > gpurun_out/${T}_${v}_$i.json \
      2> gpurun_out/${T}_${v}_$i.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/${T}_${v}_$i.json')); m=list(d['ms'].values())[0]; print('$v', round(m['fwd'],3), round(m['bwd'],3))"
  done
done
