# Kind 1 triangular inverse right-looking over all threads (tree) against one thread per column (ab/colk1, -DDPGO_SNF1_RIGHT=0):
# sweep outputs (device factor) bitwise, then the C5 GNC_TLS + exact bench's factor time and ms/step, alternated twice.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06zi}
lib() { [ $1 = tree ] && echo "" || echo "DPGO_HIP_LIB=$PWD/dpgo_amd/ab/$1/libdpgo_hip.so"; }
for v in tree colk1; do
  env $(lib $v) timeout -k 10 300 python3 -u tools/precond_dump.py gpurun_out/${T}_$v.npz > /dev/null 2>&1 || exit 1
done
python3 tools/precond_dump.py --compare gpurun_out/${T}_tree.npz gpurun_out/${T}_colk1.npz || exit 1
for i in 1 2; do
  for v in tree colk1; do
    env $(lib $v) timeout -k 10 400 python3 -u bench.py --precon exact --robust GNC_TLS --burnin 60 --boundary-leg 0 \
      --exact-leg 0 --cpu-baseline 0 > gpurun_out/${T}_${v}_$i.log 2>&1 || exit 1
    grep '^{' gpurun_out/${T}_${v}_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d['exact_factor']
print('$v', round(d['ms_per_step'],2), round(f['color0']['factor_ms'],1), round(f['color1']['factor_ms'],1))"
  done
done
