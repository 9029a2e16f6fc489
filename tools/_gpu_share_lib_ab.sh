# Same-box A/B of the 8-GPU share (k = 50, 8 agents) between library builds (DPGO_HIP_LIB), alternated twice:
#   bash tools/_gpu_share_lib_ab.sh TAG name1=path1 name2=path2 ...   ("tree" = the tree's own library)
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
for i in a b; do
  for nv in "$@"; do
    name=${nv%%=*}; lib=${nv#*=}
    if [ "$lib" = tree ]; then L=""; else L="DPGO_HIP_LIB=$PWD/$lib"; fi
    env $L timeout -k 10 300 python3 -u bench.py --k 50 --agents-per-axis 2 --steps 200 --cpu-baseline 0 \
      --boundary-leg 0 --exact-leg 0 > gpurun_out/${T}_${name}_$i.log 2>&1 || exit 1
    grep '^{' gpurun_out/${T}_${name}_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['roofline']['in_step_spmm']
print('$name', round(d['ms_per_step'],4), {k: round(v['avg_ms']*1e3,1) for k,v in s.items()})"
  done
done
