#!/bin/bash
# PMC passes over the X.Q SpMM (one colour class of the 1M-pose grid), edge-stream vs BSR Q.
# Usage (on the GPU box): bash tools/pmc_spmm.sh <outdir> ["counter group" ...]
# One rocprofv3 run per counter group (rocprofv3 does not split counters over passes).
out=${1:-gpurun_out/pmc}
shift || true
mkdir -p "$out"
export TMPDIR=/tmp
groups=("$@")
[ ${#groups[@]} -eq 0 ] && groups=("TA_BUSY_avr GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY")
for fmt in edges bsr; do
  var=1; [ "$fmt" = bsr ] && var=0
  for grp in "${groups[@]}"; do
    tag=$(echo "$grp" | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d "$out/${fmt}_$tag" -o run -- \
      python3 tools/spmm_ab.py --qfmt $fmt --variants $var --rounds 1 --reps 5 > "$out/${fmt}_$tag.log" 2>&1
    rc=$?
    if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then echo "pass $fmt $tag killed (rc=$rc): stopping"; exit $rc; fi
    [ $rc -ne 0 ] && echo "pass $fmt $tag failed rc=$rc"
  done
done
exit 0
