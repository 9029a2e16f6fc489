# Same-box A/B of the standalone X.Q over library builds (tools/build_variant.py): each build in its own process,
# alternated twice; one JSON line per run (tools/spmm_ab.py, compiled-default edge-stream variant).
#   bash tools/lib_ab_xq.sh OUT.jsonl base dpgo_amd/ab/pad0 dpgo_amd/ab/dma
set -o pipefail
OUT=$1
shift
: > "$OUT"
for round in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = base ]; then L=""; else L="$lib/libdpgo_hip.so"; fi
    line=$(DPGO_HIP_LIB=$L timeout -k 10 180 python3 tools/spmm_ab.py --variants -1 --rounds 3 --reps 20 | tail -1) || exit 1
    echo "{\"lib\": \"$lib\", \"round\": $round, \"run\": $line}" >> "$OUT"
    echo "$lib $round done"
  done
done
