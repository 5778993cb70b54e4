#!/bin/bash
# Run ON THE GPU BOX: same-box A/B of the filter long-line kernels
# (variants from tools/build_variants.sh / build_commit_variant.sh), then a
# kernel trace of long_c4 and long_c4p on the in-tree build.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/long_ab
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
REPS=2 timeout -k 10 400 bash "$R/tools/variant_bench.sh" long_c4 ${VARS_C4:-base head seeds1 c0541} > "$OUT/ab_long_c4.txt" 2>&1 || exit 1
REPS=2 timeout -k 10 300 bash "$R/tools/variant_bench.sh" long_c4p ${VARS_C4P:-base head} > "$OUT/ab_long_c4p.txt" 2>&1 || exit 1
for w in long_c4 long_c4p; do
  mkdir -p "$OUT/trace_$w"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$w" -o run -- python3 "$R/bench.py" --workload $w --steps 5 --warmup 2 --no-cpu-baseline --verify none > "$OUT/trace_$w/bench.json" 2> "$OUT/trace_$w/bench.err" || exit 1
done
echo "long ab done"
