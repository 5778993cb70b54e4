#!/bin/bash
# Run ON THE GPU BOX: the whole GPU suite on the in-tree build, then a same-box
# A/B of variant libraries (distributed-grep_amd/variants/libdgrep_<v>.so).
#   tools/gpu_ab_round.sh <tag> "<workloads>" "<variants>"
set -euo pipefail
TAG=$1; WLS=$2; VARS=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abr_$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
for w in $WLS; do
  REPS=${REPS:-3} timeout -k 10 600 bash "$R/tools/variant_bench.sh" "$w" $VARS > "$OUT/$w.txt" 2>&1
done
echo "ab round done: $OUT"
