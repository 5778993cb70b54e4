#!/bin/bash
# Same-box A/B of variant libraries over several workloads (run ON the GPU box):
#   tools/ab.sh <tag> "<workloads>" "<variants>"
set -euo pipefail
TAG=$1; WLS=$2; VARS=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p "$OUT"
for w in $WLS; do
  REPS=${REPS:-2} timeout -k 10 600 bash "$R/tools/variant_bench.sh" "$w" $VARS > "$OUT/$w.txt" 2>&1
done
echo "ab done"
