#!/bin/bash
# One GPU call: parity suite + bench lines, then variant A/B and a profile.
#   tools/r02_round.sh <tag> "<workloads>" "<variant workload>" "<variants>" [profile workload]
set -euo pipefail
TAG=$1; WLS=$2; VW=$3; VARS=$4; PW=${5:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_check.sh "$TAG" $WLS
if [ -n "$VARS" ]; then
  REPS=2 timeout -k 10 600 bash tools/variant_bench.sh "$VW" $VARS > "gpurun_out/check_$TAG/variants_$VW.txt" 2>&1
fi
if [ -n "$PW" ]; then
  timeout -k 10 900 bash tools/profile_gpu.sh "${TAG}_$PW" --workload "$PW"
fi
echo "round script done"
