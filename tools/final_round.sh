#!/bin/bash
# Run ON THE GPU BOX: GPU suite, bench lines (full-split parity + CPU baseline)
# and rocprof profiles of the shipped build, each step under its own limit.
#   tools/final_round.sh <tag> "<bench workloads>" "<profiled workloads>"
set -euo pipefail
TAG=$1; WLS=$2; PWLS=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
for w in $WLS; do
  timeout -k 10 240 python bench.py --workload "$w" > "$O/bench_$w.json" 2> "$O/bench_$w.err"
done
for w in $PWLS; do
  timeout -k 10 400 bash tools/profile_gpu.sh "${TAG}_$w" --workload "$w"
done
echo "final round done: $O"
