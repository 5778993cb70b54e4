#!/bin/bash
# Run ON THE GPU BOX (via gpurun): the given test files first (new code), then
# the whole GPU suite, then one bench line per workload. Each GPU step has its
# own time limit; the script stops at the first failure.
#   tools/gpu_round.sh <tag> "<test files>" [workload ...]
set -euo pipefail
TAG=$1; FIRST=$2; shift 2
WLS=${@:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
if [ -n "$FIRST" ]; then
  timeout -k 10 600 python -u -m pytest $FIRST -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/first.log" 2>&1
fi
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
for w in $WLS; do
  timeout -k 10 400 python bench.py --workload "$w" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
done
echo "round script done: $OUT"
