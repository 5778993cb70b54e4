#!/bin/bash
# Run ON THE GPU BOX (via gpurun): GPU parity suite, then bench lines for the
# given workloads (default c2). Every GPU step has its own time limit and the
# script stops at the first failure.
#   tools/gpu_check.sh <tag> [workload ...]
set -euo pipefail
TAG=$1; shift
WLS=${@:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/check_$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
for w in $WLS; do
  timeout -k 10 300 python bench.py --workload "$w" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
done
echo "check done: $OUT"
