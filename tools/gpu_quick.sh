#!/bin/bash
# Run ON THE GPU BOX (via gpurun): the GPU tests selected by a pytest -k
# expression ("-": none), then bench lines without the CPU baseline and with
# full-split parity, for quick A/B work. Stops at the first failure.
#   tools/gpu_quick.sh <tag> <k-expr|-> [workload ...]
set -euo pipefail
TAG=$1; shift; K=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/q_$TAG
mkdir -p "$OUT"
cd "$R"
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "$K" \
    > "$OUT/pytest_gpu.log" 2>&1
fi
for w in "$@"; do
  timeout -k 10 300 python bench.py --workload "$w" --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
done
echo "quick done: $OUT"
