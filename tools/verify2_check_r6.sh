#!/bin/bash
# Run ON THE GPU BOX: two-pass verification (mark, then compact) against the
# one-wave-per-tile build (same box), the GPU suite, then the filter
# workloads' bench lines with full parity.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/verify2
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 1
REPS=2 timeout -k 10 300 bash "$R/tools/variant_bench.sh" c4 base old base old > "$OUT/ab_c4.txt" 2>&1 || exit 1
REPS=1 timeout -k 10 300 bash "$R/tools/variant_bench.sh" long_c4p base old base old > "$OUT/ab_long_c4p.txt" 2>&1 || exit 1
for w in c4 long_c4p; do
  timeout -k 10 300 python3 bench.py --workload $w > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || exit 1
done
echo "verify2 done"
