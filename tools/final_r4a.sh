#!/bin/bash
# Round-4 final measurements, part A (run ON THE GPU BOX): GPU suite, then bench
# lines with full-split parity and the CPU baselines for the BASELINE configs.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fin4
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
for w in c2 c3 c4 c5 c1; do
  timeout -k 10 300 python bench.py --workload "$w" > "$O/bench_$w.json" 2> "$O/bench_$w.err"
done
echo "final A done"
