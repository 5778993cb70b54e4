#!/bin/bash
# Run ON THE GPU BOX: the 3.5/7 KiB pair chunk against the 4/8 KiB build
# (same box), the GPU suite, then C3's bench line with full-split parity.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/p7
mkdir -p "$OUT"
REPS=2 timeout -k 10 400 bash "$R/tools/variant_bench.sh" c3 base p8 base p8 > "$OUT/ab_c3.txt" 2>&1 || exit 1
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c3 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || exit 1
echo "p7 check done"
