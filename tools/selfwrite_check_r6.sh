#!/bin/bash
# Run ON THE GPU BOX: verification without self-writes against HEAD (same
# box), the GPU suite, then C4's bench line with full parity.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/selfwrite
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 1
REPS=2 timeout -k 10 300 bash "$R/tools/variant_bench.sh" c4 base old base old > "$OUT/ab_c4.txt" 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c4 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || exit 1
echo "selfwrite done"
