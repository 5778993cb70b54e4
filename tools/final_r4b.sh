#!/bin/bash
# Round-4 final measurements, part B: long-line workloads (full-split parity),
# then rocprof kernel traces + PMC passes for C2 / C3 / C4 / C5.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fin4
mkdir -p "$O"
cd "$R"
for w in long long1g long_c4; do
  timeout -k 10 300 python bench.py --workload "$w" --no-cpu-baseline > "$O/bench_$w.json" 2> "$O/bench_$w.err"
done
for w in ${PROFILE_WLS:-c2 c3 c4 c5}; do
  timeout -k 10 400 bash tools/profile_gpu.sh "fin4_$w" --workload "$w"
done
echo "final B done"
