#!/bin/bash
# Run ON THE GPU BOX: the round's final bench lines (every record checked
# against the oracle) for the BASELINE configs and the long-line ablations,
# then the GPU suite. Writes gpurun_out/final_r5/.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final_r5
mkdir -p "$OUT"
for w in c2 c3 c4 c5 c1 long long_c4; do
  timeout -k 10 300 python3 "$R/bench.py" --workload $w --steps 10 --warmup 3 > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { echo "bench $w failed" >> "$OUT/status.txt"; exit 1; }
  echo "bench $w ok" >> "$OUT/status.txt"
done
echo "benches done"
