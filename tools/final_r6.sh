#!/bin/bash
# Run ON THE GPU BOX: the round's final bench lines (every record checked
# against the oracle) for the BASELINE configs and the long-line workloads,
# then a C3 lane-chunk check. Writes gpurun_out/final_r6/.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${FINAL_TAG:-final_r6}
mkdir -p "$OUT"
for w in c2 c3 c4 c5 c1 long long_c4 long_c4p; do
  timeout -k 10 420 python3 "$R/bench.py" --workload $w --steps 10 --warmup 3 > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { echo "bench $w failed" >> "$OUT/status.txt"; exit 1; }
  echo "bench $w ok" >> "$OUT/status.txt"
done
timeout -k 10 300 bash "$R/tools/abl_sweep.sh" ${FINAL_TAG:-final_r6}_chunk c3 tree:16:0:0:9216 tree:16:0:0:7168 tree:16:0:0:9216 tree:16:0:0:7168 || exit 1
echo "final done"
