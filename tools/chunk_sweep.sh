#!/bin/bash
# Lane-chunk sweep of the adaptive steppers (Sheng, pair, filter) through
# dgrep_set_lane_chunk (run ON the GPU box). REPS (default 2) runs per chunk.
#   tools/chunk_sweep.sh <workload> [chunk ...]   (0 = adaptive)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
WL=${1:-c2}; shift || true
for ch in ${@:-0 4096 8192 14592 16384}; do
  for rep in $(seq ${REPS:-2}); do
    out=$(timeout -k 10 180 python3 $R/bench.py --workload $WL --steps 6 --warmup 2 --no-cpu-baseline --verify-windows 3 --lane-chunk $ch 2>/dev/null) || { echo "$ch FAILED"; exit 1; }
    echo "chunk=$ch rep$rep $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); r=d["roofline"]; print("value=%.0f kernel=%.0f GB/s frac=%.3f kms=%.3f overflow_ms=%.3f verify_ms=%.3f ovf_lanes=%d chunk=%d stepper=%s verified=%s" % (d["value"], r["achieved"], r["frac"], r["kernel_ms_avg"], r["overflow_ms_last"], r["verify_ms_last"], r["overflow_lanes"], d["config"]["lane_chunk"], d["config"]["stepper"], d["config"]["verified_windows"]))')"
  done
done
