#!/bin/bash
# A/B the tuning variants built by tools/build_variants.sh (run ON the GPU box).
#   tools/variant_bench.sh <workload> [variant ...]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
WL=${1:-c2}; shift || true
VARS=${@:-base}
for v in $VARS; do
  for rep in $(seq ${REPS:-2}); do
    out=$(DGREP_LIB=$R/distributed-grep_amd/variants/libdgrep_$v.so timeout -k 10 180 python3 $R/bench.py --workload $WL --steps 6 --warmup 2 --no-cpu-baseline --verify none 2>/dev/null) || { echo "$v FAILED"; exit 1; }
    echo "$v rep$rep $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); r=d["roofline"]; print("value=%.0f kernel=%.0f GB/s frac=%.3f kms=%.3f overflow_ms=%.3f chunk=%d stepper=%s ms_step=%.3f" % (d["value"], r["achieved"], r["frac"], r["kernel_ms_avg"], r["overflow_ms_last"], d["config"]["lane_chunk"], d["config"]["stepper"], d["ms_per_step"]))')"
  done
done
