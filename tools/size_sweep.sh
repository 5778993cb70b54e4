#!/bin/bash
# Run ON THE GPU BOX: kernel GB/s of one workload's pattern over split sizes
# (and base offsets inside the allocation), in the order given:
#   tools/size_sweep.sh <tag> <workload> <GiB[@offset]> ...
set -uo pipefail
TAG=$1; WL=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/size_$TAG
mkdir -p "$OUT"
for spec in "$@"; do
  g=${spec%@*}; o=0
  [[ "$spec" == *@* ]] && o=${spec#*@}
  out=$(timeout -k 10 180 python3 $R/bench.py --workload $WL --split-gib $g --base-offset $o --steps 6 --warmup 2 --no-cpu-baseline --verify none 2>>"$OUT/err.txt") || { echo "$spec FAILED" >> "$OUT/sweep.txt"; exit 1; }
  echo "gib=$g off=$o $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); r=d["roofline"]; print("kernel=%.0f GB/s frac=%.3f kms=%.3f chunk=%d" % (r["achieved"], r["frac"], r["kernel_ms_avg"], d["config"]["lane_chunk"]))')" >> "$OUT/sweep.txt"
done
echo "sweep done"
