#!/bin/bash
# Run ON THE GPU BOX: kernel GB/s of one workload's pattern over split sizes
# (tail rounds vs size effects): tools/size_sweep.sh <tag> <workload> <GiB ...>
set -uo pipefail
TAG=$1; WL=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/size_$TAG
mkdir -p "$OUT"
for g in "$@"; do
  out=$(timeout -k 10 180 python3 $R/bench.py --workload $WL --split-gib $g --steps 6 --warmup 2 --no-cpu-baseline --verify none 2>>"$OUT/err.txt") || { echo "$g FAILED" >> "$OUT/sweep.txt"; exit 1; }
  echo "gib=$g $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); r=d["roofline"]; print("kernel=%.0f GB/s frac=%.3f kms=%.3f tiles_per_wave=%s chunk=%d" % (r["achieved"], r["frac"], r["kernel_ms_avg"], "-", d["config"]["lane_chunk"]))')" >> "$OUT/sweep.txt"
done
echo "sweep done"
