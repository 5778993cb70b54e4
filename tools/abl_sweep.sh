#!/bin/bash
# Run ON THE GPU BOX: kernel GB/s of one workload's pattern per spec, in order:
#   tools/abl_sweep.sh <tag> <workload> <lib:gib:offset:alloc_gib[:lane_chunk]> ...
# lib = a variant name in distributed-grep_amd/variants/ (or "tree" for the
# in-tree build); offset in bytes; alloc_gib 0 = just the split.
set -uo pipefail
TAG=$1; WL=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abl_$TAG
mkdir -p "$OUT"
for spec in "$@"; do
  IFS=: read -r lib g o a ch <<< "$spec"
  L=$R/distributed-grep_amd/libdgrep.so
  [ "$lib" != tree ] && L=$R/distributed-grep_amd/variants/libdgrep_$lib.so
  # ABL_PATTERN: scan the workload's split with another pattern (ablation only)
  PAT=(); [ -n "${ABL_PATTERN:-}" ] && PAT=(--pattern "$ABL_PATTERN")
  out=$(DGREP_LIB=$L timeout -k 10 180 python3 $R/bench.py --workload $WL --split-gib $g --base-offset ${o:-0} --alloc-gib ${a:-0} --lane-chunk ${ch:-0} --steps 6 --warmup 2 --no-cpu-baseline --verify none "${PAT[@]}" 2>>"$OUT/err.txt") || { echo "$spec FAILED" >> "$OUT/sweep.txt"; exit 1; }
  echo "$spec $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); r=d["roofline"]; print("value=%.0f ms_step=%.4f kernel=%.0f GB/s frac=%.3f kms=%.4f chunk=%d verify_ms=%s" % (d["value"], d["ms_per_step"], r["achieved"], r["frac"], r["kernel_ms_avg"], d["config"]["lane_chunk"], r.get("verify_ms_last")))')" >> "$OUT/sweep.txt"
done
echo "abl done"
