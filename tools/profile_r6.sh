#!/bin/bash
# Run ON THE GPU BOX: rocprof profiles of the given workloads on one box (the
# shader clock before and after, from rocm-smi), DEEP passes for C3.
#   tools/profile_r6.sh <tag> <workload> ...
set -uo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
(rocm-smi --showclocks; rocm-smi --showperflevel) > "$OUT/smi_before.txt" 2>&1 || true
for w in "$@"; do
  D=0; [ "$w" = c3 ] && D=1
  DEEP=$D timeout -k 10 600 bash "$R/tools/profile_gpu.sh" "${TAG}_$w" --workload "$w" || { echo "profile $w failed" >> "$OUT/status.txt"; exit 1; }
  (rocm-smi --showclocks) > "$OUT/smi_after_$w.txt" 2>&1 || true
  echo "profile $w ok" >> "$OUT/status.txt"
done
echo "profiles done"
