#!/bin/bash
# Run ON THE GPU BOX: same-box lane-chunk sweeps (C3 pair 7/8/9 KiB, C4
# filter 16-32 KiB) and the bare access pattern (tools/pattern_ceiling) at the
# same chunks, to tell a memory-system effect from a kernel one.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/chunk_r6
mkdir -p "$OUT"
timeout -k 10 400 bash "$R/tools/abl_sweep.sh" c3chunkB c3 tree:16:0:0:8192 tree:16:0:0:7168 tree:16:0:0:9216 tree:16:0:0:8192 tree:16:0:0:7168 tree:16:0:0:9216 || exit 1
for c in 7168 8192 9216 6144 5120; do
  PC_LDS=43024 PC_C=$c timeout -k 10 120 "$R/tools/pattern_ceiling" 16 >> "$OUT/pattern_pair.txt" 2>&1 || exit 1
done
for c in 32768 28672 30720 24576; do
  PC_LDS=53248 PC_C=$c timeout -k 10 120 "$R/tools/pattern_ceiling" 16 >> "$OUT/pattern_sheng.txt" 2>&1 || exit 1
done
timeout -k 10 400 bash "$R/tools/abl_sweep.sh" c4chunk c4 tree:16:0:0:32768 tree:16:0:0:30720 tree:16:0:0:28672 tree:16:0:0:24576 tree:16:0:0:16384 tree:16:0:0:32768 || exit 1
echo "chunk sweep done"
