#!/bin/bash
# Run ON THE GPU BOX: the bare scan access pattern (tools/pattern_ceiling) over
# lane chunk sizes, at the pair kernel's LDS (3 x 43 KiB) and the Sheng
# kernel's (3 x 52 KiB), 16 GiB.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pattern_sweep
mkdir -p "$OUT"
for c in 4096 4608 5120 5632 6144 6656 7168 7680 8192 8704 9216 9728 10240 11264 12288; do
  PC_LDS=43024 PC_C=$c timeout -k 10 60 "$R/tools/pattern_ceiling" 16 | grep lanechunk >> "$OUT/pair.txt" || exit 1
done
for c in 16384 20480 24576 28672 32768 36864 40960 49152 65536; do
  PC_LDS=53248 PC_C=$c timeout -k 10 60 "$R/tools/pattern_ceiling" 16 32 | grep lanechunk >> "$OUT/sheng.txt" || exit 1
done
echo "pattern sweep done"
