#!/bin/bash
# Dump the gfx950 ISA of the scan kernels (for reading waits, spills, loads).
#   tools/isa_dump.sh <outdir> [extra hipcc flags...]
# Writes <outdir>/scan_dfa-hip-amdgcn-amd-amdhsa-gfx950.s and prints per-kernel
# VGPRs / LDS / scratch.
set -euo pipefail
OUT=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd "$OUT"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 "$@" -c "$R/distributed-grep_amd/csrc/kernels/scan_dfa.hip" \
  --save-temps -o "$OUT/scan_dfa.o"
S="$OUT/scan_dfa-hip-amdgcn-amd-amdhsa-gfx950.s"
grep -E "^\s+\.(name|vgpr_count|group_segment_fixed_size|private_segment_fixed_size):" "$S" | paste - - - - |
  grep scan_dfa8 | awk '{print "lds=" $2, "scratch=" $6, "vgpr=" $8, $4}'
