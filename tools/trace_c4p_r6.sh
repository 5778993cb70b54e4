#!/bin/bash
# Run ON THE GPU BOX: kernel traces of long_c4p with the in-tree build (64 KiB
# filter chunks) and the f32 variant (32 KiB), same box.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trace_c4p
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in tree f32; do
  L=$R/distributed-grep_amd/libdgrep.so; [ $v != tree ] && L=$R/distributed-grep_amd/variants/libdgrep_$v.so
  mkdir -p "$OUT/$v"
  DGREP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run -- python3 "$R/bench.py" --workload long_c4p --steps 4 --warmup 1 --no-cpu-baseline --verify none > "$OUT/$v/bench.json" 2> "$OUT/$v/bench.err" || exit 1
done
echo "trace done"
