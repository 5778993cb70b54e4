#!/bin/bash
# r01i: chunk-padding (HBM channel spread) and two-stream A/B, plus microbench (run ON the GPU box)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r01i; mkdir -p $O; cd $R
for c in 1024 1088 4096 4224; do
  timeout -k 10 120 tools/microbench_scan 8 $c > $O/mb_$c.txt 2>&1 || { echo "mb $c failed"; exit 1; }
done
timeout -k 10 600 tools/variant_bench.sh c2 base sp33 sp31 s2 > $O/var_c2.txt 2>&1 || exit 1
timeout -k 10 400 tools/variant_bench.sh c3 base tp ts2 > $O/var_c3.txt 2>&1 || exit 1
timeout -k 10 400 tools/variant_bench.sh c4 base wp ws2 > $O/var_c4.txt 2>&1 || exit 1
echo done
