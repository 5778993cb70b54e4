#!/bin/bash
# r01k: A/B of the tuning variants (chunk padding, two chunks per lane) for C2/C3/C4 (run ON the GPU box)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r01k; mkdir -p $O; cd $R
timeout -k 10 400 tools/variant_bench.sh c3 base ts2 tp > $O/var_c3.txt 2>&1 || exit 1
timeout -k 10 400 tools/variant_bench.sh c4 base ws2 wp > $O/var_c4.txt 2>&1 || exit 1
timeout -k 10 400 tools/variant_bench.sh c2 base s2 sp33 > $O/var_c2.txt 2>&1 || exit 1
echo done
