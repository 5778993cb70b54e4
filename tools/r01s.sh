#!/bin/bash
# r01s: non-temporal split loads per stepper, with FETCH_SIZE for C4 (run ON the GPU box)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r01s; mkdir -p $O; cd $R
timeout -k 10 300 tools/variant_bench.sh c4 base wnt > $O/var_c4.txt 2>&1 || exit 1
timeout -k 10 300 tools/variant_bench.sh c3 base tnt > $O/var_c3.txt 2>&1 || exit 1
timeout -k 10 300 tools/variant_bench.sh c2 base snt > $O/var_c2.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in base wnt; do
  DGREP_LIB=$R/distributed-grep_amd/variants/libdgrep_$v.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$v -o run -- python3 $R/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --verify-windows 0 > /dev/null 2> $O/pmc_$v.err || exit 1
done
echo done
