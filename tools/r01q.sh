#!/bin/bash
# r01q: table stepper block size A/B on C3 with HBM fetch counters (run ON the GPU box)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r01q; mkdir -p $O; cd $R
timeout -k 10 300 tools/variant_bench.sh c3 base tb128w2 > $O/var_c3.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in base tb128w2; do
  DGREP_LIB=$R/distributed-grep_amd/variants/libdgrep_$v.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$v -o run -- python3 $R/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --verify-windows 0 > /dev/null 2> $O/pmc_$v.err || exit 1
done
echo done
