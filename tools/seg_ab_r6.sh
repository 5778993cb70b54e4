#!/bin/bash
# Run ON THE GPU BOX: same-box A/B of long_dfa_seg1_kernel variants on the
# filter long-line workloads, plus an SQ/LDS counter pass per variant.
#   VARS="base cls8" tools/seg_ab_r6.sh <tag>
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-seg_ab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
VARS=${VARS:-base cls8}
REPS=2 timeout -k 10 400 bash "$R/tools/variant_bench.sh" long_c4 $VARS $VARS > "$OUT/ab_long_c4.txt" 2>&1 || exit 1
REPS=1 timeout -k 10 300 bash "$R/tools/variant_bench.sh" long_c4p $VARS $VARS > "$OUT/ab_long_c4p.txt" 2>&1 || exit 1
for v in $VARS; do
  DGREP_LIB=$R/distributed-grep_amd/variants/libdgrep_$v.so timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d "$OUT/pmc_$v" -o run -- python3 "$R/bench.py" --workload long_c4 --steps 2 --warmup 1 --no-cpu-baseline --verify none > /dev/null 2> "$OUT/pmc_$v.err" || exit 1
done
echo "seg ab done"
