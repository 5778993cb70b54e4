#!/bin/bash
# Run ON THE GPU BOX (via gpurun): kernel trace + PMC passes for one workload.
#   tools/profile_gpu.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/{trace,pmc_*}; copy the summaries into profiles/.
set -euo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# >= 10 timed steps after >= 3 warm-ups: the trace median is then the steady
# state the bench's roofline reports (the average also holds the sizing scan)
BENCH=("$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --verify-windows 0 "$@")
PMC_BENCH=("$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --verify-windows 0 "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "${BENCH[@]}" > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
# PMC passes: one counter group per run (FETCH_SIZE alone: it uses 3 TCC slots)
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "${PMC_BENCH[@]}" > /dev/null 2> "$OUT/pmc_fetch.err"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 "${PMC_BENCH[@]}" > /dev/null 2> "$OUT/pmc_write.err"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d "$OUT/pmc_sq" -o run -- python3 "${PMC_BENCH[@]}" > /dev/null 2> "$OUT/pmc_sq.err"
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/pmc_wait" -o run -- python3 "${PMC_BENCH[@]}" > /dev/null 2> "$OUT/pmc_wait.err"
# DEEP=1: latency / instruction-mix / instruction-cache passes (Little's law:
# SQ_INST_LEVEL_X / SQ_INSTS_X = mean cycles an X instruction is in flight)
if [ "${DEEP:-0}" = 1 ]; then
  timeout -s KILL 150 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d "$OUT/pmc_lat" -o run -- python3 "${PMC_BENCH[@]}" > /dev/null 2> "$OUT/pmc_lat.err"
  timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS_VALU --output-format csv -d "$OUT/pmc_icache" -o run -- python3 "${PMC_BENCH[@]}" > /dev/null 2> "$OUT/pmc_icache.err"
fi
echo "profile done: $OUT"
