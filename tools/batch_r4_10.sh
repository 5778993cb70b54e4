set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/q10_pytest.log 2>&1
DGREP_LIB=$PWD/distributed-grep_amd/variants/libdgrep_c64.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "sheng_adaptive or chunk_edges or lane_chunk or long or overflow or synth_corpus or c5" > gpurun_out/q10_c64_pytest.log 2>&1
bash tools/abl_sweep.sh c64 c2 tree:32 c64:32 tree:16 c64:16 tree:32 c64:32 tree:24 c64:24
for w in c2 c3 c4; do timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --verify windows > gpurun_out/q10_bench_$w.json 2> gpurun_out/q10_bench_$w.err; done
