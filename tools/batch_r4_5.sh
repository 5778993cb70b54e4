set -e
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "filter or long or keyword or partial or c4 or overflow" > gpurun_out/q5_pytest.log 2>&1
DGREP_LIB=$PWD/distributed-grep_amd/variants/libdgrep_pct.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "pair or c3 or parity or golden or long" > gpurun_out/q5_pct_pytest.log 2>&1
REPS=2 bash tools/variant_bench.sh c3 ship pct > gpurun_out/ab_pct_c3.txt 2>&1
timeout -k 10 300 python bench.py --workload long_c4 --no-cpu-baseline --verify full > gpurun_out/bench_long_c4.json 2> gpurun_out/bench_long_c4.err
REPS=2 bash tools/variant_bench.sh c4 fpark nofpark > gpurun_out/ab_fpark_c4.txt 2>&1
bash tools/abl_sweep.sh a1 c2 tree:16:0:0 tree:12:0:16 tree:16:0:32 tree:12:0:0 wg2:12:0:0 wg2:16:0:0 tree:32:0:0 tree:16:0:0
