set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/q9_pytest.log 2>&1
timeout -k 10 300 python bench.py --workload long_c4 --no-cpu-baseline --verify full > gpurun_out/bench_long_c4.json 2> gpurun_out/bench_long_c4.err
bash tools/abl_sweep.sh m1 c2 mt2:12 mt5:12 mt2:8 mt5:8 mt2:16 mt5:16
bash tools/abl_sweep.sh m1c4 c4 mt2:16 mt5:16 mt2:16 mt5:16
bash tools/abl_sweep.sh m1c3 c3 mt5:16 mt5:16:0:0:32768 mt5:16:0:0:8192
