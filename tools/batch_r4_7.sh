set -e
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "filter or long or keyword or c4 or overflow" > gpurun_out/q7_pytest.log 2>&1
timeout -k 10 300 python bench.py --workload long_c4 --no-cpu-baseline --verify full > gpurun_out/bench_long_c4.json 2> gpurun_out/bench_long_c4.err
bash tools/abl_sweep.sh d2 c2 static:12:0:0 dyn:12:0:0 static:12:0:0 dyn:12:0:0 static:32:0:0 dyn:32:0:0 dyn:16:0:0 static:16:0:0 dyn:8:0:0 static:8:0:0
