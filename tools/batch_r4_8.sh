set -e
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "filter or long or keyword or c4" > gpurun_out/q8_pytest.log 2>&1
timeout -k 10 300 python bench.py --workload long_c4 --no-cpu-baseline --verify full > gpurun_out/bench_long_c4.json 2> gpurun_out/bench_long_c4.err
bash tools/abl_sweep.sh p1 c2 static:12 dyn:12 sprio:12 dprio:12 static:32 dyn:32 sprio:32 dprio:32 static:16 dyn:16 sprio:16 dprio:16
bash tools/abl_sweep.sh k1 c2 dyn:16:0:0:16384 dyn:16:0:0:24576 dyn:16:0:0:28672 dyn:32:0:0:16384 dyn:32:0:0:24576 dyn:12:0:0:16384 dyn:12:0:0:24576
