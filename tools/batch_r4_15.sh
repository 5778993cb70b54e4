set -e
timeout -k 10 900 python -u -m pytest tests/test_gpu_long_lines.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "filter or c4 or kind4 or keyword" > gpurun_out/seg_parity.log 2>&1
timeout -k 10 300 python bench.py --workload long_c4 --no-cpu-baseline > gpurun_out/seg_long_c4.json 2> gpurun_out/seg_long_c4.err
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --verify windows > gpurun_out/seg_c4.json 2> gpurun_out/seg_c4.err
