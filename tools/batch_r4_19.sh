set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/q19_pytest.log 2>&1
timeout -k 10 300 python bench.py --workload c3 > gpurun_out/q19_c3.json 2> gpurun_out/q19_c3.err
