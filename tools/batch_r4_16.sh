set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/q16_pytest.log 2>&1
for w in long long1g c2 c5; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/q16_$w.json 2> gpurun_out/q16_$w.err
done
