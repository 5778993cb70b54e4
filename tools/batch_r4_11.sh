set -e
for w in c2 c3 c5; do timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --verify windows > gpurun_out/q11_bench_$w.json 2> gpurun_out/q11_bench_$w.err; done
REPS=2 bash tools/variant_bench.sh c3 ship pcf > gpurun_out/ab_pcf_c3.txt 2>&1
