set -e
REPS=2 timeout -k 10 900 bash tools/variant_bench.sh c2 ship w4 w4b w5 w5b ship > gpurun_out/ab_occ_c2.txt 2>&1
REPS=1 timeout -k 10 400 bash tools/variant_bench.sh c5 ship w4b ship > gpurun_out/ab_occ_c5.txt 2>&1
