set -e
L=$PWD/distributed-grep_amd/variants/libdgrep_u16.so
DGREP_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "pair or c3 or synth_corpus or edge_inputs or random_small" > gpurun_out/u16_parity.log 2>&1
REPS=2 timeout -k 10 900 bash tools/variant_bench.sh c3 ship u16 ship u16 > gpurun_out/ab_u16_c3.txt 2>&1
