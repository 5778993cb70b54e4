set -e
O=gpurun_out/pc_sweep.txt; : > $O
for c in 8192 16384 32768 65536; do for dp in 1 2 3; do
  PC_C=$c PC_DEPTH=$dp timeout -k 10 60 tools/pattern_ceiling 16 >> $O 2>&1
done; done
