set -e
O=gpurun_out/c3_chunk3.txt; : > $O
for rep in 1 2 3; do for c in 8192 16384; do
  timeout -k 10 200 python bench.py --workload c3 --lane-chunk $c --steps 6 --warmup 2 --no-cpu-baseline --verify none > gpurun_out/c3c.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/c3c.json')); r=d['roofline']; print('chunk=$c', r['achieved'], round(r['frac'],4), d['ms_per_step'])" >> $O
done; done
