set -e
O=gpurun_out/c3_chunk.txt; : > $O
for rep in 1 2; do for c in 16384 32768 8192; do
  timeout -k 10 200 python bench.py --workload c3 --lane-chunk $c --steps 6 --warmup 2 --no-cpu-baseline --verify none > gpurun_out/c3c.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/c3c.json')); r=d['roofline']; print('chunk=$c', d['config']['lane_chunk'], r['achieved'], round(r['frac'],4), d['ms_per_step'], r.get('overflow_ms_avg'))" >> $O
done; done
