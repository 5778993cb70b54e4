#!/bin/bash
# Run ON THE GPU BOX: what the box reports about itself (rocm-smi firmware,
# VBIOS, partitions) next to quick C3 / C2 kernel rates, to correlate the
# bimodal C3 box speed with something the box exposes.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/boxinfo_${1:-x}
mkdir -p "$OUT"
(rocm-smi --showvbios --showfwinfo --showmemorypartition --showcomputepartition --showproductname --showdriverversion) > "$OUT/smi.txt" 2>&1 || true
for w in c3 c2; do
  timeout -k 10 180 python3 "$R/bench.py" --workload $w --steps 6 --warmup 2 --no-cpu-baseline --verify none > "$OUT/bench_$w.json" 2>> "$OUT/err.txt" || exit 1
done
echo "boxinfo done"
