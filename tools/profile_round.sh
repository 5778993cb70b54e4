set -euo pipefail
for w in c2 c3 c4; do
  timeout -k 10 420 bash tools/profile_gpu.sh r3_$w --workload $w
done
echo all-profiles-done
