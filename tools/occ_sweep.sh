set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/occ_sweep.jsonl; : > $out
for cfg in "0 3" "0 0" "4 0" "3 0" "2 0" "2 3" "3 3"; do
  set -- $cfg
  for w in 4 8; do
    r=$(RT_MEGA_OCC=$1 RT_MEGA_ORDER_MIN=$2 timeout -k 10 120 python tools/shard_time.py --worlds $w --steps 2 2>>gpurun_out/occ_sweep.err) || exit 1
    echo "{\"occ\": $1, \"order_min\": $2, \"r\": $r}" | tee -a $out
  done
done
