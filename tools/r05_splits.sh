#!/bin/bash
# The 2- and 4-way splits of the final build (all shards, slowest = the N-GPU frame), and the
# runahead kernel at up to 4 pixels per lane for the 2-way split (v_ppl4).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/r05_splits.jsonl; : > $out
for w in 4 2; do
  timeout -k 10 150 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 1 --world $w >> $out 2>>$out.err || exit 1
  tail -1 $out
done
RT_LIB=$PWD/raytracing-hw_amd/v_ppl4/librt_hw_amd.so timeout -k 10 150 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 1 --world 2 >> $out 2>>$out.err || exit 1
tail -1 $out
