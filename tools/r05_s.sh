#!/bin/bash
# Round-5 call: the 4-way split (2 pixels per lane) on the runahead kernel (default) or on the
# plain kernel (v_ppl1: runahead only at <= 1 pixel per lane), now that the plain kernel is 8%
# faster; all shards, two runs each.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/r05s_split4.jsonl; : > $out
for rep in 1 2; do
  for lib in default raytracing-hw_amd/v_ppl1/librt_hw_amd.so; do
    if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
    timeout -k 10 150 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 1 --world 4 >> $out 2>>$out.err || exit 1
    tail -1 $out
  done
done
