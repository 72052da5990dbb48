#!/bin/bash
# Round-5 call: with the runahead priority, the pixel order (no spread; odd strata reversed) and
# one runahead job per record per pass, against the default; shards of the 8-way split.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/r05j_ab.jsonl; : > $out
for rep in 1 2; do
  for lib in default raytracing-hw_amd/v_nospread/librt_hw_amd.so raytracing-hw_amd/v_snake/librt_hw_amd.so raytracing-hw_amd/v_issue1/librt_hw_amd.so; do
    if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
    timeout -k 10 150 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 2 >> $out 2>>$out.err || exit 1
    tail -1 $out
  done
done
