#!/bin/bash
# Round-5 call: the runahead kernel's shading threshold (48 default vs 40 and 56, shards of the
# 8-way split, two runs each), then the final-build evidence (tools/r05_final_all.sh).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/r05g_shade_ab.jsonl; : > $out
for rep in 1 2; do
  for lib in default raytracing-hw_amd/v_sh40/librt_hw_amd.so raytracing-hw_amd/v_sh56/librt_hw_amd.so; do
    if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
    timeout -k 10 120 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 2 >> $out 2>>$out.err || exit 1
    tail -1 $out
  done
done
unset RT_LIB
bash tools/r05_final_all.sh r05 || exit 1
