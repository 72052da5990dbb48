#!/bin/bash
# tools/order_ab.py for each library given ("default" = the in-tree build), one JSON line each.
#   bash tools/order_ab.sh default raytracing-hw_amd/v1/librt_hw_amd.so ...
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/order_ab.jsonl; : > $out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  timeout -k 10 200 python tools/order_ab.py ${ORDER_AB_ARGS:-} 2>>gpurun_out/order_ab.err | tee -a $out || exit 1
done
