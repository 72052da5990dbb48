#!/bin/bash
# Runahead on and off for each library (tools/runahead_ab.py --off 1): 1-GPU frame + all 8 shards.
#   bash tools/ab_r03_off.sh TAG default raytracing-hw_amd/vX/librt_hw_amd.so ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
out=gpurun_out/ab_$TAG.jsonl; : > $out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  timeout -k 10 300 python tools/runahead_ab.py --off 1 --worlds ${AB_WORLDS:-8} --steps ${AB_STEPS:-2} \
      >> $out 2>>gpurun_out/ab_$TAG.err || exit 1
  tail -1 $out
done
