#!/bin/bash
# A/B of library builds on the headline frame: the 1-GPU frame and all 8 shards of the 8-way
# split (tools/runahead_ab.py, runahead on), one JSON line per library.
#   bash tools/ab_r03.sh TAG default raytracing-hw_amd/v0/librt_hw_amd.so ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
out=gpurun_out/ab_$TAG.jsonl; : > $out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  timeout -k 10 240 python tools/runahead_ab.py --off 0 --worlds ${AB_WORLDS:-8} --steps ${AB_STEPS:-2} \
      >> $out 2>>gpurun_out/ab_$TAG.err || exit 1
  tail -1 $out
done
