#!/bin/bash
# Runahead A/B over compile-time variants (make -C raytracing-hw_amd variant VDIR=var/NAME
# VFLAGS=...): 4- and 8-way shards of the headline frame, runahead on, one line per library.
#   bash tools/runahead_variants.sh default raytracing-hw_amd/var/w4fix/librt_hw_amd.so ...
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/runahead_variants.jsonl; : > $out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  timeout -k 10 200 python -u tools/runahead_ab.py --off 0 --steps 1 --worlds ${WORLDS:-4,8} >> $out 2>>gpurun_out/runahead_variants.err || exit 1
done
