#!/bin/bash
# Round-5 A/B of the coop step's memory-request knobs (rt_wavefront.h): the 1-GPU frame (with
# its float frame's sha1) and every shard of the 8-way split, per library, in one call.
#   bash tools/r05_memreq.sh default raytracing-hw_amd/v_mask/librt_hw_amd.so ...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/r05_memreq_ab.jsonl; : > $out
for rep in 1 2; do
for lib in "$@"; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  timeout -k 10 240 python3 tools/order_ab.py --natural 0 --steps 2 --shard-steps 2 >> $out 2>>gpurun_out/r05_memreq.err || { echo "failed: $lib"; exit 1; }
  tail -1 $out
done
done
