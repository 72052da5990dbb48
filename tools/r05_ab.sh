#!/bin/bash
# Round-5 A/B of library builds: the 1-GPU frame (float frame sha1) and every shard of the
# 8-way split (their sha1 too), per library, REPS times, in one call.
#   bash tools/r05_ab.sh OUT.jsonl default raytracing-hw_amd/v1/librt_hw_amd.so ...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/$1; shift; : > $out
for rep in $(seq ${REPS:-2}); do
for lib in "$@"; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  timeout -k 10 240 python3 tools/order_ab.py --natural 0 --steps 2 --shard-steps ${SHARD_STEPS:-2} >> $out 2>>$out.err || { echo "failed: $lib"; tail -5 $out.err; exit 1; }
  tail -1 $out
done
done
