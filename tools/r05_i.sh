#!/bin/bash
# Round-5 call: with the runahead priority, window 2 and 8 coop leaf records in the runahead
# kernel, and row-major order at 8-way (no pre-pass), against the default.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/r05i_ab.jsonl; : > $out
for rep in 1 2; do
  for lib in default raytracing-hw_amd/v_w2/librt_hw_amd.so raytracing-hw_amd/v_c8/librt_hw_amd.so; do
    if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
    timeout -k 10 120 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 2 >> $out 2>>$out.err || exit 1
    tail -1 $out
  done
done
unset RT_LIB
timeout -k 10 150 python3 tools/order_ab.py --natural 1 --full 1 --steps 1 --shard-steps 1 >> $out 2>>$out.err || exit 1
tail -1 $out
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05i_smoke.txt 2>&1 || { tail -5 gpurun_out/r05i_smoke.txt; exit 1; }
tail -1 gpurun_out/r05i_smoke.txt
