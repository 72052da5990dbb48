#!/bin/bash
# Round-5 call: GPU suite on the final build, the 2- and 4-way splits, and the block-shared
# runahead (each run under a short limit; a stall is reported by the diagnostics build).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 520 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r05h_gpu_tests.txt 2>&1 \
    || { tail -30 gpurun_out/r05h_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r05h_gpu_tests.txt
bash tools/r05_splits.sh || exit 1
out=gpurun_out/r05h_share.jsonl; : > $out
for v in v_share16 v_share64; do
  RT_LIB=$PWD/raytracing-hw_amd/$v/librt_hw_amd.so timeout -k 5 90 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 2 >> $out 2>>$out.err
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "share variant $v: rc $rc; diagnostics build:"
    RT_LIB=$PWD/raytracing-hw_amd/v_share_dbg/librt_hw_amd.so timeout -k 5 90 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 1 \
        > gpurun_out/r05h_share_dbg.txt 2>&1
    grep -m 40 "share stall" gpurun_out/r05h_share_dbg.txt
    exit 1
  fi
  tail -1 $out
done
RT_LIB=$PWD/raytracing-hw_amd/prof_share/librt_hw_amd.so timeout -k 10 120 python3 tools/shard_time.py --worlds 8 --steps 1 \
    > gpurun_out/r05h_megaprof_w8_share.txt 2>&1 || exit 1
echo done
