#!/bin/bash
# Round-5 call: GPU suite on the default build (runahead priority on), then one run each of the
# runahead variants against the default (frame + all 8 shards of the 8-way split, sha1 of both),
# then the block-shared runahead variant under a short limit (its first build stalled).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 520 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r05f_gpu_tests.txt 2>&1 \
    || { tail -30 gpurun_out/r05f_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r05f_gpu_tests.txt
REPS=1 bash tools/r05_ab.sh r05f_ab.jsonl default raytracing-hw_amd/v_noprio/librt_hw_amd.so raytracing-hw_amd/v_w4/librt_hw_amd.so \
    raytracing-hw_amd/v_prio2/librt_hw_amd.so raytracing-hw_amd/v_gate30/librt_hw_amd.so raytracing-hw_amd/v_sh48/librt_hw_amd.so default || exit 1
for v in v_share16; do
  RT_LIB=$PWD/raytracing-hw_amd/$v/librt_hw_amd.so timeout -k 5 100 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 2 \
      >> gpurun_out/r05f_share.jsonl 2>>gpurun_out/r05f_share.err || { echo "share variant $v failed or stalled"; exit 1; }
  tail -1 gpurun_out/r05f_share.jsonl
done
