#!/bin/bash
# Round-5 call on the final build: the idle-lane regression test (the r05m / r05n fault
# sequence); the bench line again, now that profiles/ holds this build's counter passes
# (roofline.traffic, issue); the 2- and 4-way splits; then the plain kernel's step knobs
# re-tuned on the packed build: leaf rounds while >= 4 / 16 leaf lanes are unserved (8 now),
# 3 stack pops per step (2 now), shading at 52 READY lanes (48 now); frame and shards, two runs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -k idle_lanes -x -v --timeout 120 --timeout-method thread > gpurun_out/r05q_idle_test.txt 2>&1 || { tail -20 gpurun_out/r05q_idle_test.txt; exit 1; }
tail -2 gpurun_out/r05q_idle_test.txt
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r05_bench2.json 2> gpurun_out/r05_bench2.err || { tail -5 gpurun_out/r05_bench2.err; exit 1; }
tail -c 400 gpurun_out/r05_bench2.json
: > gpurun_out/r05q_splits.jsonl
for w in 4 2; do
  timeout -k 10 150 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 1 --world $w >> gpurun_out/r05q_splits.jsonl 2>>gpurun_out/r05q_splits.err || exit 1
  tail -1 gpurun_out/r05q_splits.jsonl
done
V=raytracing-hw_amd
REPS=2 SHARD_STEPS=1 bash tools/r05_ab.sh r05q_ab.jsonl default $V/v_rm4/librt_hw_amd.so $V/v_rm16/librt_hw_amd.so \
  $V/v_pops3/librt_hw_amd.so $V/v_sh52/librt_hw_amd.so
