#!/bin/bash
# Round-5 call: the plain kernel's occupancy and batch threshold re-tuned after the register
# cuts (RT_UV_RECOMPUTE / RT_INV_RECOMPUTE now default): 4 waves/SIMD (128 VGPRs, 2 spilled),
# the same with 15 LDS stack frames, shading at 40 / 56 READY lanes; frame and shards, 2 runs.
set -o pipefail
cd "$(dirname "$0")/.."
V=raytracing-hw_amd
REPS=2 SHARD_STEPS=1 bash tools/r05_ab.sh r05l_ab.jsonl default $V/v_wpe4/librt_hw_amd.so $V/v_wpe4s15/librt_hw_amd.so \
  $V/v_sh40/librt_hw_amd.so $V/v_sh56/librt_hw_amd.so
