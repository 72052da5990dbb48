#!/bin/bash
# Round-5 call: the runahead kernel (8-way shards) after the register work: 5 waves/SIMD with 11
# LDS stack frames (96 VGPRs, 48 spilled; 72 before round 5's changes), the same with the shading
# pass's packing (46), and the packing at 4 waves/SIMD; shards and frame, two runs.
set -o pipefail
cd "$(dirname "$0")/.."
V=raytracing-hw_amd
REPS=2 SHARD_STEPS=2 bash tools/r05_ab.sh r05p_ab.jsonl default $V/v_s5/librt_hw_amd.so $V/v_s5p/librt_hw_amd.so $V/v_p4/librt_hw_amd.so
