#!/bin/bash
# Round-5 call: 1 / direction recomputed after each shading pass (RT_INV_RECOMPUTE: 42 instead
# of 48 spilled VGPRs in the plain kernel) against the default: the frame and all 8 shards, two
# runs each; then the WRITE pass of the frame for both.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
trap 'find gpurun_out -name "*.db" -delete' EXIT
REPS=2 bash tools/r05_ab.sh r05k_ab.jsonl default raytracing-hw_amd/v_inv/librt_hw_amd.so || exit 1
for lib in default raytracing-hw_amd/v_inv/librt_hw_amd.so; do
  if [ "$lib" = default ]; then unset RT_LIB; n=default; else export RT_LIB=$PWD/$lib; n=inv; fi
  PASS_TIMEOUT=120 PASSES="write sq2" bash tools/profile.sh r05k_$n --steps 1 --warmup 1 --no-cpu-baseline --fast-steps 0 --natural-steps 0 || exit 1
done
