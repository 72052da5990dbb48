#!/bin/bash
# Round-5 call: shading-pass register cuts against the default, the frame and all 8 shards,
# two runs each, then the WRITE and SQ2 passes of the frame for each build:
#   v_inv    RT_INV_RECOMPUTE  1 / direction recomputed after a shading pass
#   v_uv     RT_UV_RECOMPUTE   (u, v) of the closest hit recomputed at shading, not carried
#   v_uvinv  both
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
trap 'find gpurun_out -name "*.db" -delete' EXIT
V=raytracing-hw_amd
REPS=2 bash tools/r05_ab.sh r05k_ab.jsonl default $V/v_inv/librt_hw_amd.so $V/v_uv/librt_hw_amd.so $V/v_uvinv/librt_hw_amd.so || exit 1
for n in default v_inv v_uv v_uvinv; do
  if [ "$n" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$V/$n/librt_hw_amd.so; fi
  PASS_TIMEOUT=120 PASSES="write sq2" bash tools/profile.sh r05k_$n --steps 1 --warmup 1 --no-cpu-baseline --fast-steps 0 --natural-steps 0 || exit 1
done
