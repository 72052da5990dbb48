#!/bin/bash
# Round-5 call: loop invariants out of the plain kernel's VGPRs.  v_old = the r05k build; default = pixel divisions as
# multiply-and-shift with host constants, camera divisors as kernel arguments, claim prefix by
# mbcnt (33 spilled VGPRs); v_pk2 + RT_PACK_TRAV (20); v_tid + RT_TID_REMAT; v_pt both (16).
# Frame and shards, two runs each; then the GPU suite and the WRITE / SQ2 passes of the best
# candidate (v_pt).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
trap 'find gpurun_out -name "*.db" -delete' EXIT
V=raytracing-hw_amd
REPS=2 SHARD_STEPS=1 bash tools/r05_ab.sh r05n_ab.jsonl $V/v_old/librt_hw_amd.so default $V/v_pk2/librt_hw_amd.so $V/v_tid/librt_hw_amd.so $V/v_pt/librt_hw_amd.so || exit 1
for n in default v_pt; do
  if [ "$n" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$V/$n/librt_hw_amd.so; fi
  PASS_TIMEOUT=120 PASSES="write sq2" bash tools/profile.sh r05n_$n --steps 1 --warmup 1 --no-cpu-baseline --fast-steps 0 --natural-steps 0 || exit 1
done
export RT_LIB=$PWD/$V/v_pt/librt_hw_amd.so
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05n_gpu_tests.txt 2>&1 || { tail -20 gpurun_out/r05n_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r05n_gpu_tests.txt
