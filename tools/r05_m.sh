#!/bin/bash
# Round-5 call: RT_PACK_TRAV (a non-shading lane's phase, stack depth and state packed in one
# register through the shading pass: plain kernel 39 -> 28 spilled VGPRs) against the default,
# two runs; then the GPU suite on the packed build (counting kernel included) and its WRITE pass.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
trap 'find gpurun_out -name "*.db" -delete' EXIT
V=raytracing-hw_amd
REPS=2 SHARD_STEPS=1 bash tools/r05_ab.sh r05m_ab.jsonl default $V/v_pack/librt_hw_amd.so || exit 1
export RT_LIB=$PWD/$V/v_pack/librt_hw_amd.so
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05m_gpu_tests.txt 2>&1 || { tail -20 gpurun_out/r05m_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r05m_gpu_tests.txt
PASS_TIMEOUT=120 PASSES="write sq2" bash tools/profile.sh r05m_pack --steps 1 --warmup 1 --no-cpu-baseline --fast-steps 0 --natural-steps 0 || exit 1
