#!/bin/bash
# GPU parity tests, then an A/B of library variants (tools/ab_libs.sh) — one gpurun call.
#   bash tools/gpu_check.sh [libs...]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
if [ $# -gt 0 ]; then bash tools/ab_libs.sh "$@"; fi
