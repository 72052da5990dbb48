#!/bin/bash
# Round-5 call: the GPU suite and smoke() on the exact final tree (after the last rebuild).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r05r_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r05r_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r05r_gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05r_smoke.txt 2>&1 || { tail -10 gpurun_out/r05r_smoke.txt; exit 1; }
cat gpurun_out/r05r_smoke.txt
