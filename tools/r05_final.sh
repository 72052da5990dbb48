#!/bin/bash
# Round-5 final-build evidence, part 1 (one gpurun call): GPU suite, bench line, kernel trace
# and PMC passes of the bench command (tools/profile.sh), all on the same build.
#   bash tools/r05_final.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 520 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 \
    || { tail -30 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 600 gpurun_out/${TAG}_bench.json
PASS_TIMEOUT=150 PASSES="kt fetch write sq1 sq2 tcc" bash tools/profile.sh $TAG --steps 2 --warmup 1 --no-cpu-baseline --fast-steps 0 --natural-steps 0 || exit 1
