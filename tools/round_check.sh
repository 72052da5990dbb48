#!/bin/bash
# One gpurun call: the GPU suite, smoke, the default bench line, then (optional) the kernel
# trace of every 8-way shard and rank 0's shard PMC passes.
#   bash tools/round_check.sh TAG [tests|bench|shards|shardpmc ...]   (default: tests bench)
# Logs under gpurun_out/check_TAG/.  Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; shift
STEPS=${*:-tests bench}
OUT=gpurun_out/check_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 \
        || { tail -40 "$OUT/gpu_tests.txt"; exit 1; }
      tail -2 "$OUT/gpu_tests.txt"
      timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { cat "$OUT/smoke.txt"; exit 1; }
      cat "$OUT/smoke.txt" ;;
    bench)
      timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    shards)
      timeout -k 10 240 bash tools/kt_shards.sh "$TAG" 8 > "$OUT/kt_shards.txt" 2>&1 || { tail -20 "$OUT/kt_shards.txt"; exit 1; }
      tail -10 "$OUT/kt_shards.txt" ;;
    shardpmc)
      timeout -k 10 600 bash tools/pmc_shard.sh "$TAG" 8 fetch write sq1 sq2 > "$OUT/pmc_shard.txt" 2>&1 || { tail -20 "$OUT/pmc_shard.txt"; exit 1; }
      tail -4 "$OUT/pmc_shard.txt" ;;
  esac
done
echo "[check] $TAG done"
