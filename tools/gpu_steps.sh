#!/bin/bash
# One gpurun call as a list of steps.  Every GPU step runs under its own time limit and the
# first failure ends the call (nothing more touches the GPU after it).  Outputs go to
# gpurun_out/TAG/; tools/collect.sh copies the ones to keep into profiles/ as TAG_*.
#
#   bash tools/gpu_steps.sh TAG STEP [STEP ...]
#
# LIB below is a library path relative to the repo (raytracing-hw_amd/vX/librt_hw_amd.so), or
# "default" (raytracing-hw_amd/librt_hw_amd.so); build variants with
#   make -C raytracing-hw_amd variant VDIR=vX VFLAGS=-DRT_...
# Steps:
#   tests[=K]            pytest -m gpu (-k K when given)                    gpu_tests.txt
#   debugtests           the same on the index-checked build (make debug)   debug_gpu_tests.txt
#   smoke                __graft_entry__.smoke()                            smoke.txt
#   bench[=ARGS]         bench.py --steps 3 --warmup 1 (or ARGS, comma-separated)   bench.json
#   ab=N,REPS,LIB+LIB    per library: the 1-GPU frame + every shard of the N-way split, with
#                        the sha1 of both (tools/order_ab.py), REPS rounds   ab.jsonl
#   splits=N[,LIB]       every shard of the N-way split only                splits.jsonl
#   megaprof=W+W[,LIB]   diagnostics build (make prof): main-loop split and 5-ms buckets of
#                        rank 0's shard of each W-way split                 megaprof.txt
#   pmc=W,PASS+PASS      PMC passes over rank 0's shard (tools/pmc_shard.sh) pmc_<pass>_w<W>.csv
#   profile=PASS+PASS    kernel trace / PMC passes of the bench command (tools/profile.sh)
#   kt=N                 kernel trace of all N shards (tools/kt_shards.sh)  kt_shards_*.csv
#   rehearsal=N          bench.py --gpus N as N ranks sharing one GPU       rehearsal_wN.json
#   calib                FETCH_SIZE calibration of the kernel's load widths (tools/fetch_calib)
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$PWD
# the rocprofv3 databases are hundreds of MB: keep the CSV summaries only (gpurun merges at most
# 64 MiB of gpurun_out/ back)
trap 'find gpurun_out -name "*.db" -delete 2>/dev/null; find gpurun_out -name "*_results*" -size +1M -delete 2>/dev/null' EXIT

lib_env() {   # LIB -> RT_LIB for the next command
  if [ -z "$1" ] || [ "$1" = default ]; then unset RT_LIB; else export RT_LIB=$ROOT/$1; fi
}
fail() { echo "[steps] $TAG: $1 failed"; [ -n "$2" ] && tail -30 "$2"; exit 1; }

for step in "$@"; do
  name=${step%%=*}; arg=; [ "$name" != "$step" ] && arg=${step#*=}
  echo "[steps] $TAG: $step"
  case $name in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" \
        > "$OUT/gpu_tests.txt" 2>&1 || fail tests "$OUT/gpu_tests.txt"
      tail -2 "$OUT/gpu_tests.txt" ;;
    debugtests)
      RT_LIB=$ROOT/raytracing-hw_amd/debug/librt_hw_amd.so timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v \
        --timeout 240 --timeout-method thread > "$OUT/debug_gpu_tests.txt" 2>&1 || fail debugtests "$OUT/debug_gpu_tests.txt"
      tail -2 "$OUT/debug_gpu_tests.txt" ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 \
        || fail smoke "$OUT/smoke.txt"
      cat "$OUT/smoke.txt" ;;
    bench)
      A=(--steps 3 --warmup 1); [ -n "$arg" ] && IFS=, read -r -a A <<< "$arg"
      timeout -k 10 400 python -u bench.py "${A[@]}" >> "$OUT/bench.json" 2>> "$OUT/bench.err" || fail bench "$OUT/bench.err"
      tail -c 600 "$OUT/bench.json" ;;
    ab)
      IFS=, read -r N REPS LIBS <<< "$arg"
      for rep in $(seq "${REPS:-1}"); do
        for lib in ${LIBS//+/ }; do
          lib_env "$lib"
          timeout -k 10 300 python3 tools/order_ab.py --natural 0 --steps 2 --shard-steps 1 --world "${N:-8}" \
            >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || fail "ab $lib" "$OUT/ab.err"
          tail -1 "$OUT/ab.jsonl"
        done
      done
      unset RT_LIB ;;
    splits)
      IFS=, read -r N LIB <<< "$arg"
      lib_env "$LIB"
      timeout -k 10 300 python3 tools/order_ab.py --natural 0 --full 0 --shard-steps 1 --world "$N" \
        >> "$OUT/splits.jsonl" 2>> "$OUT/splits.err" || fail "splits $N" "$OUT/splits.err"
      tail -1 "$OUT/splits.jsonl"
      unset RT_LIB ;;
    megaprof)
      IFS=, read -r WS LIB <<< "$arg"
      lib_env "${LIB:-raytracing-hw_amd/prof/librt_hw_amd.so}"
      timeout -k 10 400 python3 tools/shard_time.py --worlds "${WS//+/,}" --steps 1 >> "$OUT/megaprof.txt" 2>&1 \
        || fail megaprof "$OUT/megaprof.txt"
      grep -h "wave end" "$OUT/megaprof.txt" | tail -4
      unset RT_LIB ;;
    pmc)
      IFS=, read -r W PASSES <<< "$arg"
      timeout -k 10 900 bash tools/pmc_shard.sh "$TAG" "${W//+/ }" ${PASSES//+/ } > "$OUT/pmc.log" 2>&1 || fail pmc "$OUT/pmc.log"
      cp gpurun_out/pmc_$TAG/*.csv "$OUT/" 2>/dev/null
      tail -3 "$OUT/pmc.log" ;;
    profile)
      PASS_TIMEOUT=150 PASSES="${arg//+/ }" timeout -k 10 1000 bash tools/profile.sh "$TAG" --steps 2 --warmup 1 \
        --no-cpu-baseline --fast-steps 0 --natural-steps 0 > "$OUT/profile.log" 2>&1 || fail profile "$OUT/profile.log"
      cp gpurun_out/prof_$TAG/*.csv "$OUT/" 2>/dev/null
      tail -3 "$OUT/profile.log" ;;
    kt)
      timeout -k 10 300 bash tools/kt_shards.sh "$TAG" "${arg:-8}" > "$OUT/kt_shards.txt" 2>&1 || fail kt "$OUT/kt_shards.txt"
      cp gpurun_out/kt_$TAG/kt_stats.csv "$OUT/kt_shards_w${arg:-8}_stats.csv" 2>/dev/null
      cp gpurun_out/kt_$TAG/kt_dispatches.csv "$OUT/kt_shards_w${arg:-8}_dispatches.csv" 2>/dev/null
      tail -"${arg:-8}" "$OUT/kt_shards.txt" ;;
    rehearsal)
      N=${arg:-8}
      RT_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
        --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus "$N" --steps 1 --warmup 1 --no-cpu-baseline \
        --fast-steps 0 --natural-steps 0 > "$OUT/rehearsal_w$N.json" 2> "$OUT/rehearsal_w$N.err" \
        || fail "rehearsal $N" "$OUT/rehearsal_w$N.err"
      tail -c 600 "$OUT/rehearsal_w$N.json" ;;
    calib)
      timeout -k 10 300 bash tools/fetch_calib.sh "$TAG" > "$OUT/calib.log" 2>&1 || fail calib "$OUT/calib.log"
      tail -12 "$OUT/calib.log" ;;
    *) echo "[steps] unknown step $step"; exit 2 ;;
  esac
done
echo "[steps] $TAG done"
