#!/usr/bin/env bash
# Profile the bench workload on the GPU box: kernel trace + separate PMC passes
# (MI355X_MICROARCH.md: counters in their own runs, no trace domains with --pmc).
#   bash tools/profile.sh TAG [bench args...]
# Writes gpurun_out/prof_TAG/{kt,fetch,write,tcc,sq1,sq2}/ and CSV summaries next to them.
set -euo pipefail
TAG=$1; shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--spp 8 --steps 1 --warmup 1 --no-cpu-baseline)
cd "$(dirname "$0")/.."
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, rocprofv3 options...
    local name=$1; shift
    timeout -k 10 ${PASS_TIMEOUT:-200} rocprofv3 "$@" -d "$OUT/$name" -o "$name" -- python3 bench.py "${ARGS[@]}" > "$OUT/$name.log" 2>&1
    python3 tools/rocpd_summary.py "$( [ "$name" = kt ] && echo stats || echo pmc )" "$OUT/$name/$name"_results.db "$OUT/$name.csv"
    echo "[profile] $name done"
}
PASSES=${PASSES:-kt fetch write tcc sq1 sq2 ta}
for p in $PASSES; do
    case $p in
        kt) run kt --kernel-trace --stats ;;
        fetch) run fetch --pmc FETCH_SIZE ;;
        write) run write --pmc WRITE_SIZE ;;
        tcc) run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum ;;
        sq1) run sq1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE ;;
        sq2) run sq2 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_INSTS_LDS ;;
        mem) run mem --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE ;;
        ta) run ta --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE ;;
        ta2) run ta2 --pmc TA_ADDR_STALLED_BY_TC_CYCLES_sum ;;
        tcp) run tcp --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum ;;
        td) run td --pmc TD_TD_BUSY_sum ;;
    esac
done
grep -h '^{' "$OUT/kt.log" > "$OUT/bench_line.json" || true
echo "[profile] all passes done"
