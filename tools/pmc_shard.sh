#!/bin/bash
# SQ counter passes over one rank's shard (tools/shard_time.py) per world size, to compare
# where wave time goes at full and at low occupancy.  One rocprofv3 --pmc pass per run.
#   bash tools/pmc_shard.sh TAG "8 128" [pass ...]        (passes: sq1 sq2 sq3 mem fetch write tcc; default sq1 sq2)
# gpurun_out/pmc_TAG/<pass>_w<N>.csv; committed as profiles/<TAG>_shard_<pass>_w<N>.csv (bench.py
# reads those for an --gpus N line).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; WORLDS=$2; shift 2
PASSES=${*:-sq1 sq2}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in $WORLDS; do
  for p in $PASSES; do
    case $p in
      sq1) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" ;;
      fetch) C="FETCH_SIZE" ;;
      write) C="WRITE_SIZE" ;;
      tcc) C="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" ;;
      sq2) C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_INSTS_LDS" ;;
      mem) C="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" ;;
      sq3) C="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_EXP SQ_LDS_BANK_CONFLICT" ;;
    esac
    timeout -s KILL 150 rocprofv3 --pmc $C -d "$OUT/${p}_w$w" -o run -- python3 tools/shard_time.py --worlds $w --steps 1 \
        > "$OUT/${p}_w$w.log" 2>&1 || { echo "pass $p w$w failed"; exit 1; }
    python3 tools/rocpd_summary.py pmc "$OUT/${p}_w$w/run_results.db" "$OUT/${p}_w$w.csv" || exit 1
    echo "[pmc] $p w$w done"
  done
done
