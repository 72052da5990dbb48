#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each) and a kernel trace over an arbitrary python script.
#   bash tools/pmc_cmd.sh TAG "script.py args" [pass ...]   (passes: kt sq1 sq2 sq3 fetch write tcc; default kt sq1 sq2)
# gpurun_out/pmccmd_TAG/<pass>.csv (tools/rocpd_summary.py summaries).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; CMD=$2; shift 2
PASSES=${*:-kt sq1 sq2}
OUT=gpurun_out/pmccmd_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for p in $PASSES; do
  case $p in
    kt) OPT="--kernel-trace --stats" ;;
    sq1) OPT="--pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" ;;
    sq2) OPT="--pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_INSTS_LDS" ;;
    sq3) OPT="--pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_EXP SQ_LDS_BANK_CONFLICT" ;;
    fetch) OPT="--pmc FETCH_SIZE" ;;
    write) OPT="--pmc WRITE_SIZE" ;;
    tcc) OPT="--pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" ;;
  esac
  timeout -s KILL 200 rocprofv3 $OPT -d "$OUT/$p" -o run -- python3 $CMD > "$OUT/$p.log" 2>&1 || { echo "pass $p failed"; tail -5 "$OUT/$p.log"; exit 1; }
  python3 tools/rocpd_summary.py "$( [ "$p" = kt ] && echo stats || echo pmc )" "$OUT/$p/run_results.db" "$OUT/$p.csv" || exit 1
  echo "[pmc] $p done"
done
