#!/bin/bash
# FETCH_SIZE calibration for the render kernel's load shapes (tools/fetch_calib.hip): the
# program's own JSON (bytes asked for, 128-B lines touched, time per shape), then one
# rocprofv3 pass for FETCH_SIZE and one for the TCC request counters, summarised into
# gpurun_out/TAG/fetch_calib.csv (tools/fetch_calib_summary.py).
#   bash tools/fetch_calib.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
EXE=tools/bin/fetch_calib
[ -x $EXE ] && [ $EXE -nt tools/fetch_calib.hip ] || /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o $EXE || exit 1
timeout -k 10 120 $EXE > "$OUT/fetch_calib_run.json" || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/calib_fetch" -o run -- $EXE > "$OUT/calib_fetch.log" 2>&1 || exit 1
python3 tools/rocpd_summary.py pmc "$OUT/calib_fetch/run_results.db" "$OUT/calib_fetch.csv" || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum -d "$OUT/calib_tcc" \
    -o run -- $EXE > "$OUT/calib_tcc.log" 2>&1 || exit 1
python3 tools/rocpd_summary.py pmc "$OUT/calib_tcc/run_results.db" "$OUT/calib_tcc.csv" || exit 1
python3 tools/fetch_calib_summary.py "$OUT/fetch_calib_run.json" "$OUT/calib_fetch.csv" "$OUT/calib_tcc.csv" \
    "$OUT/fetch_calib.csv" || exit 1
cat "$OUT/fetch_calib.csv" "$OUT/fetch_calib_gather.csv"
