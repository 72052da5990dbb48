#!/bin/bash
# Kernel trace of every shard of an N-way split (tools/runahead_ab.py): per-dispatch durations
# of the render kernels, to check the slowest-shard time against the profiler.
#   bash tools/kt_shards.sh TAG [N]
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; W=${2:-8}
OUT=gpurun_out/kt_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt -- python3 tools/runahead_ab.py --off 0 --steps 1 --worlds $W --full 0 \
    > "$OUT/kt.log" 2>&1 || { tail -20 "$OUT/kt.log"; exit 1; }
python3 tools/rocpd_summary.py stats "$OUT/kt/kt_results.db" "$OUT/kt_stats.csv" || exit 1
python3 - "$OUT/kt/kt_results.db" "$OUT/kt_dispatches.csv" <<'PY'
import csv, sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, duration from kernels where name like '%rt_mega_kernel%' order by start").fetchall()
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Kernel", "StartNs", "DurationNs"])
    for r in rows:
        w.writerow(r)
for n, s, d in rows:
    print(n[:60], round(d / 1e6, 2), "ms")
PY
