#!/usr/bin/env bash
# Parameter sweep of the wavefront tuning knobs on the GPU box (stops at the first failure).
#   bash tools/sweep.sh "VAR=a VAR2=b" "VAR=c" ... -- bench args
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
CONFIGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do CONFIGS+=("$1"); shift; done
[ $# -gt 0 ] && shift
for c in "${CONFIGS[@]}"; do
    line=$(env $c timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline 2>/dev/null | grep '^{')
    echo "$c $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_ms"], r["frac"])')"
done
