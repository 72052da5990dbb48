#!/bin/bash
# Rank-0 shard times (tools/shard_time.py) for each library given ("default" = in-tree build).
#   bash tools/ab_shards.sh WORLDS lib...
set -o pipefail
mkdir -p gpurun_out
W=$1; shift
for lib in "$@"; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  out=$(timeout -k 10 200 python tools/shard_time.py --worlds $W --steps 1 2>>gpurun_out/ab_shards.err) || exit 1
  echo "[$lib] $(echo "$out" | python3 -c "import sys,json; print(' '.join(f\"w{d['world']}:{d['rank0_ms']}\" for d in map(json.loads, sys.stdin)))")"
done
