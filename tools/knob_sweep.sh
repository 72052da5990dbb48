#!/bin/bash
# Rank-0 shard time of an N-way split (tools/shard_time.py) under environment knob settings.
#   bash tools/knob_sweep.sh WORLDS "ENV1=a ENV2=b" "ENV1=c" ...     ("" = defaults)
set -o pipefail
mkdir -p gpurun_out
W=$1; shift
for kv in "$@"; do
  out=$(env $kv timeout -k 10 150 python tools/shard_time.py --worlds $W --steps 2 2>>gpurun_out/knob_sweep.err) || exit 1
  echo "[$kv] $out" | tr '\n' ' '; echo
done
