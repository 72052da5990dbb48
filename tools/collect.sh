#!/bin/bash
# Copy a gpu_steps.sh call's outputs that are worth keeping into profiles/ as TAG_<file>
# (gpurun_out/ is scratch; profiles/ is tracked).
#   bash tools/collect.sh TAG [file ...]     (default: every .csv, .txt, .json, .jsonl)
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; shift
SRC=gpurun_out/$TAG
[ -d "$SRC" ] || { echo "no $SRC"; exit 1; }
FILES=("$@")
[ ${#FILES[@]} -eq 0 ] && FILES=($(cd "$SRC" && ls *.csv *.txt *.json *.jsonl 2>/dev/null))
for f in "${FILES[@]}"; do
  cp "$SRC/$f" "profiles/${TAG}_$f" && echo "profiles/${TAG}_$f"
done
