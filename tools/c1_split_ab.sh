#!/bin/bash
# Light-split kernel A/B on the many-light scene (practice6_1 proxy, 1,152 emissive
# triangles): RT_LIGHT_SPLIT_MIN=1 (split) against 0 (light pdf walked inline in shading),
# at C1's size and at larger frames.  One GPU call: bash tools/c1_split_ab.sh
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/c1_split_ab.jsonl
for wh in "256 256 4" "1024 1024 4" "1920 1080 16"; do
  set -- $wh
  for m in 1 0; do
    RT_LIGHT_SPLIT_MIN=$m timeout -k 10 120 python bench.py --scene practice6_1 --width $1 --height $2 --spp $3 --steps 10 --warmup 2 --no-cpu-baseline --fast-steps 3 --fast-chunk 1 > gpurun_out/c1.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/c1.json')); print(json.dumps({'size': '$1x$2x$3', 'split_min': $m, 'mrays': d['value'], 'ms': d['ms_per_step'], 'fast_c1_mrays': d['fast_mode']['value'], 'fast_ms': d['fast_mode']['ms_per_step']}))" | tee -a gpurun_out/c1_split_ab.jsonl
  done
done
