#!/bin/bash
# round-4 batch: park A/B (1 GPU), runahead tail-window variants (8-way shards), PMC passes, GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pool_ab.py --steps 3 --worlds 1 --modes lane --libs raytracing-hw_amd/librt_hw_amd.so,raytracing-hw_amd/v_park_off/librt_hw_amd.so,raytracing-hw_amd/v_sqrt_off/librt_hw_amd.so,raytracing-hw_amd/v_base3/librt_hw_amd.so > gpurun_out/r04f_park_ab.jsonl 2>&1 || { tail -5 gpurun_out/r04f_park_ab.jsonl; exit 1; }
cat gpurun_out/r04f_park_ab.jsonl | grep '^{'
WORLDS=8 timeout -k 10 400 bash tools/runahead_variants.sh default raytracing-hw_amd/v_t8w6/librt_hw_amd.so raytracing-hw_amd/v_t4w8/librt_hw_amd.so raytracing-hw_amd/v_t16w5/librt_hw_amd.so raytracing-hw_amd/v_t2w10/librt_hw_amd.so || exit 1
cp gpurun_out/runahead_variants.jsonl gpurun_out/r04f_tail_ab.jsonl
python3 -c "
import json
for l in open('gpurun_out/r04f_tail_ab.jsonl'):
    d=json.loads(l); print(d['lib'][-30:], d['shard8_max_ms_on'], d['shard8_ms_on'])"
bash tools/pmc_cmd.sh r04f_park "tools/pool_ab.py --steps 1 --worlds 1 --modes lane" write sq2 || exit 1
RT_LIB=$PWD/raytracing-hw_amd/v_park_off/librt_hw_amd.so bash tools/pmc_cmd.sh r04f_parkoff "tools/pool_ab.py --steps 1 --worlds 1 --modes lane" write sq2 || exit 1
bash tools/round_check.sh r04f tests || exit 1
echo "[r04f] done"
