#!/bin/bash
# BASELINE.json configs[3] (C4: sponza 1920x1080x1024spp over 8 GPUs) and configs[4] (C5:
# dragon-100k + sponza, 3840x2160x4096spp over 8 GPUs), measured on one MI355X: the 1-GPU
# rate at reduced spp (rays/s does not depend on spp) and rank 0's exact shard of the 8-way
# split (tools/shard_time.py), parity and fast mode.  bash tools/configs_c4_c5.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --scene sponza_dragon --width 3840 --height 2160 --spp 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5_bench.json || exit 1
echo "C5 1-GPU 16spp: $(python -c "import json; d=json.load(open('gpurun_out/c5_bench.json')); print(d['value'], d['ms_per_step'], 'fast', d['fast_mode']['value'])")"
timeout -k 10 300 python tools/shard_time.py --scene sponza_dragon --width 3840 --height 2160 --spp 64 --worlds 1,8 --steps 1 --chunks 0,2 > gpurun_out/c5_shard.jsonl || exit 1
cat gpurun_out/c5_shard.jsonl
timeout -k 10 300 python tools/shard_time.py --scene sponza --width 1920 --height 1080 --spp 1024 --worlds 8 --steps 1 --chunks 0,2 > gpurun_out/c4_shard.jsonl || exit 1
cat gpurun_out/c4_shard.jsonl
