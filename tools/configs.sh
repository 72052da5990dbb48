#!/bin/bash
# Every BASELINE.json config with the current build, one MI355X (bash tools/configs.sh TAG):
#   C1 practice6_1 256x256x4, C2 cornell 512x512x64, C3 sponza 1024x1024x256: bench.py (1 GPU,
#     the reference's CPU loop beside it);
#   C4 sponza 1920x1080x1024 over 8 GPUs: the whole frame on one GPU and every shard of the
#     8-way split (the slowest shard is the 8-GPU frame time);
#   C5 dragon-100k + sponza 3840x2160x4096 over 8 GPUs: the 1-GPU rate at 16 spp (rays/s does
#     not depend on spp) and rank 0's shard of the 8-way split at the full 4096 spp.
set -o pipefail
tag=${1:-r03}
mkdir -p gpurun_out
out=gpurun_out/configs_$tag.jsonl; : > $out
for c in "practice6_1 256 256 4" "cornell 512 512 64" "sponza 1024 1024 256"; do
  set -- $c
  timeout -k 10 300 python bench.py --scene $1 --width $2 --height $3 --spp $4 --steps 3 --warmup 1 \
      --traffic-from none --cpu-rows $(( $3 < 135 ? $3 : 135 )) --cpu-spp $(( $4 < 16 ? $4 : 16 )) \
      --cpu-stride $(( $3 / 135 > 0 ? $3 / 135 : 1 )) >> $out 2>>gpurun_out/configs_$tag.err || exit 1
done
timeout -k 10 300 python tools/runahead_ab.py --spp 1024 --worlds 8 --off 0 --steps 1 >> $out 2>>gpurun_out/configs_$tag.err || exit 1
timeout -k 10 300 python bench.py --scene sponza_dragon --width 3840 --height 2160 --spp 16 --steps 2 --warmup 1 \
    --traffic-from none --no-cpu-baseline >> $out 2>>gpurun_out/configs_$tag.err || exit 1
timeout -k 10 300 python tools/runahead_ab.py --scene sponza_dragon --width 3840 --height 2160 --spp 4096 --worlds 8 \
    --max-ranks 1 --full 0 --off 0 --steps 1 >> $out 2>>gpurun_out/configs_$tag.err || exit 1
cat $out
