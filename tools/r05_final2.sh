#!/bin/bash
# Round-5 final-build evidence, part 2 (one gpurun call): kernel trace of all 8 shards of the
# 8-way split, PMC passes of rank 0's shard, the N = 8 rehearsal of bench.py on one GPU
# (RT_BENCH_SHARE_GPU=1: 8 ranks, gloo; the frame digest must be the reference's), and the
# diagnostics build's event counts of the 8-way shard (default and block-shared runahead).
#   bash tools/r05_final2.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r05}
mkdir -p gpurun_out
bash tools/kt_shards.sh $TAG 8 || exit 1
bash tools/pmc_shard.sh $TAG 8 sq1 sq2 fetch write || exit 1
RT_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 8 --steps 1 --warmup 1 --no-cpu-baseline --fast-steps 0 --natural-steps 0 \
    > gpurun_out/${TAG}_rehearsal_w8.json 2> gpurun_out/${TAG}_rehearsal_w8.err || { tail -5 gpurun_out/${TAG}_rehearsal_w8.err; exit 1; }
tail -c 400 gpurun_out/${TAG}_rehearsal_w8.json
for lib in prof prof_share; do
  RT_LIB=$PWD/raytracing-hw_amd/$lib/librt_hw_amd.so timeout -k 10 200 python3 tools/shard_time.py --worlds 8 --steps 1 \
      > gpurun_out/${TAG}_megaprof_w8_$lib.txt 2>&1 || exit 1
done
echo done
