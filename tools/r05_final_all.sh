#!/bin/bash
# Round-5 final-build evidence in one gpurun call: bench line, kernel trace + PMC passes of the
# bench command (tools/profile.sh), kernel trace of all 8 shards of the 8-way split, PMC passes of
# rank 0's shard, the N = 8 rehearsal of bench.py on one GPU (RT_BENCH_SHARE_GPU=1), and the
# diagnostics build's event counts of the 8-way shard.
#   bash tools/r05_final_all.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r05}
mkdir -p gpurun_out
# the rocprofv3 databases are hundreds of MB: keep the CSV summaries only (gpurun merges at most
# 64 MiB of gpurun_out/ back)
trap 'find gpurun_out -name "*.db" -delete; find gpurun_out -name "*_results*" -size +1M -delete' EXIT
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 300 gpurun_out/${TAG}_bench.json
PASS_TIMEOUT=120 PASSES="kt fetch write sq1 sq2" bash tools/profile.sh $TAG --steps 2 --warmup 1 --no-cpu-baseline --fast-steps 0 --natural-steps 0 || exit 1
bash tools/kt_shards.sh $TAG 8 || exit 1
bash tools/pmc_shard.sh $TAG 8 sq1 sq2 fetch write || exit 1
RT_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 8 --steps 1 --warmup 1 --no-cpu-baseline --fast-steps 0 --natural-steps 0 \
    > gpurun_out/${TAG}_rehearsal_w8.json 2> gpurun_out/${TAG}_rehearsal_w8.err || { tail -5 gpurun_out/${TAG}_rehearsal_w8.err; exit 1; }
tail -c 300 gpurun_out/${TAG}_rehearsal_w8.json
RT_LIB=$PWD/raytracing-hw_amd/prof/librt_hw_amd.so timeout -k 10 150 python3 tools/shard_time.py --worlds 8 --steps 1 \
    > gpurun_out/${TAG}_megaprof_w8.txt 2>&1 || exit 1
echo done
