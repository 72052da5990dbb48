#!/bin/bash
# A/B of compile-time variants: bench (1 GPU, default workload) + rank-0 shard of an 8-way
# split, for each library given (paths relative to the repo; "default" = the in-tree build).
#   bash tools/ab_libs.sh default raytracing-hw_amd/v1/librt_hw_amd.so ...
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_libs.jsonl; : > $out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  b=$(timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fast-steps 0 --traffic-from none 2>>gpurun_out/ab_libs.err) || exit 1
  w=$(timeout -k 10 120 python tools/shard_time.py --worlds ${AB_WORLDS:-8} --steps 2 2>>gpurun_out/ab_libs.err) || exit 1
  python3 -c "import json,sys; b=json.loads(sys.argv[2]); print(json.dumps({'lib': sys.argv[1], 'mrays': b['value'], 'ms': b['ms_per_step'], 'match': b['config'].get('frame_matches_reference'), 'shard': sys.argv[3]}))" "$lib" "$b" "$w" | tee -a $out
done
