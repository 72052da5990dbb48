#!/bin/bash
# A/B of LLVM scheduler strategies (make variant VFLAGS='-mllvm -amdgpu-sched-strategy=S'):
# 1-GPU bench (frame digest must not change) and every shard of the 8-way split.  AB_LIBS="default var/x/librt_hw_amd.so ..."
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sched_ab.jsonl
for lib in ${AB_LIBS:-default}; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  b=$(timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fast-steps 0 --traffic-from none 2>>gpurun_out/sched_ab.err) || exit 1
  w=$(timeout -k 10 200 python -u tools/runahead_ab.py --off 0 --steps 1 --worlds 8 --full 0 2>>gpurun_out/sched_ab.err) || exit 1
  python3 -c "import json,sys; b=json.loads(sys.argv[2]); w=json.loads(sys.argv[3]); print(json.dumps({'lib': sys.argv[1], 'ms': b['ms_per_step'], 'sha': b['config']['frame_sha1'], 'shard8_max': w.get('shard8_max_ms_on'), 'shard8': w.get('shard8_ms_on')}))" "$lib" "$b" "$w" | tee -a gpurun_out/sched_ab.jsonl
done
