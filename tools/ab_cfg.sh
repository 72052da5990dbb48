#!/bin/bash
# A/B of library builds on one config through bench.py (1 GPU), one JSON line per library.
#   AB_CFG="--scene cornell --width 512 --height 512 --spp 64" bash tools/ab_cfg.sh TAG default raytracing-hw_amd/va/librt_hw_amd.so ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
out=gpurun_out/ab_$TAG.jsonl; : > $out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  b=$(timeout -k 10 200 python bench.py $AB_CFG --steps ${AB_STEPS:-5} --warmup 1 --no-cpu-baseline --fast-steps 0 \
      --natural-steps 0 --traffic-from none 2>>gpurun_out/ab_$TAG.err) || exit 1
  python3 -c "import json,sys; b=json.loads(sys.argv[2]); c=b['config']; print(json.dumps({'lib': sys.argv[1], 'cfg': sys.argv[3], 'ms': b['ms_per_step'], 'mrays': b['value'], 'sha1': c.get('frame_sha1')}))" \
      "$lib" "$b" "$AB_CFG" | tee -a $out
done
