set -o pipefail
out=gpurun_out/lockstep.jsonl; : > $out
for lib in default raytracing-hw_amd/vk4/librt_hw_amd.so raytracing-hw_amd/vk16/librt_hw_amd.so raytracing-hw_amd/vk64/librt_hw_amd.so; do
  if [ "$lib" = default ]; then unset RT_LIB; else export RT_LIB=$PWD/$lib; fi
  timeout -k 10 200 python tools/runahead_ab.py --worlds 1080 --row-block 1 --rank-stride 8 --full 0 --off 1 --steps 1 >> $out 2>>gpurun_out/lockstep.err || exit 1
done
