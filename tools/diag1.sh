set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/shard_time.py --worlds 1,2,4,8,128 --steps 1 > gpurun_out/diag_worlds.txt 2>&1
RT_MEGA_TIMES=1 timeout -k 10 100 python tools/shard_time.py --worlds 8,128 --steps 1 > gpurun_out/diag_times.txt 2>&1
RT_LIB=$PWD/raytracing-hw_amd/prof/librt_hw_amd.so timeout -k 10 100 python tools/shard_time.py --worlds 1,8,128 --steps 1 > gpurun_out/diag_prof.txt 2>&1
