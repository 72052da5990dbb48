#!/bin/bash
# WRITE_SIZE / FETCH_SIZE passes (one counter set per rocprofv3 run) of a short bench
# (1080p x 32 spp) for each library given ("default" = the in-tree build).
#   bash tools/pmc_write_exp.sh default raytracing-hw_amd/var/prev/librt_hw_amd.so
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcexp
for lib in "$@"; do
  if [ "$lib" = default ]; then unset RT_LIB; tag=default; else export RT_LIB=$PWD/$lib; tag=$(basename $(dirname $lib)); fi
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmcexp/${c}_$tag -o p -- python3 bench.py --spp 32 --steps 1 --warmup 1 --no-cpu-baseline --fast-steps 0 --natural-steps 0 --traffic-from none > gpurun_out/pmcexp/${c}_$tag.log 2>&1 || exit 1
    python3 tools/rocpd_summary.py pmc gpurun_out/pmcexp/${c}_$tag/p_results.db gpurun_out/pmcexp/${c}_$tag.csv || exit 1
  done
done
