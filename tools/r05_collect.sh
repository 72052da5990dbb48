#!/bin/bash
# Copy the round-5 final-build evidence from gpurun_out/ into profiles/ under the names bench.py
# reads (PROFILE_PREFIX / SHARD_PROFILE_PREFIX = r05).
set -e
cd "$(dirname "$0")/.."
T=${1:-r05}
P=gpurun_out/prof_$T
for p in kt fetch write sq1 sq2 tcc; do
  [ -f $P/$p.csv ] && cp $P/$p.csv profiles/${T}_${p}_1080p256.csv
done
grep -h '^{' $P/kt.log > profiles/${T}_bench_under_rocprof.json || true
grep -h '^{' gpurun_out/${T}_bench.json | tail -1 > profiles/${T}_bench_1080p256.json
cp gpurun_out/kt_$T/kt_stats.csv profiles/${T}_kt_shards_w8_stats.csv
cp gpurun_out/kt_$T/kt_dispatches.csv profiles/${T}_kt_shards_w8_dispatches.csv
for p in sq1 sq2 fetch write; do cp gpurun_out/pmc_$T/${p}_w8.csv profiles/${T}_shard_${p}_w8.csv; done
grep -h '^{' gpurun_out/${T}_rehearsal_w8.json | tail -1 > profiles/${T}_rehearsal_w8.json
grep -h "mega prof\|mega tb" gpurun_out/${T}_megaprof_w8.txt > profiles/${T}_megaprof_w8.txt
ls -la profiles/${T}_*
