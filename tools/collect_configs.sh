#!/bin/bash
# Copies a tools/gpu_configs.sh run (gpurun_out/configs_TAG, scratch) into the
# tracked profiles/TAG: per config the rocprofv3 kernel-trace summary, the PMC
# summary (json + text) and the bench line; then profiles/traffic.json.
set -e
cd "$(dirname "$0")/.."
TAG=$1
SRC=gpurun_out/configs_$TAG
DST=profiles/$TAG
mkdir -p $DST
for d in $SRC/*_trace; do
  name=$(basename $d _trace)
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp $f $DST/kernel_stats_$name.csv
  [ -f $SRC/${name}_pmc/summary.json ] && cp $SRC/${name}_pmc/summary.json $DST/pmc_summary_$name.json
  [ -f $SRC/pmc_summary_$name.txt ] && cp $SRC/pmc_summary_$name.txt $DST/pmc_summary_$name.txt
  [ -f $SRC/bench_$name.json ] && cp $SRC/bench_$name.json $DST/bench_$name.json
done
cp $SRC/traffic.json profiles/traffic.json
ls $DST
