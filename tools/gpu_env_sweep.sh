#!/bin/bash
# Bench kernel times under one environment variable's values:
#   tools/gpu_env_sweep.sh VAR "v1 v2 ..." ["2048 1024 4096"]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=$1; VALS=$2; SIZES=${3:-"2048 1024 4096"}
for s in $SIZES; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --size $s $s > gpurun_out/sweep.json 2> gpurun_out/sweep.err || { tail -5 gpurun_out/sweep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/sweep.json')); print('size $s $VAR=$v', 'ms/step %.4f'%d['ms_per_step'], 'kernel %.4f'%d['roofline']['avg_kernel_ms'], 'Mrays/s %.0f'%d['value'])"
  done
done
