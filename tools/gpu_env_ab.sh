#!/bin/bash
# Whole-step A/B of an environment switch: tools/gpu_env_ab.sh VAR "v1 v2 ..." [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/envab
VAR=$1; VALS=$2; shift 2
for r in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/envab/${v}_$r.json 2>/dev/null || exit 1
  done
done
for v in $VALS; do for r in 1 2; do python3 -c "
import json; d=json.loads(open('gpurun_out/envab/${v}_$r.json').read().strip().splitlines()[-1]); print('$VAR=$v', d['config']['workload'], round(d['ms_per_step']*1000,1), round(d['roofline']['avg_kernel_ms']*1000,1))"; done; done
