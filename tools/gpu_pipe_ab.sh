#!/bin/bash
# Pipelined vs serial preparation, with and without timing events, + traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pipe
for r in 1 2; do
  for pl in 0 1; do
    for e in 0 1; do
      XRT_PIPELINE=$pl XRT_NO_EVENTS=$e timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/pipe/p${pl}e${e}_$r.json 2>/dev/null || exit 1
    done
  done
done
for pl in 0 1; do
  XRT_PIPELINE=$pl XRT_NO_EVENTS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pipe/prof$pl -o run -- python3 bench.py --no-cpu-baseline --steps 10 "$@" > /dev/null 2>&1 || exit 1
done
for f in gpurun_out/pipe/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step']*1000,1), round(d['roofline']['avg_kernel_ms']*1000,1))"; done
