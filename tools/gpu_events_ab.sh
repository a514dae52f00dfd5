#!/bin/bash
# Cost of the per-frame timing events: bench with and without them, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ev
for r in 1 2; do
  for e in 0 1; do
    XRT_NO_EVENTS=$e timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/ev/e${e}_$r.json 2>/dev/null || exit 1
  done
done
for f in gpurun_out/ev/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step']*1000,1), round(d['roofline']['avg_kernel_ms']*1000,1))"; done
