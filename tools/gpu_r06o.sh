#!/bin/bash
# Box tile masks as a runtime policy (XRT_BOX_MASKS, default 1): the whole GPU
# suite, then the bench with masks off (0) and on (1) alternating, per config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CONFIGS=("2048|--size 2048 2048|--steps 200 --warmup 20"
         "1024|--size 1024 1024|--steps 200 --warmup 20"
         "4096|--size 4096 4096|--steps 60 --warmup 10"
         "8192|--size 8192 8192|--steps 20 --warmup 5")
for rep in 1 2; do
  for c in "${CONFIGS[@]}"; do
    IFS='|' read -r name cfg steps <<< "$c"
    for m in 0 1; do
      d=$OUT/${name}_m${m}_$rep
      XRT_BOX_MASKS=$m timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-latency --no-timing-check --orbit-legs --no-tile-plan-leg $cfg $steps > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
      python3 -c "import json,sys; b=json.load(open(sys.argv[1])); lo=b.get('at_loaded_clocks') or {}; print(sys.argv[2], 'value', round(b['value']), 'step', round(b['ms_per_step']*1e3,2), 'loaded', round(lo.get('ms_per_step',0)*1e3,2))" $d.json "$name masks=$m rep $rep"
    done
  done
done
