#!/bin/bash
# A/B of one environment knob of the production library: the GPU tests named
# by TESTS under each setting, then the bench per config, REPS times each.
# Usage: KNOB=XRT_TILE_PLAN VALUES="0 1" TESTS="fill_plan or frames_batch" tools/gpu_env_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-env_ab}; mkdir -p $OUT
for v in $VALUES; do
  if [ -n "$TESTS" ]; then
    env $KNOB=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "$TESTS" > $OUT/tests_$v.txt 2>&1 || { tail -30 $OUT/tests_$v.txt; exit 1; }
    echo "$KNOB=$v tests: $(tail -1 $OUT/tests_$v.txt)"
  fi
done
for rep in $(seq 1 ${REPS:-2}); do
for v in $VALUES; do
for cfg in "1024|--size 1024 1024" "2048|--size 2048 2048" "4096|--size 4096 4096 --steps 100 --warmup 10" "1m|--size 8192 8192 --tile-mesh 7 --steps 30 --warmup 5"; do
  IFS='|' read -r name args <<< "$cfg"
  f=$OUT/${v}_${name}_$rep
  env $KNOB=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-latency $args > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$f.json')); lo=d['at_loaded_clocks']
print('$KNOB=$v $name rep$rep step %.1f us loaded %.1f us span %.1f check %s' % (d['ms_per_step']*1e3, lo['ms_per_step']*1e3, d['roofline']['avg_kernel_ms']*1e3, d.get('frames_in_flight_exact')))"
done; done; done
