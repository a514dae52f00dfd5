#!/bin/bash
# Moving camera on device-sized lists, the committed fixtures, the exit test;
# the driver's bench (orbit legs); the stall probe; k_prep 16 vs 32 triangles
# per wave.   Usage: tools/gpu_r06c.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "moving_camera or fixture or orbit or tile_plan or prepared_ahead or frames_in_flight or exit or fill_plan or overflow" > $OUT/pytest_sel.log 2>&1
rc=$?; tail -3 $OUT/pytest_sel.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_driver.json')); o=d['orbit']
print('value %.0f ms %.4f' % (d['value'], d['ms_per_step']*1e3), 'e2e', d['latency'].get('end_to_end_ms'))
for k in ('deg_0.25','deg_1'): print(k, {x: o[k][x] for x in ('ms_per_step','vs_fixed_camera','sizings','reused_lists','overflows','host_waits')})
"
timeout -k 10 200 python tools/evict_probe.py > $OUT/evict.json 2> $OUT/evict.err || { tail -20 $OUT/evict.err; exit 1; }
cat $OUT/evict.err | cut -c1-200
VARIANTS="t32 t16" tools/gpu_prep_ab.sh $TAG/prep || exit 1
