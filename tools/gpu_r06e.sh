#!/bin/bash
# Moving camera with the pair scatter; the driver's bench; the orbit's kernel
# timeline.   Usage: tools/gpu_r06e.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "moving_camera or orbit or fixture or prepared_ahead or frames_in_flight or overflow or fill_plan" > $OUT/pytest_sel.log 2>&1
rc=$?; tail -3 $OUT/pytest_sel.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_driver.json')); o=d['orbit']; l=d['latency']
print('value %.0f ms %.4f' % (d['value'], d['ms_per_step']*1e3), 'e2e', l.get('end_to_end_ms'), 'fresh', l.get('again_fresh_buffers_ms'), 'child', l['child_process'].get('end_to_end_ms'))
for k in ('deg_0.25','deg_1'): print(k, {x: o[k][x] for x in ('ms_per_step','vs_fixed_camera','sizings','reused_lists','overflows','host_waits')})
"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/orbit_1 -o run -- python3 bench.py --no-cpu-baseline --no-latency --no-timing-check --loaded-ms 0 --orbit-legs --steps 60 --warmup 5 --orbit 1 > $OUT/orbit_1.json 2> $OUT/orbit_1.err || { tail -5 $OUT/orbit_1.err; exit 1; }
python3 tools/trace_timeline.py $OUT/orbit_1 --frames 5
