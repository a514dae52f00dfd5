#!/bin/bash
# k_size_lists / k_scatter_pairs on the render's stream: the moving-camera
# tests, two driver benches (orbit legs), the orbit's kernel timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06h}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "moving_camera or orbit or prepared_ahead or frames_in_flight or overflow" > $OUT/pytest_sel.log 2>&1
rc=$?; tail -3 $OUT/pytest_sel.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --steps 20 --warmup 5 > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || { tail -20 $OUT/bench_$rep.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$rep.json')); o=d['orbit']
print('rep $rep value %.0f ms %.4f' % (d['value'], d['ms_per_step']*1e3), ' '.join('%s %.1f us (%.2fx)' % (k, o[k]['ms_per_step']*1e3, o[k]['vs_fixed_camera']) for k in ('deg_0.25','deg_1')))
"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/orbit_1 -o run -- python3 bench.py --no-cpu-baseline --no-latency --no-timing-check --loaded-ms 0 --orbit-legs --steps 60 --warmup 5 --orbit 1 > $OUT/orbit_1.json 2> $OUT/orbit_1.err || { tail -5 $OUT/orbit_1.err; exit 1; }
python3 tools/trace_timeline.py $OUT/orbit_1 --frames 5
