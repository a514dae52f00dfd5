#!/bin/bash
# Host cost of a moving frame: XRT_HOST_PROFILE=1 over an orbit run and a
# fixed-camera run (one xrt_render_rows_device call per frame).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for a in "--orbit 1" "--orbit 0.25" "--host-loop python"; do
  n=$(echo $a | tr -d ' -')
  XRT_HOST_PROFILE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-latency --orbit-legs --no-tile-plan-leg --loaded-ms 0 --steps 200 --warmup 5 $a > $OUT/hp_$n.json 2> $OUT/hp_$n.err || { tail -5 $OUT/hp_$n.err; exit 1; }
  echo "== $a: $(python3 -c "import json; d=json.load(open('$OUT/hp_$n.json')); print('%.1f us/step' % (d['ms_per_step']*1e3))")"
  grep "xrt host profile\|xrt geometry" $OUT/hp_$n.err | head -4
done
