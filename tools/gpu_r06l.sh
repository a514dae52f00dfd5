#!/bin/bash
# Box tile masks (XRT_TILE_MASK): the whole GPU suite on the default build
# (masks on), tools/gpu_prep_ab.sh's A/B of masks off vs on, and the moving
# camera's orbit legs of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06l}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="nomask mask" tools/gpu_prep_ab.sh $TAG/ab || exit 1
for v in nomask mask; do
  XRT_LIB=simpleraytracing_amd/lib/var/libxrt_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-latency --no-timing-check --no-tile-plan-leg > $OUT/orbit_$v.json 2> $OUT/orbit_$v.err || { tail -5 $OUT/orbit_$v.err; exit 1; }
  python3 -c "import json,sys; b=json.load(open(sys.argv[1])); o=b.get('orbit') or {}; print(sys.argv[2], round(b['value']), {k: (round(v['ms_per_step']*1e3,1), round(v['vs_fixed_camera'],2)) for k, v in o.items() if isinstance(v, dict) and 'ms_per_step' in v})" $OUT/orbit_$v.json $v
done
