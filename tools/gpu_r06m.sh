#!/bin/bash
# Box tile masks, second form (mask atomics issued last, buffer atomic OR):
# tools/gpu_prep_ab.sh's A/B of masks off / first form / second form, and the
# orbit legs of masks off and the second form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06m}
OUT=gpurun_out/$TAG
mkdir -p $OUT
VARIANTS="${AB:-nomask mask1 mask2}" tools/gpu_prep_ab.sh $TAG/ab || exit 1
for v in ${ORBIT:-nomask mask2}; do
  XRT_LIB=simpleraytracing_amd/lib/var/libxrt_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-latency --no-timing-check --no-tile-plan-leg > $OUT/orbit_$v.json 2> $OUT/orbit_$v.err || { tail -5 $OUT/orbit_$v.err; exit 1; }
  python3 -c "import json,sys; b=json.load(open(sys.argv[1])); o=b.get('orbit') or {}; print(sys.argv[2], round(b['value']), {k: (round(v['ms_per_step']*1e3,1), round(v['vs_fixed_camera'],2)) for k, v in o.items() if isinstance(v, dict) and 'ms_per_step' in v})" $OUT/orbit_$v.json $v
done
