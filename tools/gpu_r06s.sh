#!/bin/bash
# Device fill plan for moving frames (XRT_DEVICE_FILL, default on): the moving
# camera's parity tests, then the bench's orbit legs with it off / on, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "moving or orbit or box_masks or share_device or frames_in_flight or prepared_ahead" > $OUT/pytest_sel.log 2>&1
rc=$?; tail -2 $OUT/pytest_sel.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for df in 0 1; do
    XRT_DEVICE_FILL=$df timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-latency --no-tile-plan-leg > $OUT/b_${df}_$rep.json 2> $OUT/b_${df}_$rep.err || { tail -5 $OUT/b_${df}_$rep.err; exit 1; }
    python3 - $OUT/b_${df}_$rep.json "fill=$df rep $rep" <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
o = b.get("orbit") or {}
print(sys.argv[2], "value", round(b["value"]), " ".join(f"{k}: {v['ms_per_step']*1e3:.1f} us (fixed {v['fixed_camera_same_context_ms_per_step']*1e3:.1f}, x{v['vs_fixed_camera']:.2f}, main x{v['vs_main_loop_step']:.2f}, exact {v['last_frames_bit_exact']})" for k, v in o.items() if isinstance(v, dict)))
PY
  done
done
