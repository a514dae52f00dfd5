#!/bin/bash
# Device-sized frames' k_size_lists / k_scatter_pairs on the prep stream
# (XRT_DEV_SIZE_ON_PREP): the moving-camera parity tests of each variant, then
# the bench's orbit legs with each, alternating, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06ac}
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=simpleraytracing_amd/lib/var
for v in sp0 sp1; do
  XRT_LIB=$L/libxrt_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "moving or orbit or first_frame or share_device or box_masks" > $OUT/pytest_$v.log 2>&1 || { tail -20 $OUT/pytest_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $OUT/pytest_$v.log)"
done
for rep in 1 2; do
  for v in sp0 sp1; do
    XRT_LIB=$L/libxrt_$v.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-latency --no-tile-plan-leg > $OUT/b_${v}_$rep.json 2> $OUT/b_${v}_$rep.err || { tail -5 $OUT/b_${v}_$rep.err; exit 1; }
    python3 - $OUT/b_${v}_$rep.json "$v rep $rep" <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
o = b.get("orbit") or {}
print(sys.argv[2], "value", round(b["value"]), " ".join(f"{k}: {v['ms_per_step']*1e3:.1f} us (fixed {v['fixed_camera_same_context_ms_per_step']*1e3:.1f}, x{v['vs_fixed_camera']:.2f}, exact {v['last_frames_bit_exact']})" for k, v in o.items() if isinstance(v, dict)))
PY
  done
done
