#!/bin/bash
# Orbit legs after a clock ramp, with the same-context fixed-camera step beside
# them: the default bench twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $BENCH_ARGS > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || { tail -5 $OUT/bench_$rep.err; exit 1; }
  python3 - $OUT/bench_$rep.json <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
lo = b.get("at_loaded_clocks") or {}
print("value", round(b["value"]), "step", round(b["ms_per_step"] * 1e3, 2), "loaded", round(lo.get("ms_per_step", 0) * 1e3, 2))
for k, v in (b.get("orbit") or {}).items():
    if isinstance(v, dict):
        print(k, "moving", round(v["ms_per_step"] * 1e3, 1), "fixed same ctx", round(v["fixed_camera_same_context_ms_per_step"] * 1e3, 1),
              "ratio", round(v["vs_fixed_camera"], 2), "vs main", round(v["vs_main_loop_step"], 2), "ramp frames", v["ramp_frames"],
              "sizings", v["sizings"], "overflows", v["overflows"], "exact", v["last_frames_bit_exact"])
PY
done
