#!/bin/bash
# Orbit timelines under the kernel tracer, the stall probe's triggers, the
# driver's bench (latency windows before the host copies), k_prep's 8-stamp
# wave timeline.   Usage: tools/gpu_r06d.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for deg in 1 0.25 0; do
  if [ "$deg" = "0" ]; then a="--host-loop python"; else a="--orbit $deg"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/orbit_$deg -o run -- python3 bench.py --no-cpu-baseline --no-latency --no-timing-check --loaded-ms 0 --orbit-legs --steps 60 --warmup 5 $a > $OUT/orbit_$deg.json 2> $OUT/orbit_$deg.err || { tail -5 $OUT/orbit_$deg.err; exit 1; }
  echo "== orbit $deg"; python3 tools/trace_timeline.py $OUT/orbit_$deg --frames 6
done
timeout -k 10 200 python tools/evict_probe.py > $OUT/evict.json 2> $OUT/evict.err || { tail -20 $OUT/evict.err; exit 1; }
grep trigger $OUT/evict.err | cut -c1-260
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_driver.json')); o=d['orbit']; l=d['latency']
print('value %.0f ms %.4f' % (d['value'], d['ms_per_step']*1e3), 'e2e', l.get('end_to_end_ms'), 'fresh', l.get('again_fresh_buffers_ms'), 'child', l['child_process'].get('end_to_end_ms'))
for k in ('deg_0.25','deg_1'): print(k, {x: o[k][x] for x in ('ms_per_step','vs_fixed_camera','sizings','reused_lists','overflows','host_waits')})
"
timeout -k 10 120 python tools/prep_timeline.py --out $OUT/prep_2048.json > /dev/null 2> $OUT/prep_2048.err || { tail -5 $OUT/prep_2048.err; exit 1; }
timeout -k 10 200 python tools/prep_timeline.py --size 8192 8192 --tile-mesh 7 --frames 40 --out $OUT/prep_1m.json > /dev/null 2> $OUT/prep_1m.err || { tail -5 $OUT/prep_1m.err; exit 1; }
python3 - $OUT/prep_2048.json $OUT/prep_1m.json <<'PY'
import json, sys
ph = ["load_record", "footprint", "stage_scan", "union", "cells_small", "cells_large", "commit_stores"]
for f in sys.argv[1:]:
    d = json.load(open(f))
    for tag, x in (("alone", d["alone"][-1]), ("beside", d["beside"])):
        print(d["size"], tag, "span %.1f start p90 %.1f wave p50 %.1f |" % (x["span_us"], x["start_us"]["p90"], x["wave_us"]["p50"]),
              " ".join("%s %.2f/%.2f" % (k, x[k + "_us"]["p50"], x[k + "_us"]["p100"]) for k in ph if k + "_us" in x))
PY
