#!/bin/bash
# k_prep's stores before / after its binning (XRT_PREP_LATE_STORES variants):
# tools/gpu_prep_ab.sh's traces, steps and parity, then each variant's k_prep
# wave timeline at 2048^2 and at the 1.12 M-triangle 8192^2 frame.
# Usage: tools/gpu_r06b.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
VARIANTS="${VARIANTS:-early late}" tools/gpu_prep_ab.sh $TAG || exit 1
for v in ${VARIANTS:-early late}; do
  XRT_LIB=simpleraytracing_amd/lib/var/libxrt_$v.so timeout -k 10 120 python tools/prep_timeline.py --out $OUT/tl_${v}_2048.json > /dev/null 2> $OUT/tl_${v}_2048.err || { tail -5 $OUT/tl_${v}_2048.err; exit 1; }
  XRT_LIB=simpleraytracing_amd/lib/var/libxrt_$v.so timeout -k 10 200 python tools/prep_timeline.py --size 8192 8192 --tile-mesh 7 --frames 40 --out $OUT/tl_${v}_1m.json > /dev/null 2> $OUT/tl_${v}_1m.err || { tail -5 $OUT/tl_${v}_1m.err; exit 1; }
  python3 - $OUT/tl_${v}_2048.json $OUT/tl_${v}_1m.json $v <<'PY'
import json, sys
for f in sys.argv[1:3]:
    d = json.load(open(f)); b = d["beside"]; a = d["alone"][-1]
    ph = ["load_record", "footprint", "stage_scan", "union", "cells_small", "cells_large", "commit_stores"]
    for tag, x in (("alone", a), ("beside", b)):
        print(sys.argv[3], d["size"], tag, "span %.1f start p90 %.1f wave p50 %.1f |" % (x["span_us"], x["start_us"]["p90"], x["wave_us"]["p50"]),
              " ".join("%s %.2f" % (k, x[k + "_us"]["p50"]) for k in ph if k + "_us" in x))
PY
done
