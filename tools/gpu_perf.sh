#!/bin/bash
# Parity subset + kernel timings of the culled kernels (no CPU baseline).
# Usage: tools/gpu_perf.sh [pytest -k pattern] [kernels]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/perf
export TMPDIR=/tmp
PAT="${1:-golden or kernels_equal or footprint or overflow or degenerate}"
KS="${2:-binned tiled}"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "$PAT" > gpurun_out/perf/pytest.log 2>&1
rc=$?
tail -2 gpurun_out/perf/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then exit $rc; fi
for k in $KS; do
  timeout -k 10 200 python bench.py --kernel $k --no-cpu-baseline --steps 30 > gpurun_out/perf/$k.json 2> gpurun_out/perf/$k.err || exit 1
done
python3 - "$KS" <<'PY'
import json, sys
for k in sys.argv[1].split():
    d = json.loads(open(f"gpurun_out/perf/{k}.json").read().strip().splitlines()[-1])
    print(k, "ms/step %.1f us" % (d["ms_per_step"] * 1000), "render %.1f us" % (d["roofline"]["avg_kernel_ms"] * 1000),
          "Mrays/s %.0f" % d["value"])
PY
