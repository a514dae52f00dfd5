#!/bin/bash
# Device-sized first frames (XRT_DEVICE_FIRST, default on): the GPU suite, the
# first-frame probe with it on and off, the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head -20; exit $rc; }
for df in 1 0; do
  XRT_DEVICE_FIRST=$df timeout -k 10 120 python3 tools/first_frame_probe.py --host > $OUT/ff_$df.txt 2>&1 || { tail -5 $OUT/ff_$df.txt; exit 1; }
  echo "device_first=$df"; grep rep $OUT/ff_$df.txt
done
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; b=json.load(open('$OUT/bench.json')); l=b['latency']; print('value', round(b['value']), 'first_frame_ms', l['first_frame_ms'], 'e2e', l['end_to_end_ms'], 'child e2e', l['child_process']['end_to_end_ms'])"
