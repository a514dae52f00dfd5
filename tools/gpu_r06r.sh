#!/bin/bash
# Shared device streams (acquire_streams): the GPU suite, the probe with a busy
# second context, and the bench (fresh-context orbit legs) twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/still_after_moving.py --bench-leg --extra-contexts 1 --busy-extra > $OUT/probe_busy.txt 2>&1 || { tail -5 $OUT/probe_busy.txt; exit 1; }
grep "us per frame" $OUT/probe_busy.txt
tools/gpu_r06q.sh $TAG/q || exit 1
