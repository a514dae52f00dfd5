#!/bin/bash
# Tight region rectangles (XRT_BIN_TIGHT): the whole GPU suite on the default
# build (tight), then tools/gpu_prep_ab.sh's A/B of loose vs tight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06j}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="loose tight" tools/gpu_prep_ab.sh $TAG/ab || exit 1
VARIANTS="loose tight" tools/gpu_prep_ab.sh $TAG/ab2 || exit 1
