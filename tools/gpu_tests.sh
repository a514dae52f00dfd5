#!/bin/bash
# GPU parity suite (optionally a -k pattern), smoke(), then the default bench.
# Usage: tools/gpu_tests.sh [PATTERN]     (logs under gpurun_out/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
K=()
if [ -n "$1" ]; then K=(-k "$1"); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread "${K[@]}" > gpurun_out/pytest_gpu.log 2>&1 \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -3 gpurun_out/pytest_gpu.log
cat gpurun_out/smoke.log gpurun_out/bench.json 2>/dev/null
exit $rc
