#!/bin/bash
# Quick GPU check: selected tests (pattern $1) + tiled bench without CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PAT="${1:-footprint or golden}"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "$PAT" > gpurun_out/quick_pytest.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/quick_tiled.json 2> gpurun_out/quick_tiled.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/quick_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/quick_prof.err
