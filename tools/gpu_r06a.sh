#!/bin/bash
# Round 6, first GPU pass: the GPU suite, the driver's bench command (tile plan
# off in `value`, orbit legs beside it) and k_prep's wave timeline.
# Usage: tools/gpu_r06a.sh TAG [PATTERN]        (outputs under gpurun_out/TAG)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
K=()
if [ -n "$2" ]; then K=(-k "$2"); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
cut -c1-400 $OUT/bench_driver.json
timeout -k 10 120 python tools/prep_timeline.py --out $OUT/prep_2048.json > /dev/null 2> $OUT/prep_2048.err || { tail -20 $OUT/prep_2048.err; exit 1; }
timeout -k 10 200 python tools/prep_timeline.py --size 8192 8192 --tile-mesh 7 --frames 40 --out $OUT/prep_1m.json > /dev/null 2> $OUT/prep_1m.err || { tail -20 $OUT/prep_1m.err; exit 1; }
echo done
