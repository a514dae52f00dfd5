#!/bin/bash
# Round evidence on one GPU: the GPU parity suite (optionally -k PATTERN),
# smoke(), the driver's bench command (20 steps, 5 warm-up), a 200-step bench
# and a rocprofv3 kernel-trace summary of a 50-step bench.
# Usage: tools/gpu_round.sh TAG [PATTERN]      (outputs under gpurun_out/TAG)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
K=()
if [ -n "$2" ]; then K=(-k "$2"); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err \
 && timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_200.json 2> $OUT/bench_200.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --no-latency --steps 50 --warmup 5 > $OUT/trace_bench.json 2> $OUT/trace.err
rc=$?
tail -3 $OUT/pytest_gpu.log
cat $OUT/smoke.log $OUT/bench_driver.json $OUT/bench_200.json 2>/dev/null | cut -c1-600
exit $rc
