#!/bin/bash
# Round-6 evidence on one GPU: the whole GPU suite, smoke(), the driver's bench
# command, the same command under rocprofv3 --kernel-trace --stats, then every
# BASELINE config's traces + PMC + bench line (tools/gpu_configs.sh).
# Usage: tools/gpu_r06g.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
cut -c1-300 $OUT/bench_driver.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/driver_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/driver_trace_bench.json 2> $OUT/driver_trace.err || { tail -5 $OUT/driver_trace.err; exit 1; }
tools/gpu_configs.sh $TAG || exit 1
echo done
