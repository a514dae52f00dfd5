#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel-trace summary.
# Every GPU step has its own time limit; steps are chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
  && timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_tiled.json 2> gpurun_out/bench_tiled.err \
  && timeout -k 10 300 python bench.py --steps 3 --warmup 1 --kernel brute --no-cpu-baseline > gpurun_out/bench_brute.json 2> gpurun_out/bench_brute.err
