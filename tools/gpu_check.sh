#!/bin/bash
# One GPU session: parity tests, benches (auto / binned / tiled / brute),
# a 2-rank rehearsal of the multi-rank path on the one GPU, and the rocprof
# kernel-trace summary of the default bench.  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
  && timeout -k 10 300 python bench.py > gpurun_out/bench_auto.json 2> gpurun_out/bench_auto.err \
  && timeout -k 10 300 python bench.py --kernel binned --no-cpu-baseline > gpurun_out/bench_binned.json 2> gpurun_out/bench_binned.err \
  && timeout -k 10 300 python bench.py --kernel tiled --no-cpu-baseline > gpurun_out/bench_tiled.json 2> gpurun_out/bench_tiled.err \
  && timeout -k 10 300 python bench.py --kernel brute --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_brute.json 2> gpurun_out/bench_brute.err \
  && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --same-device --steps 5 > gpurun_out/bench_rehearse2.json 2> gpurun_out/bench_rehearse2.err \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_auto -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_auto.json 2> gpurun_out/prof_auto.err
