#!/bin/bash
# Dispatch timelines of the steady-state bench (rocprofv3 kernel trace) for the
# given bench configurations: per-dispatch start/end/gap of the render and
# k_prep over the timed frames (tools/render_timeline.py).
# Usage: tools/gpu_timeline.sh TAG ["BENCH ARGS" ...]   (outputs under gpurun_out/TAG)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-tl}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
CFGS=("$@")
[ ${#CFGS[@]} -eq 0 ] && CFGS=("--size 2048 2048" "--size 1024 1024")
i=0
for cfg in "${CFGS[@]}"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl_$i -o run -- python3 bench.py --no-cpu-baseline --no-latency --steps 40 --warmup 5 $cfg > $OUT/bench_$i.json 2> $OUT/tl_$i.err || exit 1
  f=$(find $OUT/tl_$i -name "*kernel_trace.csv" | head -1)
  python3 tools/render_timeline.py "$f" > $OUT/timeline_$i.txt || exit 1
  echo "== $cfg"
  python3 -c "import json; d=json.load(open('$OUT/bench_$i.json')); print('ms/step %.4f'%d['ms_per_step'], 'event kernel_ms %.4f'%d['roofline']['avg_kernel_ms'])"
  tail -4 $OUT/timeline_$i.txt
done
