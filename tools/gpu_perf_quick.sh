#!/bin/bash
# A GPU parity subset (-k PATTERN; "none" skips it), then bench lines at
# 1024^2 / 2048^2 / 4096^2 and the 1.12M-tri 8192^2 frame (no CPU baseline),
# one summary line each.  Logs under gpurun_out/quick.
# Usage: tools/gpu_perf_quick.sh [PATTERN] [CONFIGS...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/quick
mkdir -p $OUT
export TMPDIR=/tmp
PAT="${1:-golden or full_256 or ragged or overflow or corner or 2048 or 1024 or pipelined or device_buffers or fill_plan or moving or multi}"
shift
if [ "$PAT" != none ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$PAT" > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
i=0
CFGS=("$@")
if [ ${#CFGS[@]} -eq 0 ]; then
  CFGS=("--size 1024 1024" "--size 2048 2048" "--size 4096 4096" "--size 8192 8192 --tile-mesh 7 --steps 100 --warmup 10")
fi
[ "${CFGS[0]}" = none ] && exit 0
for cfg in "${CFGS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline $cfg > $OUT/perf_$i.json 2> $OUT/perf_$i.err
  rc=$?
  if [ $rc -ne 0 ]; then tail -2 $OUT/perf_$i.err; [ $rc -eq 1 ] && continue; exit $rc; fi
  python3 -c "import json,sys; d=json.load(open('$OUT/perf_$i.json')); r=d['roofline']; print('$cfg', 'Mrays/s %.0f'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'kernel_ms %.4f'%r['avg_kernel_ms'], 'ratio %.3f'%(d['ms_per_step']/r['avg_kernel_ms']), 'tests/ray %.2f'%d['render_stats']['ray_triangle_tests_per_ray'], 'first_ms %.3f'%d['latency']['first_frame_ms'])"
done
