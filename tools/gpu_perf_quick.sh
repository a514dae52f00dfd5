#!/bin/bash
# Parity subset on the binned path, then bench lines at 2048^2 / 1024^2 / 4096^2
# and the 1.12M-tri 8192^2 frame (no CPU baseline).  Logs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PAT="${1:-golden or full_256 or ragged or overflow or deep_stack or corner or 2048 or 1024 or pipelined or device_buffers}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "$PAT" > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cfg in "--size 2048 2048" "--size 1024 1024" "--size 4096 4096" "--size 8192 8192 --tile-mesh 7 --steps 20 --warmup 3"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $cfg > gpurun_out/perf.json 2> gpurun_out/perf.err || { cat gpurun_out/perf.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/perf.json')); r=d['roofline']; print('$cfg', 'Mrays/s %.0f'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'kernel_ms %.4f'%r['avg_kernel_ms'], 'tests/ray %.2f'%d['render_stats']['ray_triangle_tests_per_ray'], 'overflow', d['render_stats']['overflow_rays'], 'cand', d['render_stats']['region_candidates'], 'glob', d['render_stats']['global_triangles'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pq_prof -o run -- python3 bench.py --no-cpu-baseline --steps 100 > /dev/null 2> gpurun_out/pq_prof.err || exit 1
f=$(find gpurun_out/pq_prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -6
XRT_PIPELINE=0 timeout -k 10 120 python tools/prep_stamps.py --lib simpleraytracing_amd/lib/ab/libxrt_stamps.so > gpurun_out/stamps.json 2>/dev/null && cat gpurun_out/stamps.json
for m in 2 0; do
  XRT_PIPELINE=$m timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/perf.json 2> gpurun_out/perf.err || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/perf.json')); r=d['roofline']; print('pipeline $m', 'Mrays/s %.0f'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'kernel_ms %.4f'%r['avg_kernel_ms'])"
done
XRT_LIB=simpleraytracing_amd/lib/ab/libxrt_g512.so timeout -k 10 300 python bench.py --no-cpu-baseline --size 8192 8192 --tile-mesh 7 --steps 20 --warmup 3 > gpurun_out/perf.json 2> gpurun_out/perf.err || exit 1
python3 -c "import json,sys; d=json.load(open('gpurun_out/perf.json')); r=d['roofline']; print('g512 tiled 8192', 'Mrays/s %.0f'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'kernel_ms %.4f'%r['avg_kernel_ms'], 'glob', d['render_stats']['global_triangles'], 'cand', d['render_stats']['region_candidates'])"
