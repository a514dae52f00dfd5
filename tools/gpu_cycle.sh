#!/bin/bash
# One GPU round trip of the build -> measure loop: the GPU parity suite (-k
# PATTERN; "all" = everything, "none" = skip), then step time and kernel span
# of each libxrt variant (VARIANTS="name=path ..."; "cur" = the in-tree build)
# at every BASELINE one-GPU config, interleaved per config.  Logs under
# gpurun_out/cycle.  Usage: tools/gpu_cycle.sh [PATTERN] [CONFIG...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cycle/${CYCLE_TAG:-run}_$(date +%H%M%S)_$$
mkdir -p $OUT
echo "[cycle] outputs in $OUT"
export TMPDIR=/tmp
PAT="${1:-all}"
shift
if [ "$PAT" != none ]; then
  K=(); [ "$PAT" != all ] && K=(-k "$PAT")
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
CFGS=("$@")
[ ${#CFGS[@]} -eq 0 ] && CFGS=("--size 2048 2048" "--size 1024 1024" "--size 4096 4096" "--size 8192 8192 --tile-mesh 7 --steps 100 --warmup 10")
[ "${CFGS[0]}" = none ] && exit 0
i=0
for cfg in "${CFGS[@]}"; do
  for v in ${VARIANTS:-cur=}; do
    name=${v%%=*}; lib=${v#*=}
    i=$((i+1))
    XRT_LIB=$lib timeout -k 10 240 python bench.py --no-cpu-baseline $cfg > $OUT/b_$i.json 2> $OUT/b_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then tail -5 $OUT/b_$i.err; exit $rc; fi
    python3 -c "import json; d=json.load(open('$OUT/b_$i.json')); r=d['roofline']; l=d['latency']; print('%-6s'%'$name', '%-36s'%'$cfg'[:36], 'Mrays/s %7.0f'%d['value'], 'step %.4f'%d['ms_per_step'], 'span %.4f'%r['avg_kernel_ms'], 'e2e %.2f'%l.get('end_to_end_ms', -1), 'r+d2h %.2f'%l.get('render_and_d2h_ms', -1), 'tests/ray %.2f'%d['render_stats']['ray_triangle_tests_per_ray']); b=l.get('render_and_d2h_breakdown_ms', {}); print('       slow host call:', {k: v for k, v in b.items() if v > 1.0}, 'camera %.2f'%l.get('camera_ms', 0)) if l.get('render_and_d2h_ms', 0) > 10 else None"
  done
done
