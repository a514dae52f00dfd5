#!/bin/bash
# Every BASELINE.json config on one GPU, plus the LDS staging batch sweep
# (XRT_STAGE candidates staged per round, variant builds from
# tools/build_variants.sh named in $VARIANTS, e.g. "stage128 stage256") on dragon
# 2048^2 and the 1.12M-triangle tiled mesh at 8192^2.  Each GPU step has its own
# limit; a summary table at the end.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/configs
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline"
timeout -k 10 120 $B --size 1024 1024 > $OUT/binned_1024.json 2> $OUT/binned_1024.err \
 && timeout -k 10 120 $B --kernel tiled --size 1024 1024 > $OUT/tiled_1024.json 2> $OUT/tiled_1024.err \
 && timeout -k 10 120 $B --size 2048 2048 > $OUT/binned_2048.json 2> $OUT/binned_2048.err \
 && timeout -k 10 120 $B --size 4096 4096 > $OUT/binned_4096.json 2> $OUT/binned_4096.err \
 && timeout -k 10 120 $B --size 8192 8192 --steps 20 --warmup 3 > $OUT/binned_8192.json 2> $OUT/binned_8192.err \
 && timeout -k 10 200 $B --size 8192 8192 --tile-mesh 7 --steps 5 --warmup 2 > $OUT/binned_1m_8192.json 2> $OUT/binned_1m_8192.err \
 || exit 1
for v in ${VARIANTS:-}; do
  L=simpleraytracing_amd/lib/ab/libxrt_$v.so
  XRT_LIB=$L timeout -k 10 120 $B --size 2048 2048 > $OUT/${v}_2048.json 2> $OUT/${v}_2048.err \
   && XRT_LIB=$L timeout -k 10 200 $B --size 8192 8192 --tile-mesh 7 --steps 5 --warmup 2 > $OUT/${v}_1m_8192.json 2> $OUT/${v}_1m_8192.err \
   || exit 1
done
for f in $OUT/*.json; do python3 -c "
import json,sys
try:
    d=json.loads(open('$f').read().strip().splitlines()[-1])
    print('%-34s'%'$f'.split('/')[-1], d['config']['workload'], d['config']['kernel'], 'Mrays/s %.0f'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'render %.4f'%d['roofline']['avg_kernel_ms'], 'tests/ray %.2f'%d['render_stats']['ray_triangle_tests_per_ray'])
except Exception as e: print('$f', 'ERR', e)
"; done
