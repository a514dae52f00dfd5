#!/bin/bash
# Every BASELINE.json config on one GPU (binned and tiled), plus the rocprof
# kernel-trace summary of the binned 2048^2 bench.  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/configs
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline"
timeout -k 10 120 $B --kernel binned --size 1024 1024 > $OUT/binned_1024.json 2> $OUT/binned_1024.err \
 && timeout -k 10 120 $B --kernel tiled --size 1024 1024 > $OUT/tiled_1024.json 2> $OUT/tiled_1024.err \
 && timeout -k 10 120 $B --kernel binned --size 4096 4096 > $OUT/binned_4096.json 2> $OUT/binned_4096.err \
 && timeout -k 10 120 $B --kernel tiled --size 4096 4096 > $OUT/tiled_4096.json 2> $OUT/tiled_4096.err \
 && timeout -k 10 200 $B --kernel binned --size 8192 8192 --tile-mesh 7 --steps 5 --warmup 1 > $OUT/binned_1m_8192.json 2> $OUT/binned_1m_8192.err \
 && timeout -k 10 120 $B --kernel tiled --size 2048 2048 > $OUT/tiled_2048.json 2> $OUT/tiled_2048.err \
 && timeout -k 10 120 $B --kernel brute --size 2048 2048 --steps 3 --warmup 1 > $OUT/brute_2048.json 2> $OUT/brute_2048.err \
 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_binned -o run -- python3 bench.py --no-cpu-baseline --kernel binned > $OUT/prof_binned.json 2> $OUT/prof_binned.err
rc=$?
for f in $OUT/*.json; do python3 -c "
import json,sys
try:
    d=json.loads(open('$f').read().strip().splitlines()[-1])
    print('$f', d['config']['workload'], d['config']['kernel'], 'Mrays/s %.0f'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'render %.4f'%d['roofline']['avg_kernel_ms'])
except Exception as e: print('$f', 'ERR', e)
"; done
exit $rc
