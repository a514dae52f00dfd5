#!/bin/bash
# BASELINE configs[4]'s LDS batch-size sweep: the binned render's candidates
# per round (XRT_STAGE = 64 / 128 / 256: 1 / 2 / 4 footprints per lane per
# round; survivors' records still staged 64 at a time) at dragon 2048^2 and
# the 1.12M-triangle 8192^2 frame.  Variants from tools/build_variants.sh
# (st128, st256); 64 is the in-tree build.  Outputs gpurun_out/stage/stage{N}_{cfg}.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/stage
mkdir -p $OUT
L=simpleraytracing_amd/lib/var
for cfg in "2048|--size 2048 2048" "1m_8192|--size 8192 8192 --tile-mesh 7 --steps 100 --warmup 10"; do
  name=${cfg%%|*}; args=${cfg#*|}
  for st in 64 128 256; do
    lib=""; [ $st != 64 ] && lib=$L/libxrt_st$st.so
    XRT_LIB=$lib timeout -k 10 240 python bench.py --no-cpu-baseline --no-timing-check $args > $OUT/stage${st}_$name.json 2> $OUT/stage${st}_$name.err || { tail -3 $OUT/stage${st}_$name.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/stage${st}_$name.json')); r=d['roofline']; print('stage $st', '$name', 'step %.4f'%d['ms_per_step'], 'span %.4f'%r['avg_kernel_ms'])"
  done
done
