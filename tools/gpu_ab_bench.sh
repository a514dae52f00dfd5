#!/bin/bash
# Step time and kernel span of libxrt variants (tools/build_variants.sh) through bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
export TMPDIR=/tmp
L=simpleraytracing_amd/lib/var
for v in ${VARIANTS:-base noprio}; do
  for cfg in "--size 2048 2048" "--size 1024 1024" "--size 4096 4096" "--size 8192 8192 --tile-mesh 7 --steps 100 --warmup 10"; do
    XRT_LIB=$L/libxrt_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-timing-check $cfg > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -5 gpurun_out/ab_bench.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.json')); r=d['roofline']; print('$v', '$cfg'[:16], 'step %.4f'%d['ms_per_step'], 'span %.4f'%r['avg_kernel_ms'], 'events %s'%r['avg_kernel_ms_hip_events'])"
  done
done
