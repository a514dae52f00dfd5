#!/bin/bash
# A/B of variant builds (tools/build_variants.sh): bench lines per library.
# Usage: tools/gpu_ab_libs.sh "name1 name2 ..." ["--size 2048 2048" "--size 4096 4096" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NAMES="$1"; shift
CFGS=("$@"); [ ${#CFGS[@]} -eq 0 ] && CFGS=("--size 2048 2048" "--size 4096 4096" "--size 1024 1024")
for rep in 1 2; do
for n in $NAMES; do
  for cfg in "${CFGS[@]}"; do
    lib=simpleraytracing_amd/lib/ab/libxrt_$n.so; [ "$n" = base ] && lib=simpleraytracing_amd/lib/libxrt.so
    XRT_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 $cfg > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$n', '$cfg', 'ms/step %.4f'%d['ms_per_step'], 'kernel %.4f'%d['roofline']['avg_kernel_ms'])"
  done
done
done
