#!/bin/bash
# Bench kernel times of library variants (tools/build_variants.sh) at sizes:
#   tools/gpu_lib_bench.sh "name1 name2 ..." ["2048 1024 4096"]   (env passes through)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NAMES=$1; SIZES=${2:-"2048 1024 4096"}
for s in $SIZES; do
  for n in $NAMES; do
    lib=simpleraytracing_amd/lib/ab/libxrt_$n.so
    [ "$n" = "default" ] && lib=simpleraytracing_amd/lib/libxrt.so
    XRT_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --size $s $s > gpurun_out/lb.json 2> gpurun_out/lb.err || { tail -5 gpurun_out/lb.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/lb.json')); print('size $s $n', 'ms/step %.4f'%d['ms_per_step'], 'kernel %.4f'%d['roofline']['avg_kernel_ms'], 'Mrays/s %.0f'%d['value'])"
  done
done
