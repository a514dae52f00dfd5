#!/bin/bash
# Builds libxrt.so variants with extra -D flags for tools/ab.py:
#   tools/build_variants.sh name1 "-DFOO=1" name2 "-DFOO=0" ...
set -e
cd "$(dirname "$0")/../simpleraytracing_amd/csrc"
OUT=../lib/var
mkdir -p $OUT
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fno-fast-math \
      -I../../include -DXRT_KERNEL_NS=xrt_$name $flags -shared -o $OUT/libxrt_$name.so xrt_abi.hip \
      -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
done
wait
ls -la $OUT
