#!/bin/bash
# A/B of library variants (tools/build_variants.sh) with tools/host_loop.py,
# alternating: tools/gpu_lib_ab.sh rounds name1 name2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$1; shift
for r in $(seq 1 $R); do
  for n in "$@"; do
    echo "== $n round $r"
    XRT_LIB=simpleraytracing_amd/lib/ab/libxrt_$n.so timeout -k 10 120 python tools/host_loop.py 2>&1 | grep timed || exit 1
  done
done
