#!/bin/bash
# A/B of variant builds (tools/build_variants.sh) over several configs.
# Usage: tools/gpu_ab_multi.sh kernel "name1 name2 ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
K="${1:-binned}"
V=""
for n in $2; do V="$V $n=simpleraytracing_amd/lib/ab/libxrt_$n.so"; done
timeout -k 10 120 python tools/ab.py --kernel $K --variants $V --size 2048 2048 > gpurun_out/ab/2048.json 2> gpurun_out/ab/2048.err \
 && timeout -k 10 120 python tools/ab.py --kernel $K --variants $V --size 1024 1024 > gpurun_out/ab/1024.json 2> gpurun_out/ab/1024.err \
 && timeout -k 10 120 python tools/ab.py --kernel $K --variants $V --size 4096 4096 > gpurun_out/ab/4096.json 2> gpurun_out/ab/4096.err \
 && timeout -k 10 300 python tools/ab.py --kernel $K --variants $V --size 8192 8192 --tile-mesh 7 --rounds 3 --frames 3 > gpurun_out/ab/1m.json 2> gpurun_out/ab/1m.err
rc=$?
cat gpurun_out/ab/*.json; grep -h WARN gpurun_out/ab/*.err
exit $rc
