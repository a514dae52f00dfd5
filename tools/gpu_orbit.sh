#!/bin/bash
# A projection sweep (bench.py --orbit: every frame a new camera, 1 degree
# apart) against the fixed camera, 1024^2 / 2048^2 / 4096^2, with the host
# profile's geometry line (sizings, camera reuses, frames k_prep flagged).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/orbit
for s in ${SIZES:-1024 2048 4096}; do
 for o in ${ORBITS:-0 1}; do
  f=gpurun_out/orbit/o${o}_$s
  XRT_HOST_PROFILE=1 timeout -k 10 120 python bench.py --no-cpu-baseline --size $s $s --orbit $o --steps 60 --warmup 5 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f.json')); print('$s orbit $o', 'ms/step %.4f'%d['ms_per_step'], 'kernel %.4f'%d['roofline']['avg_kernel_ms'], 'Mrays/s %.0f'%d['value'])"
  grep "xrt geometry" $f.err || true
 done
done
