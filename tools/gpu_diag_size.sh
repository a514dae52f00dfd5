#!/bin/bash
# Where a frame size's time goes: bench (pipelined and XRT_PIPELINE=0), the
# ablation build's XRT_ABLATE 0 / 1 / 32, the workgroup timeline (stamps build)
# and a rocprof kernel-trace summary (k_prep beside the render).
# Usage: tools/gpu_diag_size.sh SIZE      (needs tools/build_variants.sh ablate / stamps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=${1:-1024}
OUT=gpurun_out/diag_$S
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --size $S $S --steps 100"
row() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'ms/step %.4f'%d['ms_per_step'], 'kernel %.4f'%d['roofline']['avg_kernel_ms'], 'Mrays/s %.0f'%d['value'])" "$@"; }
timeout -k 10 120 $B > $OUT/default.json 2> $OUT/default.err && row $OUT/default.json default || exit 1
XRT_PIPELINE=0 timeout -k 10 120 $B > $OUT/serial.json 2> $OUT/serial.err && row $OUT/serial.json serial || exit 1
for a in 0 1 32; do
  XRT_LIB=simpleraytracing_amd/lib/ab/libxrt_ablate.so XRT_ABLATE=$a timeout -k 10 120 $B > $OUT/ablate_$a.json 2> $OUT/ablate_$a.err && row $OUT/ablate_$a.json ablate_$a || exit 1
done
timeout -k 10 120 python tools/stamps.py --lib simpleraytracing_amd/lib/ab/libxrt_stamps.so --size $S $S > $OUT/stamps.json 2> $OUT/stamps.err || exit 1
cat $OUT/stamps.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --size $S $S --steps 50 > $OUT/prof.json 2> $OUT/prof.err || exit 1
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
