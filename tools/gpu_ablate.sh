#!/bin/bash
# Ablation timing study of the culled kernels (outputs are wrong under XRT_ABLATE).
# Usage: tools/gpu_ablate.sh "binned tiled" "0 1 32 64 29"
# Needs the ablation build (production kernels ignore XRT_ABLATE), made on the
# CPU beforehand:  tools/build_variants.sh ablate "-DXRT_ABLATION=1"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ablate
export TMPDIR=/tmp
KS="${1:-tiled binned}"
AS="${2:-0 1 3 4 8 16 24 28 29 31 32 64}"
for k in $KS; do
  for a in $AS; do
    XRT_LIB=${XRT_LIB:-simpleraytracing_amd/lib/ab/libxrt_ablate.so} XRT_ABLATE=$a timeout -k 10 120 python bench.py --kernel $k --no-cpu-baseline --steps 20 > gpurun_out/ablate/${k}_$a.json 2>/dev/null || exit 1
  done
done
python3 - "$KS" "$AS" <<'PY'
import json, sys
for k in sys.argv[1].split():
    for a in sys.argv[2].split():
        d = json.loads(open(f"gpurun_out/ablate/{k}_{a}.json").read().strip().splitlines()[-1])
        print(k, a, round(d["ms_per_step"] * 1000, 1), round(d["roofline"]["avg_kernel_ms"] * 1000, 1))
PY
