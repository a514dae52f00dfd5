#!/bin/bash
# Ablation + workgroup-timeline study of the binned render (diagnostics).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB="${1:-simpleraytracing_amd/lib/ab/libxrt_stamps.so}"
bash tools/gpu_ablate.sh "binned" "0 1 4 8 16 24 29 32 64" > gpurun_out/ablate_summary.txt 2>&1 && \
timeout -k 10 120 python tools/stamps.py --lib $LIB --kernel binned > gpurun_out/stamps_binned.txt 2>&1
