#!/bin/bash
# Ablation timing study of the culled kernels (outputs are wrong under XRT_ABLATE).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ablate
export TMPDIR=/tmp
for k in tiled binned; do
  for a in 0 1 3 4 8 16 24 28 29 31; do
    XRT_ABLATE=$a timeout -k 10 120 python bench.py --kernel $k --no-cpu-baseline --steps 20 > gpurun_out/ablate/${k}_$a.json 2>/dev/null || exit 1
  done
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LEVEL_WAVES --output-format csv -d gpurun_out/ablate/pmc1 -o run -- python3 bench.py --kernel tiled --no-cpu-baseline --steps 5 > /dev/null 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ablate/pmc2 -o run -- python3 bench.py --kernel tiled --no-cpu-baseline --steps 5 > /dev/null 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/ablate/pmc3 -o run -- python3 bench.py --kernel tiled --no-cpu-baseline --steps 5 > /dev/null 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/ablate/pmc4 -o run -- python3 bench.py --kernel tiled --no-cpu-baseline --steps 5 > /dev/null 2>&1
echo done
