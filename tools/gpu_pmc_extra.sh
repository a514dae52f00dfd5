#!/bin/bash
# Extra PMC passes on the render (latency levels, LDS conflicts, issue mix) for
# one bench configuration.  Usage: tools/gpu_pmc_extra.sh TAG [BENCH ARGS]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-extra}; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
PASSES=("SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES"
        "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES"
        "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LEVEL_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY")
i=0
for grp in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py --no-cpu-baseline --no-latency --ramp-ms 0 --no-timing-check --steps 8 --warmup 2 "$@" > /dev/null 2> $OUT/p$i.err || exit 1
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
