#!/bin/bash
# Evidence for profiles/: rocprofv3 kernel-trace summary of the default bench,
# PMC passes (each counter group in its own run) for the render kernel's HBM
# traffic and instruction mix, then the default bench line (with cpu_baseline).
# Usage: tools/gpu_round_profile.sh TAG     (outputs under gpurun_out/round_TAG)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
B="bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace_bench.json 2> $OUT/trace.err || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 $B --steps 8 --warmup 2 > /dev/null 2> $OUT/pmc$i.err || exit 1
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt || exit 1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json
