#!/bin/bash
# Evidence for profiles/: for the binned render (the default bench) and the
# brute-force render (renderLoop as written), a rocprofv3 kernel-trace summary
# and PMC passes (each counter group in its own run: HBM traffic, instruction
# mix); then the brute bench line and the default bench line (with cpu_baseline).
# Usage: tools/gpu_round_profile.sh TAG     (outputs under gpurun_out/round_TAG)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
PASSES=("FETCH_SIZE" "WRITE_SIZE"
        "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES"
        "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
for K in binned brute; do
  if [ $K = binned ]; then B="bench.py --no-cpu-baseline"; P="--steps 8 --warmup 2"; else B="bench.py --no-cpu-baseline --kernel brute"; P="--steps 2 --warmup 1"; fi
  echo "[$K] kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${K}_trace -o run -- python3 $B $P > $OUT/${K}_trace_bench.json 2> $OUT/${K}_trace.err || exit 1
  i=0
  for grp in "${PASSES[@]}"; do
    i=$((i+1))
    echo "[$K] pmc pass $i: $grp"
    timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/${K}_pmc$i -o run -- python3 $B $P > /dev/null 2> $OUT/${K}_pmc$i.err || exit 1
  done
  mkdir -p $OUT/pmc_$K && cp -r $OUT/${K}_pmc* $OUT/pmc_$K/ 2>/dev/null
  python3 tools/pmc_summary.py $OUT/pmc_$K > $OUT/pmc_summary_$K.txt || exit 1
done
echo "[brute] bench"
timeout -k 10 300 python bench.py --no-cpu-baseline --kernel brute --steps 3 --warmup 1 > $OUT/bench_brute.json 2> $OUT/bench_brute.err || exit 1
echo "[binned] bench"
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json
