#!/bin/bash
# Every one-GPU BASELINE.json config with its own counter record: per config a
# rocprofv3 kernel-trace summary, PMC passes (HBM bytes, instruction mix, wait
# states; each counter group in its own run), the record added to
# profiles/traffic.json (copied to the output), then the bench line, which reads
# that record for its VALU roofline.  Each GPU step has its own time limit.
# Usage: tools/gpu_configs.sh TAG        (outputs under gpurun_out/configs_TAG)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03}
OUT=gpurun_out/configs_$TAG
mkdir -p $OUT
PASSES=("FETCH_SIZE" "WRITE_SIZE"
        "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES"
        "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
# name | bench arguments | short run for the counters | workload key (bench.py)
CONFIGS_ALL=(
  "1024|--size 1024 1024|--steps 8 --warmup 2|dragon.ply 1024x1024"
  "2048|--size 2048 2048|--steps 8 --warmup 2|dragon.ply 2048x2048"
  "4096|--size 4096 4096|--steps 8 --warmup 2|dragon.ply 4096x4096"
  "8192|--size 8192 8192 --steps 100 --warmup 10|--steps 4 --warmup 2|dragon.ply 8192x8192"
  "1m_8192|--size 8192 8192 --tile-mesh 7 --steps 100 --warmup 10|--steps 4 --warmup 2|dragon.ply tiled 7x7 8192x8192"
)
# ONLY="2048 1m_8192" limits the run to those configs
CONFIGS=()
for c in "${CONFIGS_ALL[@]}"; do
  n=${c%%|*}
  if [ -z "$ONLY" ] || [[ " $ONLY " == *" $n "* ]]; then CONFIGS+=("$c"); fi
done
for c in "${CONFIGS[@]}"; do
  IFS='|' read -r name args short key <<< "$c"
  base=$(echo "$args" | sed -e 's/--steps [0-9]*//' -e 's/--warmup [0-9]*//')
  echo "[$name] kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${name}_trace -o run -- python3 bench.py --no-cpu-baseline --no-latency --no-timing-check --orbit-legs --no-tile-plan-leg $base $short > $OUT/${name}_trace_bench.json 2> $OUT/${name}_trace.err || exit 1
  i=0
  for grp in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/${name}_pmc/p$i -o run -- python3 bench.py --no-cpu-baseline --no-latency --ramp-ms 0 --no-timing-check --orbit-legs --no-tile-plan-leg $base $short > /dev/null 2> $OUT/${name}_pmc$i.err || exit 1
  done
  python3 tools/pmc_summary.py $OUT/${name}_pmc > $OUT/pmc_summary_${name}.txt || exit 1
  python3 tools/make_traffic_json.py $OUT/${name}_pmc/summary.json "binned:$key" --kernel "k_render_binned<false>" --source-as profiles/$TAG/pmc_summary_${name}.json > /dev/null || exit 1
  echo "[$name] bench"
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $OUT/bench_${name}.json 2> $OUT/bench_${name}.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench_${name}.json')); r=d['roofline']; print('$name', 'Mrays/s %.0f'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'kernel_ms %.4f'%r['avg_kernel_ms'], r['bound'], 'frac %.3f'%r['frac'])"
done
cp profiles/traffic.json $OUT/traffic.json
