#!/bin/bash
# Kernel-trace summaries and PMC counter passes for the two render kernels.
# Counters are collected in their own runs (one --pmc group per pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="bench.py --no-cpu-baseline"
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tiled -o run -- python3 $B --steps 20 --warmup 3 > $OUT/tiled_bench.json 2> $OUT/tiled.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/brute -o run -- python3 $B --kernel brute --steps 3 --warmup 1 > $OUT/brute_bench.json 2> $OUT/brute.err \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/tiled_fetch -o run -- python3 $B --steps 5 --warmup 1 > /dev/null 2> $OUT/tiled_fetch.err \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/tiled_write -o run -- python3 $B --steps 5 --warmup 1 > /dev/null 2> $OUT/tiled_write.err \
 && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/tiled_sq -o run -- python3 $B --steps 5 --warmup 1 > /dev/null 2> $OUT/tiled_sq.err \
 && timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT/tiled_sq2 -o run -- python3 $B --steps 5 --warmup 1 > /dev/null 2> $OUT/tiled_sq2.err \
 && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/brute_sq -o run -- python3 $B --kernel brute --steps 2 --warmup 1 > /dev/null 2> $OUT/brute_sq.err
echo "rc=$?"
find $OUT -name "*.csv" | head -50
