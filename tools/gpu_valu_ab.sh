#!/bin/bash
# VALU attribution / A/B of libxrt variants (simpleraytracing_amd/lib/var,
# built with -DXRT_KERNEL_NS=xrt_<name>): per variant and config one PMC pass
# (instruction counts of the render) and the bench step (loaded clocks).
# Usage: VARIANTS="base noshade" CONFIGS="4096 1m" tools/gpu_valu_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-valu_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=simpleraytracing_amd/lib/var
declare -A CFG=(["1024"]="--size 1024 1024" ["2048"]="--size 2048 2048" ["4096"]="--size 4096 4096"
                ["8192"]="--size 8192 8192" ["1m"]="--size 8192 8192 --tile-mesh 7")
for v in ${VARIANTS:-base}; do
  for c in ${CONFIGS:-4096}; do
    d=$OUT/${v}_$c
    XRT_LIB=$L/libxrt_$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $d -o run -- python3 bench.py --no-cpu-baseline --no-latency --no-timing-check --loaded-ms 0 ${CFG[$c]} --steps 6 --warmup 2 > /dev/null 2> $d.pmc.err || { tail -5 $d.pmc.err; exit 1; }
    python3 tools/pmc_summary.py $d > /dev/null || exit 1
    XRT_LIB=$L/libxrt_$v.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-latency --no-timing-check ${CFG[$c]} --steps 50 --warmup 5 > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
    python3 - "$d" "$v" "$c" <<'PY'
import json, sys
d, v, c = sys.argv[1:4]
s = json.load(open(d + "/summary.json"))
k = [k for k in s if "k_render_binned" in k and "true" not in k][0]
r = s[k]
b = json.load(open(d + ".json"))
lo = b.get("at_loaded_clocks") or {}
w = r["SQ_WAVES"]
print(f"{v:10s} {c:5s} VALU/wave {r['SQ_INSTS_VALU'] / w:7.1f} SALU/wave {r['SQ_INSTS_SALU'] / w:6.1f} "
      f"LDS/wave {r['SQ_INSTS_LDS'] / w:5.1f} VMEM/wave {r['SQ_INSTS_VMEM_RD'] / w:5.1f} waves {w:9.0f} | "
      f"step {b['ms_per_step'] * 1e3:8.1f} loaded {lo.get('ms_per_step', 0) * 1e3:8.1f} us", flush=True)
PY
  done
done
