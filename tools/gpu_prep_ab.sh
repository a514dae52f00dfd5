#!/bin/bash
# k_prep A/B of libxrt variants (tools/build_variants.sh): per variant and
# config, the rocprofv3 kernel-trace means of k_prep and the render (a short
# bench under the tracer) and the bench's own step without the tracer; then a
# parity check of each variant (the binned-vs-brute GPU tests through XRT_LIB).
# Usage: VARIANTS="base rank256" tools/gpu_prep_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-prep_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=simpleraytracing_amd/lib/var
CONFIGS=("1m|--size 8192 8192 --tile-mesh 7|--steps 30 --warmup 5"
         "2048|--size 2048 2048|--steps 200 --warmup 20"
         "1024|--size 1024 1024|--steps 200 --warmup 20")
for v in ${VARIANTS:-base}; do
  for c in "${CONFIGS[@]}"; do
    IFS='|' read -r name cfg steps <<< "$c"
    d=$OUT/${v}_${name}
    XRT_LIB=$L/libxrt_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --no-cpu-baseline --no-latency --no-timing-check --loaded-ms 0 $cfg $steps > $d.trace.json 2> $d.trace.err || { tail -5 $d.trace.err; exit 1; }
    XRT_LIB=$L/libxrt_$v.so timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-latency --no-timing-check $cfg $steps > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
    python3 - "$d" "$v" "$name" <<'EOF'
import csv, glob, json, sys
d, v, name = sys.argv[1:4]
st = {}
for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = "k_prep" if "k_prep" in row["Name"] else "render" if "k_render" in row["Name"] else None
        if k:
            st[k] = float(row["AverageNs"]) / 1e3
b = json.load(open(d + ".json"))
lo = b.get("at_loaded_clocks") or {}
print(f"{v:12s} {name:5s} k_prep {st.get('k_prep', 0):9.1f} us  render {st.get('render', 0):9.1f} us | "
      f"step {b['ms_per_step'] * 1e3:8.1f} us  loaded {lo.get('ms_per_step', 0) * 1e3:8.1f} us  span "
      f"{b['roofline']['avg_kernel_ms'] * 1e3:8.1f} us", flush=True)
EOF
  done
done
for v in ${VARIANTS:-base}; do
  XRT_LIB=$L/libxrt_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 280 --timeout-method thread -k "overflow or all_kernels_equal_2048 or tiled_mesh_8192_strip_rows or binned_equals_brute_full_4096 or fill_plan or split_tiles" > $OUT/${v}_pytest.txt 2>&1 || { tail -20 $OUT/${v}_pytest.txt; exit 1; }
  echo "$v parity: $(tail -1 $OUT/${v}_pytest.txt)"
done
