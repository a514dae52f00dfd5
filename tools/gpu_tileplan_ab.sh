#!/bin/bash
# A/B of the tile plan (XRT_TILE_PLAN=1 default vs 0) through bench.py at the
# BASELINE configs, alternating, each a cold 200-step region and its
# loaded-clock twin; then the tile-plan tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-tileplan_ab}
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "2048|--size 2048 2048" "1024|--size 1024 1024" "4096|--size 4096 4096" "1m|--size 8192 8192 --tile-mesh 7 --steps 60 --warmup 5"; do
    IFS='|' read -r name args <<< "$cfg"
    for tp in 1 0; do
      XRT_TILE_PLAN=$tp timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-latency --no-timing-check $args > $OUT/${name}_tp${tp}_$rep.json 2> $OUT/${name}_tp${tp}_$rep.err || { tail -5 $OUT/${name}_tp${tp}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${name}_tp${tp}_$rep.json')); l=d['at_loaded_clocks']; print('$name tp$tp rep$rep step %.1f us loaded %.1f us span %.1f us' % (d['ms_per_step']*1e3, l['ms_per_step']*1e3, d['roofline']['avg_kernel_ms']*1e3))"
    done
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 280 --timeout-method thread -k "tile_plan or fill_plan or prepared_ahead or frames_in_flight or all_kernels_equal" > $OUT/pytest.txt 2>&1; echo "pytest rc=$? $(tail -1 $OUT/pytest.txt)"
