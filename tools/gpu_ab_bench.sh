#!/bin/bash
# Whole-step A/B of variant builds: bench.py per variant (LIBXRT override),
# interleaved twice, plus a kernel trace of the first variant.
# Usage: tools/gpu_ab_bench.sh "name1 name2 ..." [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abb
export TMPDIR=/tmp
V="$1"; shift
for round in 1 2; do
  for n in $V; do
    XRT_LIB=simpleraytracing_amd/lib/ab/libxrt_$n.so timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/abb/${n}_$round.json 2> gpurun_out/abb/${n}_$round.err || exit 1
  done
done
python3 - "$V" <<'PY'
import json, sys
for n in sys.argv[1].split():
    r = []
    for k in (1, 2):
        d = json.loads(open(f"gpurun_out/abb/{n}_{k}.json").read().strip().splitlines()[-1])
        r.append((round(d["ms_per_step"] * 1000, 1), round(d["roofline"]["avg_kernel_ms"] * 1000, 1), d["config"]["workload"]))
    print(n, r)
PY
