#!/bin/bash
# A/B of variant builds under rocprofv3 --kernel-trace --stats: per-kernel
# averages of every variant (kernel names carry the variant namespace).
# Usage: tools/gpu_ab_prof.sh kernel "name1 name2 ..." [size W H]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abprof
export TMPDIR=/tmp
K="${1:-binned}"
V=""
for n in $2; do V="$V $n=simpleraytracing_amd/lib/ab/libxrt_$n.so"; done
SZ="${3:-2048 2048}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abprof/run -o run -- python3 tools/ab.py --kernel $K --variants $V --size $SZ > gpurun_out/abprof/ab.json 2> gpurun_out/abprof/ab.err
rc=$?
cat gpurun_out/abprof/ab.json
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/abprof/run/run_kernel_stats.csv")):
    print("%-60s %6s %9.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
exit $rc
