#!/bin/bash
# DESIGN.md section 9's strip model at loaded clocks (tools/transit_sizes.py):
# BASELINE configs[3] (dragon 4096^2) and configs[4] (1.12 M triangles at
# 8192^2), every split (weighted, equal, bench's balanced, the C ABI's own plan).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-strip_model}
mkdir -p $OUT
timeout -k 10 400 python3 tools/transit_sizes.py --size 4096 4096 > $OUT/strip_model_4096.json 2> $OUT/strip_model_4096.err || { tail -5 $OUT/strip_model_4096.err; exit 1; }
echo "4096 done"
timeout -k 10 500 python3 tools/transit_sizes.py --size 8192 8192 --tile-mesh 7 --ranks 2 4 8 --frames 8 --splits equal balanced capi > $OUT/strip_model_1m_8192.json 2> $OUT/strip_model_1m_8192.err || { tail -5 $OUT/strip_model_1m_8192.err; exit 1; }
echo "1m done"
