#!/bin/bash
# A/B kernel variants (tools/ab.py); args are passed through.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/ab.py "$@" > gpurun_out/ab.json 2> gpurun_out/ab.err
