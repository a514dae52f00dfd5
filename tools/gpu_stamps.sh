set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && XRT_PIPELINE=0 timeout -k 10 120 python tools/prep_stamps.py --lib simpleraytracing_amd/lib/ab/libxrt_stamps.so > gpurun_out/stamps.json 2>&1; cat gpurun_out/stamps.json
