set -o pipefail
for v in st1 st2; do
  timeout -k 10 120 python tools/stamps.py --lib simpleraytracing_amd/lib/ab/libxrt_$v.so --kernel binned --out gpurun_out/stamps_$v.npy > gpurun_out/stamps_$v.txt 2>&1 || exit 1
done
