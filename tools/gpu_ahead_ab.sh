L=simpleraytracing_amd/lib/var
for steps in "--steps 20 --warmup 5" "--steps 200 --warmup 20"; do
for rep in 1 2; do
for v in a2 a1; do
  XRT_LIB=$L/libxrt_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline $steps > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); r=d['roofline']; print('$v', '$steps', 'step %.4f'%d['ms_per_step'], 'span %.4f'%r['avg_kernel_ms'])"
done; done; done
