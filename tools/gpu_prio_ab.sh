set -o pipefail
for r in 1 2; do
XRT_PREP_PRIORITY=0 timeout -k 10 120 python bench.py --no-cpu-baseline --kernel binned > gpurun_out/prio0_$r.json 2>/dev/null || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --kernel binned > gpurun_out/prio1_$r.json 2>/dev/null || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_prio -o run -- python3 bench.py --no-cpu-baseline --kernel binned > /dev/null 2>&1
for f in gpurun_out/prio*_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step']*1000,1), round(d['roofline']['avg_kernel_ms']*1000,1))"; done
