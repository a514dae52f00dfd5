#!/bin/bash
# Summarise the last gpu_check.sh outputs.
cd "$(dirname "$0")/.."
python3 - <<'PY'
import csv, json, os
print(open('gpurun_out/pytest_gpu.log').read().strip().splitlines()[-1] if os.path.exists('gpurun_out/pytest_gpu.log') else 'no pytest log')
for k in ('auto', 'binned', 'tiled', 'brute', 'rehearse2'):
    p = f'gpurun_out/bench_{k}.json'
    if not os.path.exists(p):
        print(k, 'missing'); continue
    d = json.loads(open(p).read().strip().splitlines()[-1])
    rs = d['render_stats']
    print(f"{k:7s} {d['value']:10.1f} Mrays/s  {d['ms_per_step']:.4f} ms/step  kernel {d['roofline']['avg_kernel_ms']:.4f} ms"
          f"  cand {rs['region_candidates']} tests {rs['wave_tile_tests']}"
          + (f"  cpu {d['cpu_baseline']['value']:.4f}" if d.get('cpu_baseline') else ''))
p = 'gpurun_out/prof_auto/run_kernel_stats.csv'
if os.path.exists(p):
    for r in csv.DictReader(open(p)):
        print('  ', r['Name'].split('(')[0][:40].ljust(42), r['Calls'], r['AverageNs'], r['Percentage'])
PY
