#!/usr/bin/env python3
"""profiles/traffic.json from a rocprofv3 PMC summary (tools/pmc_summary.py).

    python tools/make_traffic_json.py gpurun_out/round_r01/summary.json KEY [--kernel NAME]

KEY is bench.py's "<kernel>:<workload>" (e.g. "binned:dragon.ply 2048x2048").
HBM bytes per launch = FETCH_SIZE x 2 (gfx950 reports half of the bytes of a
wide streaming read: MI355X_MICROARCH.md, HBM section) + WRITE_SIZE, both in KB
per dispatch; the VALU instruction count per launch is SQ_INSTS_VALU.  The x 2
holds for contiguous reads (the region entries); a 64-B gather through an index
(the survivors' records) is counted at its full size
(tools/probes/fetch_calib.hip, profiles/r04e/fetch_calib.txt), so the true
bytes lie between hbm_bytes_per_launch_low (FETCH_SIZE x 1 + WRITE_SIZE) and
hbm_bytes_per_launch."""
import json
import os
import sys

src, key = sys.argv[1], sys.argv[2]
opts = dict(zip(sys.argv[3::2], sys.argv[4::2]))
kname = opts.get("--kernel", "k_render_" + key.split(":")[0])
# --source-as: the tracked copy the record cites (profiles/<round>/pmc_summary_<config>.json),
# where the summary is copied from gpurun_out/ (scratch) after the run
source = opts.get("--source-as", os.path.relpath(src))
summ = json.load(open(src))
row = next(v for k, v in summ.items() if k.endswith("::" + kname))
out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
try:
    data = json.load(open(out_path))
except (OSError, ValueError):
    data = {}
data[key] = {
    "kernel": kname,
    "fetch_kb_per_launch": row.get("FETCH_SIZE"),
    "write_kb_per_launch": row.get("WRITE_SIZE"),
    "hbm_bytes_per_launch": (2 * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024
    if "FETCH_SIZE" in row and "WRITE_SIZE" in row else None,
    "hbm_bytes_per_launch_low": (row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024
    if "FETCH_SIZE" in row and "WRITE_SIZE" in row else None,
    "valu_wave_instr_per_launch": row.get("SQ_INSTS_VALU"),
    "salu_instr_per_launch": row.get("SQ_INSTS_SALU"),
    "waves_per_launch": row.get("SQ_WAVES"),
    "source": source,
}
json.dump(data, open(out_path, "w"), indent=1, sort_keys=True)
print(json.dumps(data[key]))
