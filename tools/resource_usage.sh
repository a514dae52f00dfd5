#!/bin/bash
# Per-kernel VGPR/SGPR/LDS/occupancy of libxrt's kernels (compiler remarks).
cd "$(dirname "$0")/../simpleraytracing_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fno-fast-math \
    -I../../include "$@" --cuda-device-only -c -o /dev/null xrt_abi.hip -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c '
import re, sys
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m: continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": re.sub(r"^_ZN\w*?\d+(k_\w+?)E.*", r"\1", t.split(":",1)[1].strip())}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    print("%-24s VGPR %4s  SGPR %4s  LDS %6s  occ %s  scratch %s" % (r["name"][:24], r.get("VGPRs"), r.get("TotalSGPRs"),
          r.get("LDS Size [bytes/block]"), r.get("Occupancy [waves/SIMD]"), r.get("ScratchSize [bytes/lane]")))
'
