#!/usr/bin/env python3
"""Prints the last N dispatches of a rocprofv3 kernel-trace CSV as a timeline
(start/end relative to the first shown, duration, gap to the previous)."""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    prev = e
    print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {gap:6.1f}  {r['Kernel_Name'][:50]}")
