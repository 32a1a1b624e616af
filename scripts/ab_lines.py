"""Summarise bench JSON lines of a GPU session (gpurun_out/*.log): C2/C4 ms per step and roofline,
C5 encode/decode ms and repair passes. Usage: python scripts/ab_lines.py [dir]"""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for p in sorted(glob.glob(os.path.join(d, "*.log"))):
    line = None
    for s in open(p, errors="replace"):
        s = s.strip()
        if s.startswith("{") and '"metric"' in s:
            line = json.loads(s)
    if line is None:
        continue
    r = line.get("roofline", {})
    x = ""
    if "encode" in line:
        x = f" enc {line['encode']['ms']:.3f} dec {line['decode']['ms']:.3f} rep {line['decode']['repair_passes']}"
    else:
        x = f" kernel {r.get('kernel_ms', 0):.3f} rep {r.get('repair_passes')}"
    print(f"{os.path.basename(p):22s} ms/step {line['ms_per_step']:7.3f} frac {r.get('frac', 0):.3f}{x}")
