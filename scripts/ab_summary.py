"""Summarise gpurun_out/ab_*.log bench lines (scripts/gpu_ab.sh)."""
import glob
import json
import sys

for f in sorted(glob.glob("gpurun_out/ab_c*_*.log")):
    line = [l for l in open(f) if l.startswith("{")]
    if not line:
        print(f, "NO RESULT", open(f).read()[-300:])
        continue
    d = json.loads(line[-1])
    r = d["roofline"]
    extra = ""
    if "decode" in d:
        extra = f" enc {d['encode']['ms']:.2f} ms dec {d['decode']['ms']:.2f} ms repairs {d['decode']['repair_passes']} " \
                f"fallbacks {d['decode']['exact_fallbacks']}"
    else:
        extra = f" kernel {r['kernel_ms']:.2f} ms repairs {r['repair_passes']} fallbacks {r['exact_fallbacks']}"
    print(f"{f:40s} step {d['ms_per_step']:.3f} ms frac {r['frac']:.3f}{extra}")
