"""One-screen summary of a bench.py JSON line (C2 + c4/c5 sub-lines). Usage: python scripts/bench_summary.py LOG"""
import json
import sys

for line in open(sys.argv[1]):
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    r = d["roofline"]
    print(f"C2  {d['ms_per_step']:.3f} ms/step  {d['value'] / 1e9:.2f} G frames/s  frac {r['frac']:.3f}  "
          f"kernel {r['kernel_ms']:.3f} ms  repairs {r['repair_passes']} relisted {r['verify_relisted_tiles']}")
    c4 = d.get("c4")
    if c4:
        r = c4["roofline"]
        print(f"C4  {c4['ms_per_step']:.3f} ms/step  frac {r['frac']:.3f}  kernel {r['kernel_ms']:.3f} ms  "
              f"relisted {r['verify_relisted_tiles']}")
    c5 = d.get("c5") or (d if "encode" in d else None)
    if c5:
        print(f"C5  {c5['ms_per_step']:.3f} ms/step  frac {c5['roofline']['frac']:.3f}  encode {c5['encode']['ms']:.3f} ms "
              f"({c5['encode']['frac']:.3f})  decode {c5['decode']['ms']:.3f} ms ({c5['decode']['frac']:.3f}) "
              f"repairs {c5['decode']['repair_passes']}")
