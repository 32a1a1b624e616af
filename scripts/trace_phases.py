"""Per-workload kernel times of a `bench.py --no-cpu` rocprofv3 kernel trace (C2, then C4, then C5:
warmup + steps decodes each): the dispatches of each drp kernel in time order, split into the three
phases by the tile_prefix launches (one per decode). Usage: python scripts/trace_phases.py TRACE.csv [per]"""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "drp" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 7  # decodes per phase (warmup + steps)
phase, seen = 0, 0
acc = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("drp::spec::", "").replace("drp::", "").replace("void ", "")
    if k.startswith("tile_prefix_kernel") or k.startswith("prologue_kernel"):
        seen += 1
        phase = (seen - 1) // per
    acc[(phase, k)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
names = ["C2", "C4", "C5"]
for ph in range(3):
    items = sorted(((k, v) for (p, k), v in acc.items() if p == ph), key=lambda kv: -sum(kv[1]))
    tot = 0.0
    print(f"{names[ph] if ph < 3 else ph}:")
    for k, v in items:
        steady = sorted(v[2:] if len(v) > 3 else v)
        med = steady[len(steady) // 2]
        if med * len(v) / per < 0.002:
            continue
        tot += med * len(v) / per
        print(f"  {k:34s} {len(v):3d} calls  median {med:7.3f} ms")
    print(f"  sum of medians per decode ~ {tot:.3f} ms")
