"""Print the drp kernels of a rocprofv3 kernel_stats.csv (average ms per call)."""
import csv
import sys

top = int(sys.argv[2]) if len(sys.argv) > 2 else None  # (only the first `top` kernels)
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "drp" in r["Name"]]
for r in rows[:top]:
    print(f"{r['Name'][:64]:64s} {r['Calls']:>4} {float(r['AverageNs']) / 1e6:8.3f} ms")
