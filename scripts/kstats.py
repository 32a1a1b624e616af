"""Print the drp kernels of a rocprofv3 kernel_stats.csv (average ms per call)."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "drp" in n:
        print(f"{n[:64]:64s} {r['Calls']:>4} {float(r['AverageNs']) / 1e6:8.3f} ms")
