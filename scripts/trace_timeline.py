"""Timeline of one decode in a rocprofv3 kernel trace: the drp kernels from the k-th tile_prefix
launch (one per decode) to the next, with start offsets and durations.
Usage: python scripts/trace_timeline.py TRACE.csv [k (default: the last)]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "drp" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "tile_prefix" in r["Kernel_Name"] or "prologue_kernel" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) - 1
i0 = starts[k]
i1 = starts[k + 1] if k + 1 < len(starts) else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
end = t0
for r in rows[i0:i1]:
    name = r["Kernel_Name"].split("(")[0].replace("drp::spec::", "").replace("drp::", "").replace("void ", "")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    end = max(end, e)
    print(f"{(s - t0) / 1e6:8.3f} ms  {name:30s} {(e - s) / 1e6:7.3f} ms")
print(f"decode {k}: {(end - t0) / 1e6:.3f} ms from the first launch to the last kernel's end")
