"""Per-kernel PMC summary of scripts/gpu_pmc.sh passes (gpurun_out/pmc/<pass>/): average per dispatch
and per frame, FETCH_SIZE doubled per the gfx950 note. Usage: python scripts/pmc_kernels.py [frames]"""
import collections
import csv
import glob
import sys

frames = float(sys.argv[1]) if len(sys.argv) > 1 else 20e6
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in glob.glob("gpurun_out/pmc/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "drp" not in k:
            continue
        k = k.split("(")[0].replace("drp::spec::", "").replace("drp::", "")
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add((f, r["Dispatch_Id"]))
kern = sorted({k for k, _ in tot})
for k in kern:
    avg = {c: tot[(kk, c)] / len(disp[(kk, c)]) for kk, c in tot if kk == k}
    if "FETCH_SIZE" in avg:
        avg["FETCH_SIZE"] *= 2
    w = avg.get("SQ_WAVES", 0)
    out = [f"{k:22s}"]
    for c in ["FETCH_SIZE", "WRITE_SIZE"]:
        if c in avg:
            out.append(f"{c[:5]}={avg[c] * 1024 / frames:6.1f}B/f")
    if w:
        out.append(f"waves={w:.0f}")
        for c in sorted(avg):
            if c.startswith("SQ_") and c != "SQ_WAVES":
                out.append(f"{c[3:]}={avg[c] / w:.0f}")
    print(" ".join(out))
