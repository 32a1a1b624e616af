"""Per-kernel, per-wave SQ counters from gpurun_out/pmcab/<variant>/ (scripts/gpu_pmc_ablate.sh).
Usage: python scripts/pmc_table.py v1 v2 ... [--kernel spec_claims]"""
import collections
import csv
import glob
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
kern = "spec_claims"
for a in sys.argv[1:]:
    if a.startswith("--kernel="):
        kern = a.split("=", 1)[1]
for v in args:
    fs = glob.glob(f"gpurun_out/pmcab/{v}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print(v, "no data")
        continue
    tot, disp = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(fs[0])):
        if kern in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    avg = {k: tot[k] / len(disp[k]) for k in tot}
    w = avg.get("SQ_WAVES", 1) or 1
    print(f"{v:10s} waves {w:10.0f} " + " ".join(f"{k[3:]}={avg[k] / w:.0f}" for k in sorted(avg) if k != "SQ_WAVES"))
