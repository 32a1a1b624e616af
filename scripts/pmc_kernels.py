"""Per-kernel PMC summary of scripts/gpu_pmc.sh passes (gpurun_out/pmc/<pass>/): average per dispatch
and per frame, FETCH_SIZE doubled per the gfx950 note (MI355X_MICROARCH.md: 128-B requests
tallied at 64 B). Usage: python scripts/pmc_kernels.py [frames (default: from the passes' bench lines)] [--dir gpurun_out/pmc] [--workload c2|c3|c4|c5] [--calls N]
[--write profiles/pmc_<workload>.json] (c5: the encode kernels are counted too: its roofline prices the
round trip)"""
import collections
import csv
import glob
import json
import sys

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import DECODE_PATH as KNAME, decode_code_hash  # noqa: E402  (bench.py's kernel name and source hash)
PMC_DIR = sys.argv[sys.argv.index("--dir") + 1] if "--dir" in sys.argv else "gpurun_out/pmc"
WORKLOAD = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "c2"
# --calls N: the passes ran N whole decode calls of `frames` frames each, in dispatches of varying
# sizes (C3: a host batch staged in pieces); per-frame figures are then the kernels' totals over
# all dispatches / (frames x N), not per-dispatch averages
CALLS = float(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else None
opt_vals = {sys.argv[sys.argv.index(o) + 1] for o in ("--dir", "--write", "--workload", "--calls") if o in sys.argv}
args = [a for a in sys.argv[1:] if not a.startswith("--") and a not in opt_vals]


def frames_from_logs():
    """The frames one dispatch of the workload decodes, from the bench JSON line a pass logged
    (C2: frames_per_gpu; C4: frames_node; C5: the Changes per GPU in its workload string)."""
    import re
    for f in sorted(glob.glob(PMC_DIR + "/*.log")):
        for line in open(f, errors="replace"):
            if line.startswith('{"metric"'):
                cfg = json.loads(line).get("config", {})
                if "frames_per_gpu" in cfg:
                    return float(cfg["frames_per_gpu"])
                if "frames_node" in cfg:
                    return float(cfg["frames_node"])
                m = re.match(r"C5: (\d+) Changes", cfg.get("workload", ""))
                if m:
                    return float(m.group(1))
                if cfg.get("workload", "").startswith("C3") and "frames" in cfg:
                    return float(cfg["frames"])
    return None


frames = float(args[0]) if args else (frames_from_logs() or 20e6)
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in glob.glob(PMC_DIR + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "drp" not in k:
            continue
        k = k.split("(")[0].replace("drp::spec::", "").replace("drp::", "")
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add((f, r["Dispatch_Id"]))
kern = sorted({k for k, _ in tot})
per = {}
for k in kern:
    avg = {c: tot[(kk, c)] / (CALLS if CALLS else len(disp[(kk, c)])) for kk, c in tot if kk == k}
    if "FETCH_SIZE" in avg:
        avg["FETCH_SIZE"] *= 2
    w = avg.get("SQ_WAVES", 0)
    out = [f"{k:22s}"]
    rd = avg.get("FETCH_SIZE", 0) * 1024 / frames
    wr = avg.get("WRITE_SIZE", 0) * 1024 / frames
    per[k] = {"fetch_B_per_frame": round(rd, 2), "write_B_per_frame": round(wr, 2)}
    out.append(f"FETCH={rd:6.1f}B/f WRITE={wr:6.1f}B/f")
    if w:
        out.append(f"waves={w:.0f}")
        for c in sorted(avg):
            if c.startswith("SQ_") and c != "SQ_WAVES":
                out.append(f"{c[3:]}={avg[c] / w:.0f}")
                per[k][c] = round(avg[c] / w, 1)
    print(" ".join(out))
if "--write" in sys.argv:
    path = sys.argv[sys.argv.index("--write") + 1]
    dec = {k: v for k, v in per.items() if WORKLOAD == "c5" or not k.startswith("enc")}
    # the ctx's first decode (bench warmup) runs claims_fast<true>, the steady state <false>
    if "void claims_fast<false>" in dec and "void claims_fast<true>" in dec:
        dec.pop("void claims_fast<true>")
    for k in ("kernels", "code_hash"):
        assert k not in dec
    hbm = sum(v["fetch_B_per_frame"] + v["write_B_per_frame"] for v in dec.values())
    json.dump({"kernel": KNAME, "code_hash": decode_code_hash(), "kernels": sorted(dec), "workload": f"{WORKLOAD.upper()}, {frames:g} frames per dispatch "
               f"(scripts/gpu_pmc.sh {WORKLOAD})",
               "frames": frames, "note": "rocprofv3 --pmc, one pass per counter group (scripts/gpu_pmc.sh); "
               "FETCH_SIZE doubled per MI355X_MICROARCH.md; per wave for SQ counters",
               "hbm_bytes_per_frame": round(hbm, 2), "per_kernel": dec}, open(path, "w"), indent=1)
    print("wrote", path, "hbm B/frame", round(hbm, 1))
