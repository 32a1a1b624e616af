"""Size sweep of the C2 decode (measurement only): decodes C2 streams of several sizes, REPS
times each, so a rocprofv3 kernel trace shows how the per-frame time of each kernel changes
when the wire fits the 256 MiB Infinity Cache (emission re-reads what the claims pass read).

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 scripts/probe_sizes.py
    python3 scripts/probe_sizes.py --summarize DIR/run_kernel_trace.csv
"""
import csv
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = [1_000_000, 2_000_000, 2_500_000, 4_000_000, 10_000_000, 40_000_000]
REPS = 6


def run():
    import torch
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "dat-replication-protocol_amd", "python"))
    import bench
    import drp_amd
    dev = torch.device("cuda", 0)
    ctx = drp_amd.Ctx(0)
    for n in SIZES:
        wire = bench.c2_on_device(n, seed=5, dev=dev)
        so = torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev)
        outs = bench.alloc_outputs(n + 64, dev)
        res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
        for _ in range(REPS):
            ctx.decode_device(wire, so, None, outs, n + 64, res)
        torch.cuda.synchronize(dev)
        bench.verify_c2(outs, res, n, dev)
        print(f"size {n} ok", flush=True)
        del wire, outs
        torch.cuda.empty_cache()
    ctx.close()


def summarize(path):
    rows = [r for r in csv.DictReader(open(path)) if "drp::spec" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = ["claims_fast", "emit_tiles<true>", "verify_lite"]
    seq = {k: [] for k in names}
    for r in rows:
        for k in names:
            if k in r["Kernel_Name"]:
                seq[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k in names:
        v = seq[k]
        print(k)
        for i, n in enumerate(SIZES):
            chunk = sorted(v[i * REPS + 1:(i + 1) * REPS])  # (first decode of a size: cold)
            if chunk:
                med = chunk[len(chunk) // 2]
                print(f"  {n:>10} frames  {med:8.3f} ms  {med * 1e9 / n:7.1f} ps/frame")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
