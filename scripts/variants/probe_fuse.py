"""Probe (measurement, not product code): claims_fast's in-kernel emission (fuse_tile) on C2-shaped
streams of a few sizes: decode time with DRP_FUSE on and off and, with DRP_STATS=1, its outcome
counters (rows written, unproven tiles, timed-out waits, wait cycles). Usage:
python scripts/probe_fuse.py [frames ...]"""
import ctypes as C
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(nframes, fuse, stats):
    os.environ["DRP_FUSE"] = str(fuse)
    if stats:
        os.environ["DRP_STATS"] = "1"
    import torch
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda", 0)
    wire = bench.c2_on_device(nframes, seed=1234, dev=dev)
    so = torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev)
    cap = nframes + 64
    outs = bench.alloc_outputs(cap, dev)
    res = torch.zeros(C.sizeof(bench.drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    ctx = bench.drp_amd.Ctx(0)
    ctx.decode_device(wire, so, None, outs, cap, res)
    torch.cuda.synchronize()
    bench.verify_c2(outs, res, nframes, dev)
    ms = []
    for _ in range(1 if stats else 5):
        ctx.decode_device(wire, so, None, outs, cap, res)
        torch.cuda.synchronize()
        ms.append(ctx.timing().decode_ms)
    t = ctx.timing()
    print(f"frames={nframes} fuse={fuse} stats={stats}: decode_ms min {min(ms):.3f} repairs {t.spec_repairs} "
          f"relisted {t.verify_relisted}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
        sys.exit(0)
    args = sys.argv[1:]
    combos = [(0, 0), (1, 0), (1, 1)]
    if args and args[0] == "--nostats":
        args, combos = args[1:], [(0, 0), (1, 0)]
    sizes = [int(a) for a in args] or [2_000_000, 20_000_000, 100_000_000]
    for n in sizes:
        for fuse, stats in combos:
            t0 = time.time()
            r = subprocess.run([sys.executable, "-u", __file__, "--child", str(n), str(fuse), str(stats)],
                               capture_output=True, text=True, timeout=300)
            out = (r.stdout + r.stderr).strip().splitlines()
            keep = [x for x in out if "fused:" in x or "frames=" in x or "Error" in x or "error" in x]
            print("\n".join(keep[-3:]) or "\n".join(out[-5:]), f"({time.time() - t0:.0f} s, rc {r.returncode})",
                  flush=True)
            if r.returncode != 0:
                sys.exit(r.returncode)
