"""Probe: claims_fast's link rounds (total, maximum, tiles over 8) and tiles with deferred restarts
on a clean C2 decode, the dense two-framing cascade and a C5 decode (DRP_STATS counters, printed by libdrp on
stderr). Usage: python scripts/probe_stats.py"""
import ctypes as C
import os
import sys

os.environ["DRP_STATS"] = "1"
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import _streams as S  # noqa: E402
import bench  # noqa: E402
from _gpu import drp_amd  # noqa: E402

dev = torch.device("cuda", 0)
with drp_amd.Ctx(0) as ctx:
    n = 4_000_000
    wire = bench.c2_on_device(n, seed=3, dev=dev)
    outs = bench.alloc_outputs(n + 64, dev)
    res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    print(f"C2 {n} frames ({(wire.numel() + 8191) // 8192} tiles):", flush=True)
    ctx.decode_device(wire, torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev), None, outs, n + 64, res)
    torch.cuda.synchronize()
    del wire, outs
    period = 200
    n = int(0.2e9) // period
    w = torch.from_numpy(S.shadow_stream_np(n, period=period, shadow_at=20, small=4)).to(dev)
    outs = bench.alloc_outputs(n + 64, dev)
    print(f"dense cascade 0.2 GB ({(w.numel() + 8191) // 8192} tiles):", flush=True)
    ctx.decode_device(w, torch.tensor([0, w.numel()], dtype=torch.int64, device=dev), None, outs, n + 64, res)
    torch.cuda.synchronize()
    del w, outs
with drp_amd.Ctx(0) as ctx:  # (a ctx of its own: the long-frame check from the first decode on)
    n = 200_000
    cols, heap, frame = bench.c5_on_device(n, seed=55, dev=dev)
    W = int(frame.sum())
    out = torch.zeros(W + 64, dtype=torch.uint8, device=dev)
    foff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.encode_device(cols, heap, n, foff, out, W + 64)
    outs = bench.alloc_outputs(n + 64, dev)
    print(f"C5 {n} Changes ({(W + 8191) // 8192} tiles):", flush=True)
    ctx.decode_device(out[:W], torch.tensor([0, W], dtype=torch.int64, device=dev), None, outs, n + 64, res)
    torch.cuda.synchronize()
