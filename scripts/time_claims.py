"""Decode C2 frames on the device a few times (for rocprofv3 kernel stats of ablated builds:
their outputs are invalid by design). Usage: python scripts/time_claims.py [frames | c5 | dense]
(dense: 0.4 GB of the two-framing cascade stream, tests/_streams.shadow_stream_np)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ctypes as C  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
import drp_amd  # noqa: E402

arg = sys.argv[1] if len(sys.argv) > 1 else "20000000"
dev = torch.device("cuda", 0)
if arg == "c5":  # the C5 round trip's wire (1M Changes, 4 KB values), encoded once
    n = 1_000_000
    cols, heap, frame = bench.c5_on_device(n, seed=55, dev=dev)
    W = int(frame.sum())
    out = torch.empty(W + 64, dtype=torch.uint8, device=dev)
    foff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    with drp_amd.Ctx(0) as ectx:
        ectx.encode_device(cols, heap, n, foff, out, W + 64)
    torch.cuda.synchronize()
    wire = out[:W]
elif arg == "dense":
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _streams as S  # noqa: E402
    n = int(0.4e9) // 200
    wire = torch.from_numpy(S.shadow_stream_np(n, period=200, shadow_at=20, small=4)).to(dev)
else:
    n = int(arg)
    wire = bench.c2_on_device(n, seed=1234, dev=dev)
so = torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev)
outs = bench.alloc_outputs(n + 64, dev)
res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
with drp_amd.Ctx(0) as ctx:
    for _ in range(4):
        ctx.decode_device(wire, so, None, outs, n + 64, res)
    torch.cuda.synchronize()
print("done")
