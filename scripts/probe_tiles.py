"""Probe: per-tile decode cost without look-back. Builds N independent streams of exactly
one 4 KiB tile each (47 C2 frames + a 54-byte partial frame), decodes them in one call and
prints the kernel time. Usage: python scripts/probe_tiles.py [nstreams] [tile_bytes]"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dat-replication-protocol_amd", "python"))
import bench  # noqa: E402
import drp_amd  # noqa: E402

ns = int(sys.argv[1]) if len(sys.argv) > 1 else 400000
tile = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
dev = torch.device("cuda", 0)
per = tile // 86
frames = bench.c2_on_device(ns * (per + 1), seed=3, dev=dev).view(ns, per + 1, 86)
wire = torch.empty((ns, tile), dtype=torch.uint8, device=dev)
wire[:, : per * 86] = frames[:, :per].reshape(ns, -1)
wire[:, per * 86:] = frames[:, per, : tile - per * 86]
wire = wire.reshape(-1)
del frames
stream_off = torch.arange(ns + 1, device=dev, dtype=torch.int64) * tile
outs = bench.alloc_outputs(ns * per + 64, dev)
res = torch.zeros(ns * C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
ctx = drp_amd.Ctx(0, tile=tile)
for it in range(3):
    ctx.decode_device(wire, stream_off, None, outs, ns * per + 64, res)
    t = ctx.timing()
    print(f"streams={ns} tile={tile} decode_ms={t.decode_ms:.3f} "
          f"frames/s={ns * per / t.decode_ms * 1e3 / 1e9:.3f}G "
          f"wire_GBps={ns * tile / t.decode_ms / 1e6:.1f}", flush=True)
r = drp_amd.StreamResult.from_buffer_copy(res[: C.sizeof(drp_amd.StreamResult)].cpu().numpy().tobytes())
print("stream0:", r.frames, r.tail_kind, r.err_code)
assert r.frames == per and r.tail_kind == 2
ctx.close()
