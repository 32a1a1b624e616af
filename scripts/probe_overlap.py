"""Measurement only: do the C2 claims kernel (instruction-bound) and the lean emit (HBM-bound) share
the GPU when run side by side? Decodes a C2 stream, then drp_probe_overlap times claims alone, emit
alone and both at once on two streams (over the same 100M frames)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dat-replication-protocol_amd", "python"))
import torch  # noqa: E402

import bench  # noqa: E402
import drp_amd  # noqa: E402

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
wire = bench.c2_on_device(n, seed=5, dev=dev)
so = torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev)
outs = bench.alloc_outputs(n + 64, dev)
res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
ctx = drp_amd.Ctx(0)
for _ in range(3):
    ctx.decode_device(wire, so, None, outs, n + 64, res)
torch.cuda.synchronize()
bench.verify_c2(outs, res, n, dev)
L = drp_amd.lib()
L.drp_probe_overlap.argtypes = [C.c_void_p, C.POINTER(C.c_float)]
for rep in range(4):
    ms = (C.c_float * 6)()
    assert L.drp_probe_overlap(ctx.h, ms) == 0
    print(f"claims alone {ms[0]:.3f} ms, emit alone {ms[1]:.3f} ms, sum {ms[0] + ms[1]:.3f} ms, "
          f"side by side {ms[2]:.3f} ms, one launch (emit lag 0 / 64 / 1024 tiles) "
          f"{ms[3]:.3f} / {ms[4]:.3f} / {ms[5]:.3f} ms", flush=True)
ctx.close()
