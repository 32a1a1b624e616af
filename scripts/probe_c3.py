"""Probe: the C3 stream (1000 C2 frames + a 1 MiB blob per unit) decoded whole on the device, per
claims form (DRP_CLAIMS auto / fast / hop), with the decode's repair counters and the kernel time;
then the host-batch path (drp_decode_batch) in each blob-skip mode. Usage: python scripts/probe_c3.py"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from _gpu import drp_amd  # noqa: E402

dev = torch.device("cuda", 0)
units = int(os.environ.get("C3_UNITS", "300"))
host = bench.c3_host(units)
nf = units * 1001
wire = torch.from_numpy(host).to(dev)
so = torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev)
outs = bench.alloc_outputs(nf + 64, dev)
res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
print(f"C3 {units} units, {wire.numel() / 1e9:.2f} GB, {nf} frames", flush=True)
for mode in ["auto", "fast", "hop"]:
    os.environ["DRP_CLAIMS"] = mode if mode != "auto" else ""
    with drp_amd.Ctx(0) as ctx:  # (knobs are read by drp_open)
        for rep in range(3):
            t0 = time.perf_counter()
            ctx.decode_device(wire, so, None, outs, nf + 64, res)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            t = ctx.timing()
            r = drp_amd.StreamResult.from_buffer_copy(res.cpu().numpy().tobytes()[:C.sizeof(drp_amd.StreamResult)])
            print(f"  device {mode:4s} rep {rep}: {dt * 1e3:8.2f} ms wall, decode {t.decode_ms:8.2f} ms, total "
                  f"{t.total_ms:8.2f} ms, repairs {t.spec_repairs}, seg {t.seg_repairs}, relisted {t.verify_relisted}, "
                  f"exact {t.strict_reruns}, frames {r.frames} err {r.err_code}", flush=True)
os.environ["DRP_CLAIMS"] = ""
del wire, outs
pinned = torch.empty(host.size, dtype=torch.uint8, pin_memory=True)
pinned.numpy()[:] = host
houts = drp_amd.alloc_host_outputs(nf + 64)
for name, m in [("off", drp_amd.BLOB_SKIP_OFF), ("auto", drp_amd.BLOB_SKIP_AUTO), ("always", drp_amd.BLOB_SKIP_ALWAYS)]:
    with drp_amd.Ctx(0) as ctx:
        ctx.set_blob_skip(m)
        for rep in range(3):
            t0 = time.perf_counter()
            g = ctx.decode_batch(pinned.numpy(), outs=houts)
            dt = time.perf_counter() - t0
            t = ctx.timing()
            print(f"  host {name:6s} rep {rep}: {dt * 1e3:8.2f} ms wall, decode {t.decode_ms:8.2f} total {t.total_ms:8.2f} "
                  f"h2d {t.h2d_ms:7.2f} ms ({t.h2d_bytes / 1e6:.0f} MB staged, {t.h2d_skipped / 1e6:.0f} skipped), "
                  f"repairs {t.spec_repairs}, seg {t.seg_repairs}, relisted {t.verify_relisted}, frames {g['nframes']}",
                  flush=True)
