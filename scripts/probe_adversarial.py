"""GPU probe: decode time and repair behaviour on the prediction-defeating shadow streams
(tests/_streams.shadow_stream). Usage: python scripts/probe_adversarial.py [MB ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import _gpu  # noqa: E402,F401  (torch first, then libdrp)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _streams as S  # noqa: E402
import drp_amd  # noqa: E402
import bench  # noqa: E402


def run(ctx, wire, exact=False):
    dev = torch.device("cuda", 0)
    w = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).to(dev)
    so = torch.tensor([0, w.numel()], dtype=torch.int64, device=dev)
    cap = w.numel() // 2 + 64
    outs = bench.alloc_outputs(cap, dev)
    res = torch.zeros(C_SIZE, dtype=torch.uint8, device=dev)
    ctx.set_exact(exact)
    best = None
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.decode_device(w, so, None, outs, cap, res)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
    t = ctx.timing()
    ctx.set_exact(False)
    return best * 1e3, t


import ctypes as C  # noqa: E402
C_SIZE = C.sizeof(drp_amd.StreamResult)
sizes = [float(a) for a in sys.argv[1:]] or [16, 128]
with drp_amd.Ctx(0) as ctx:
    for mb in sizes:
        for period, at, small in [(8192, 100, 10), (8229, 100, 10), (4100, 300, 12), (20000, 100, 10)]:
            n = int(mb * 2**20 / period)
            wire = S.shadow_stream(n, period=period, shadow_at=at, small=small)
            ms, t = run(ctx, wire)
            print(f"{mb:6.0f} MB period {period:5d}: spec path {ms:8.2f} ms  repairs {t.spec_repairs} "
                  f"exact_rerun {t.strict_reruns} relisted {t.verify_relisted}", flush=True)
            if mb <= 16:
                ms2, _ = run(ctx, wire, exact=True)
                print(f"{'':6s}    exact kernel alone {ms2:8.2f} ms", flush=True)
