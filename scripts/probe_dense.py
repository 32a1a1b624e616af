"""Probe: decode times of dense two-framing (shadow) streams on the default path, with the
path taken (repair passes, segmented repairs, exact re-runs). Usage: python scripts/probe_dense.py [k]
(k: only the k-th case, e.g. under rocprofv3)"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import _streams as S  # noqa: E402
import bench  # noqa: E402
from _gpu import drp_amd  # noqa: E402

dev = torch.device("cuda", 0)
ctx = drp_amd.Ctx(0)
CASES = [(200, 20, 4, 0.2), (200, 20, 4, 1.7), (1000, 40, 10, 1.7), (3000, 70, 4, 1.7), (6000, 200, 40, 0.5)]
for period, at, small, gb in ([CASES[int(sys.argv[1])]] if len(sys.argv) > 1 else CASES):
    n = int(gb * 1e9) // period
    w = torch.from_numpy(S.shadow_stream_np(n, period=period, shadow_at=at, small=small)).to(dev)
    so = torch.tensor([0, w.numel()], dtype=torch.int64, device=dev)
    outs = bench.alloc_outputs(n + 64, dev)
    res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    ts = []
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.decode_device(w, so, None, outs, n + 64, res)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = ctx.timing()
    ok = torch.equal(outs["payload_off"][:n], torch.arange(n, device=dev, dtype=torch.int64) * period +
                     len(S.varint(period - 2)) + 1)
    print(f"period {period} shadow {at}/{small} {gb} GB: {min(ts) * 1e3:.1f} ms ok={ok} repairs {t.spec_repairs} "
          f"seg {t.seg_repairs} exact {t.strict_reruns} decode_ms {t.decode_ms:.1f}", flush=True)
    del w, outs
    torch.cuda.empty_cache()
