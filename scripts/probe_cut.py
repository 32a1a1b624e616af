"""Probe: misses on C2 frames cut into streams at arbitrary bytes (tests/test_gpu_decode.py
test_cut_streams_edge_tiles' input): DRP_STATS prints the first missed tiles (tile, entry, claim,
exact exit); this script prints where each lies in its stream. Usage: python scripts/probe_cut.py"""
import ctypes as C
import os
import random
import sys

os.environ["DRP_STATS"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import _streams as S  # noqa: E402
import bench  # noqa: E402
from _gpu import drp_amd  # noqa: E402

dev = torch.device("cuda", 0)
rng = random.Random(404)
wire = S.c2_stream(60_000, seed=6).tobytes()
fb = 86
cuts = sorted(set([0] + [c for c in rng.sample(range(1, len(wire)), 149) if c % fb] + [len(wire)]))
entry = [(-a) % fb for a in cuts[:-1]]
ns = len(cuts) - 1
tp = [0]
for a, b in zip(cuts[:-1], cuts[1:]):
    tp.append(tp[-1] + (b + 8191) // 8192 - a // 8192)
print("stream tile ranges (first 12):", [(cuts[s], cuts[s + 1], tp[s], tp[s + 1]) for s in range(12)], flush=True)
cap = 60_000 + 64
outs = bench.alloc_outputs(cap, dev)
res = torch.zeros(ns * C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
w = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).to(dev)
with drp_amd.Ctx(0) as ctx:
    ctx.decode_device(w, torch.tensor(cuts, dtype=torch.int64, device=dev),
                      torch.tensor(entry, dtype=torch.int64, device=dev), outs, cap, res)
    torch.cuda.synchronize()
    t = ctx.timing()
    print(f"repairs {t.spec_repairs} relisted {t.verify_relisted}", flush=True)
