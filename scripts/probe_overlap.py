"""Probe: do two C2 decodes in flight (two contexts, two HIP streams, one host thread each) finish
sooner than the same decodes one after another? claims_fast is VALU-bound and emit_recs HBM-bound,
so a claims pass of one batch could run beside the emission of another. Prints ms per decode for
the serial and the two-in-flight runs (and checks each run's frame count)."""
import ctypes as C
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from bench import drp_amd  # noqa: E402

N = int(os.environ.get("FRAMES", "100000000"))
K = int(os.environ.get("STEPS", "10"))
dev = torch.device("cuda", 0)
wire = bench.c2_on_device(N, seed=1234, dev=dev)
so = torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev)
cap = N + 64
ctxs, outs, ress = [], [], []
for _ in range(2):
    ctxs.append(drp_amd.Ctx(0))
    outs.append(bench.alloc_outputs(cap, dev))
    ress.append(torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev))
torch.cuda.synchronize()


def run(i, k):
    for _ in range(k):
        ctxs[i].decode_device(wire, so, None, outs[i], cap, ress[i])


def frames(i):
    return drp_amd.StreamResult.from_buffer_copy(ress[i].cpu().numpy().tobytes()).frames


for i in range(2):
    run(i, 2)
    assert frames(i) == N
torch.cuda.synchronize()
t0 = time.perf_counter()
run(0, 2 * K)
torch.cuda.synchronize()
serial = (time.perf_counter() - t0) / (2 * K) * 1e3
th = [threading.Thread(target=run, args=(i, K)) for i in range(2)]
t0 = time.perf_counter()
for t in th:
    t.start()
for t in th:
    t.join()
torch.cuda.synchronize()
dual = (time.perf_counter() - t0) / (2 * K) * 1e3
assert frames(0) == N and frames(1) == N
print(f"serial {serial:.3f} ms/decode, two in flight {dual:.3f} ms/decode ({serial / dual:.2f}x)")
