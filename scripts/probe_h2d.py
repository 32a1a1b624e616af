"""Probe: H2D rate of a 1 GiB page-locked buffer into HBM, as one copy, in 128 MiB chunks on one
stream, and in chunks spread over 2 or 4 streams (do several DMA engines beat one?)."""
import time

import torch

dev = torch.device("cuda", 0)
N = 1 << 30
CH = 128 << 20
h = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h.numpy()[:] = 7
d = torch.empty(N, dtype=torch.uint8, device=dev)
streams = [torch.cuda.Stream(dev) for _ in range(4)]


def run(ns, chunk):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k, o in enumerate(range(0, N, chunk)):
        s = streams[k % ns]
        with torch.cuda.stream(s):
            d[o:o + chunk].copy_(h[o:o + chunk], non_blocking=True)
    torch.cuda.synchronize()
    return N / (time.perf_counter() - t0) / 1e9


for ns, chunk in [(1, N), (1, CH), (2, CH), (4, CH), (2, 32 << 20), (4, 32 << 20)]:
    r = [run(ns, chunk) for _ in range(5)]
    print(f"{ns} stream(s), {chunk >> 20} MiB chunks: {max(r):.1f} GB/s best, {sum(r) / len(r):.1f} mean")
