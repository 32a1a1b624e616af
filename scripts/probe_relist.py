"""Probe: tiles the records-only verification relists (drp_timing.verify_relisted) against the
number of streams the same C2 frames are cut into (C4 relists ~8000 more tiles than C2 for the
same frames), and where in its stream each relisted tile lies (drp_probe_relist re-runs the last
decode's claims + verification and copies the list out). Usage: python scripts/probe_relist.py"""
import collections
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import drp_amd  # noqa: E402

TILE = 8192
dev = torch.device("cuda", 0)
n = 4_000_000
wire = bench.c2_on_device(n, seed=1234, dev=dev)
fb = 86  # C2 frame bytes
outs = bench.alloc_outputs(n + 64, dev)
res = torch.zeros(8192 * C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
L = drp_amd.lib()
L.drp_probe_relist.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32)]
L.drp_probe_tile.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)]
with drp_amd.Ctx(0) as ctx:
    for s in (1, 64, 512, 4096):
        per = n // s
        cuts = [i * per * fb for i in range(s)] + [wire.numel()]
        so = torch.tensor(cuts, dtype=torch.int64, device=dev)
        for _ in range(2):
            ctx.decode_device(wire, so, None, outs, n + 64, res)
        torch.cuda.synchronize()
        t = ctx.timing()
        print(f"streams {s:5d}: relisted {t.verify_relisted}, repairs {t.spec_repairs}, "
              f"decode {t.decode_ms:.3f} ms", flush=True)
        # tile -> (stream, index in stream, tiles in stream): tiles are the absolute 8 KiB blocks
        # a stream touches
        first, count = [], []
        for k in range(s):
            a, b = cuts[k], cuts[k + 1]
            first.append(sum(count))
            count.append((b + TILE - 1) // TILE - a // TILE)
        cap = 1 << 20
        buf = (C.c_uint32 * cap)()
        cnt = C.c_uint32(0)
        assert L.drp_probe_relist(ctx.h, buf, cap, C.byref(cnt)) == 0
        where = collections.Counter()
        for i in range(min(cnt.value, cap)):
            tt = buf[i]
            lo, hi = 0, s
            while hi - lo > 1:
                mid = (lo + hi) // 2
                if first[mid] <= tt:
                    lo = mid
                else:
                    hi = mid
            j = tt - first[lo]
            where["first" if j == 0 else ("last" if j == count[lo] - 1 else
                                         ("second" if j == 1 else ("second last" if j == count[lo] - 2
                                                                    else "interior")))] += 1
        print(f"  relisted tiles by place in their stream: {dict(where)}", flush=True)
        if s == 64:  # one relisted last tile in detail
            for i in range(min(cnt.value, cap)):
                tt = buf[i]
                k = next((q for q in range(s) if first[q] <= tt < first[q] + count[q]), None)
                if k is not None and tt == first[k] + count[k] - 1:
                    rec = (C.c_uint8 * 384)()
                    cl = (C.c_uint64 * 2)()
                    assert L.drp_probe_tile(ctx.h, tt, rec, cl) == 0
                    A = (cuts[k + 1] - 1) // TILE * TILE
                    print(f"  tile {tt} (stream {k}, A={A}, stream end {cuts[k + 1]} = A + {cuts[k + 1] - A}): "
                          f"claim of the tile before {cl[0]:#x} (A + {cl[0] - A}), claim {cl[1]:#x}", flush=True)
                    print("  records (thread: entry byte / frames / changes):",
                          " ".join(f"{th}:{rec[th]:02x}/{rec[128 + th]}/{rec[256 + th]}" for th in range(128)
                                   if rec[th] != 0xFF), flush=True)
                    break
