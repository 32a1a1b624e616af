"""Probe: how the claims kernels' predictions fail on the C3 shape (1000 C2 frames + a 1 MiB blob
per unit, decoded whole). Dumps the head's claims (DRP_DUMP_CLAIMS) and classifies every tile
against the oracle's frame starts: blob-interior tiles that claimed a chain, tiles whose claim is
not the exact chain's exit. Usage: python scripts/probe_c3_claims.py [units]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = os.path.join(ROOT, "gpurun_out", "c3_claims.bin")
os.environ["DRP_DUMP_CLAIMS"] = DUMP
os.environ["DRP_STATS"] = "1"
import torch  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import _oracle as O  # noqa: E402
import bench  # noqa: E402
from _gpu import drp_amd  # noqa: E402

units = int(sys.argv[1]) if len(sys.argv) > 1 else int(os.environ.get("C3_UNITS", "300"))
host = bench.c3_host(units)
wire = host.tobytes()
nf = units * 1001
if os.path.exists(DUMP):
    os.unlink(DUMP)
dev = torch.device("cuda", 0)
for mode in ["fast", "hop"]:
    os.environ["DRP_CLAIMS"] = mode
    w = torch.from_numpy(host).to(dev)
    so = torch.tensor([0, w.numel()], dtype=torch.int64, device=dev)
    outs = bench.alloc_outputs(nf + 64, dev)
    res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    with drp_amd.Ctx(0) as ctx:
        ctx.decode_device(w, so, None, outs, nf + 64, res)
        torch.cuda.synchronize()
        t = ctx.timing()
    print(f"{mode}: repairs {t.spec_repairs} seg {t.seg_repairs} relisted {t.verify_relisted}", flush=True)
    raw = open(DUMP, "rb").read()
    os.unlink(DUMP)
    ntl = int(np.frombuffer(raw[:8], np.uint64)[0])
    claims = np.frombuffer(raw[8:8 + 8 * ntl], np.uint64)
    r = O.decode_batch(wire)
    starts = (r["payload_off"].astype(np.int64) - 1)  # (id byte; the header start is before it)
    # frame header starts: payload_off - 1 - varint bytes
    hs = []
    for i in range(r["nframes"]):
        po, pl = int(r["payload_off"][i]), int(r["payload_len"][i])
        k = 1 if pl + 1 < 128 else 2 if pl + 1 < 16384 else 3
        hs.append(po - 1 - k)
    hs = np.array(hs, np.int64)
    T = 8192
    C_ID = 1 << 62
    stats = {"blob_interior": 0, "blob_interior_claimed": 0, "with_frames": 0, "wrong_claim": 0}
    examples = []
    for tt in range(ntl):
        a, b = tt * T, (tt + 1) * T
        inside = np.searchsorted(hs, a, "left") < np.searchsorted(hs, b, "left")
        j = np.searchsorted(hs, b, "left")
        exit_true = int(hs[j]) if j < len(hs) else None
        cl = int(claims[tt])
        if not inside:
            stats["blob_interior"] += 1
            if cl != C_ID:
                stats["blob_interior_claimed"] += 1
                if len(examples) < 8:
                    examples.append((tt, hex(cl), exit_true))
        else:
            stats["with_frames"] += 1
            if cl != exit_true and not (cl & (1 << 61)):
                stats["wrong_claim"] += 1
    print(f"  {ntl} tiles: {stats}; examples (tile, claim, true exit) {examples}", flush=True)
