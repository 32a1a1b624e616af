#!/usr/bin/env python3
"""Benchmark: decoded Change frames/s + wire GB/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): per GPU one 8.6 GB replication
stream of 100,000,000 Change frames of exactly 86 B (10-digit key, change=(i%100)+1,
from=i%128, to=(i+1)%128, 64 random value bytes), synthesised on the device (seeded) and
resident in HBM before timing. One step = one full decode of that stream by libdrp
(frame split + Change decode into SoA columns, decode.js:144-262 + messages/index.js:5)
plus, for N > 1, the RCCL all-gather of per-stream stats and the global index scan.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Prints ONE JSON line (rank 0). `roofline` prices the decode kernel from HIP events on
the libdrp stream; `cpu_baseline` times the C restatement of the reference (oracle/) on
a bounded sample on this host's cores.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dat-replication-protocol_amd", "python"))
import drp_amd  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FRAME = 86


def c2_on_device(nframes, seed, dev):
    """C2 stream generated on the GPU (same layout as tests/_streams.c2_stream)."""
    a = torch.empty((nframes, FRAME), dtype=torch.uint8, device=dev)
    i = torch.arange(nframes, device=dev, dtype=torch.int64)
    a[:, 0] = 85
    a[:, 1] = 1
    a[:, 2] = 0x12
    a[:, 3] = 10
    for k in range(10):
        a[:, 4 + k] = (48 + torch.div(i, 10 ** (9 - k), rounding_mode="floor") % 10).to(torch.uint8)
    a[:, 14] = 0x18
    a[:, 15] = ((i % 100) + 1).to(torch.uint8)
    a[:, 16] = 0x20
    a[:, 17] = (i % 128).to(torch.uint8)
    a[:, 18] = 0x28
    a[:, 19] = ((i + 1) % 128).to(torch.uint8)
    a[:, 20] = 0x32
    a[:, 21] = 64
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    a[:, 22:] = torch.randint(0, 256, (nframes, 64), generator=g, device=dev, dtype=torch.uint8)
    del i
    return a.reshape(-1)


def alloc_outputs(cap, dev):
    o = {"payload_off": torch.empty(cap, dtype=torch.int64, device=dev),
         "payload_len": torch.empty(cap, dtype=torch.int32, device=dev),
         "type": torch.empty(cap, dtype=torch.uint8, device=dev),
         "flags": torch.empty(cap, dtype=torch.uint8, device=dev)}
    for k in drp_amd.COLS32:
        o[k] = torch.empty(cap, dtype=torch.int32, device=dev)
    for k in drp_amd.COLS64:
        o[k] = torch.empty(cap, dtype=torch.int64, device=dev)
    return o


def verify_c2(o, res, nframes, dev):
    """Size-independent properties of the full-size decode (bit-exact vs the generator)."""
    r = drp_amd.StreamResult.from_buffer_copy(res.cpu().numpy().tobytes()[:C.sizeof(drp_amd.StreamResult)])
    o = {k: v[:nframes] for k, v in o.items()}  # columns are allocated with slack past nframes
    assert (r.frames, r.changes, r.blobs, r.err_code, r.tail_kind, r.consumed) == \
        (nframes, nframes, 0, 0, 0, nframes * FRAME), (r.frames, r.err_code, r.tail_kind, r.consumed)
    i = torch.arange(nframes, device=dev, dtype=torch.int64)
    checks = {
        "payload_off": torch.equal(o["payload_off"], i * FRAME + 2),
        "payload_len": bool((o["payload_len"] == 84).all()), "type": bool((o["type"] == 1).all()),
        "key_off": bool((o["key_off"] == 2).all()), "key_len": bool((o["key_len"] == 10).all()),
        "value_off": bool((o["value_off"] == 20).all()), "value_len": bool((o["value_len"] == 64).all()),
        "subset_len": bool((o["subset_len"] == 0).all()), "flags": bool((o["flags"] == 2).all()),
        "change": torch.equal(o["change"], (i % 100) + 1), "from": torch.equal(o["from"], i % 128),
        "to": torch.equal(o["to"], (i + 1) % 128),
    }
    bad = [k for k, v in checks.items() if not v]
    assert not bad, f"decoded columns differ from the generator: {bad}"


def cpu_baseline(min_seconds=10.0, sample_frames=2_000_000):
    """The C restatement of decode.js (oracle/, 1 thread) over a C2 sample in 64 KiB writes."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    import _streams as S
    wire = S.c2_stream(sample_frames, seed=7).tobytes()
    outs = O.alloc_outputs(sample_frames + 16)
    O.decode_batch(wire, chunk=65536, outs=outs)
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < min_seconds:
        r = O.decode_batch(wire, chunk=65536, outs=outs)
        assert r["nframes"] == sample_frames
        reps += 1
    dt = time.perf_counter() - t0
    return {"value": reps * sample_frames / dt, "unit": "frames/s", "cores": 1, "kind": "port",
            "wire_GBps": reps * len(wire) / dt / 1e9,
            "sample": f"C2 sample of {sample_frames} frames ({len(wire)} B) decoded {reps}x in 64 KiB "
                      f"writes by oracle/drp_oracle.c (decode.js + protocol-buffers@2 restatement), "
                      f"{dt:.1f} s on 1 host core"}


def h2d_rate(dev, nbytes=1 << 30):
    """Pinned host -> HBM copy rate for one batch (reported separately, never `value`)."""
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(3):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / 3
    del h, d
    return {"GBps": nbytes / dt / 1e9, "bytes": nbytes, "note": "pinned host -> HBM, 1 GiB batch"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames", type=int, default=100_000_000)
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    nframes = args.frames
    wire = c2_on_device(nframes, seed=1234 + rank, dev=dev)
    stream_off = torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev)
    outs = alloc_outputs(nframes + 64, dev)
    res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    stats = torch.zeros(4, dtype=torch.int64, device=dev)
    gathered = torch.zeros(world * 4, dtype=torch.int64, device=dev)
    gbase = torch.zeros(world, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)

    ctx = drp_amd.Ctx(local, tile=args.tile)
    L = ctx.L
    sp = lambda t: C.c_void_p(t.data_ptr())

    def step():
        ctx.decode_device(wire, stream_off, None, outs, nframes + 64, res)
        if dist:
            drp_amd._chk("stats", L.drp_stream_stats_from_results(ctx.h, sp(res), sp(stream_off), 1, sp(stats)))
            drp_amd._chk("sync", L.drp_synchronize(ctx.h))
            torch.distributed.all_gather_into_tensor(gathered, stats)  # RCCL over xGMI
            torch.cuda.synchronize(dev)
            drp_amd._chk("index", L.drp_index_scan(ctx.h, sp(gathered), world, sp(gbase)))
            drp_amd._chk("sync", L.drp_synchronize(ctx.h))

    for _ in range(args.warmup):
        step()
    verify_c2(outs, res, nframes, dev)

    ext = torch.cuda.ExternalStream(ctx.stream, device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    dec_ms = []
    t0 = time.perf_counter()
    ev0.record(ext)
    for _ in range(args.steps):
        step()
        t = ctx.timing()
        dec_ms.append(t.decode_ms)
    ev1.record(ext)
    torch.cuda.synchronize(dev)
    if dist:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(tt.item())

    frames_total = nframes * world * args.steps
    wire_total = nframes * FRAME * world * args.steps
    ms_per_step = elapsed / args.steps * 1e3
    dec_avg_s = float(np.mean(dec_ms)) / 1e3
    b_dec = nframes * FRAME + 13 * nframes + 49 * nframes  # W + 13F + 49C
    achieved = b_dec / dec_avg_s / 1e9

    if rank == 0:
        out = {
            "metric": "decoded Change frames/sec + wire GB/s (whole node) at 1/2/4/8 MI355X",
            "value": frames_total / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: C2 generator on device (seeded), resident in HBM before timing",
            "config": {"workload": "C2: 100M Change frames x 86 B (64 B values), one 8.6 GB stream per GPU",
                       "frames_per_gpu": nframes, "wire_bytes_per_gpu": nframes * FRAME,
                       "parallelism": f"independent streams, {world} GPU(s); RCCL all-gather of stream stats",
                       "tile_bytes": args.tile or 8192},
            "wire_GBps": wire_total / elapsed / 1e9,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                         "kernel": f"decode_tiles<{(args.tile or 8192) // 64}>", "kernel_ms": dec_avg_s * 1e3,
                         "bytes_per_launch": b_dec,
                         "bytes_model": "W + 13*frames + 49*changes (86+13+49 = 148 B/frame)"},
            "step_ms_hip_events": ev_ms / args.steps,
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline()
            out["h2d"] = h2d_rate(dev)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
