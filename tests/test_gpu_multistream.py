"""GPU parity for the segmented multi-stream decode (BASELINE configs[3] shape, small): many
independent streams in one drp_decode_device call, per-stream results and columns vs the
oracle on each stream, and the stats + index-scan path the multi-GPU all-gather feeds."""
import ctypes as C
import os
import random
import sys

import numpy as np
import pytest

import _oracle as O
import _streams as S

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dat-replication-protocol_amd", "python"))


def _streams(rng, n):
    out = []
    for s in range(n):
        k = s % 6
        if k == 0:
            w = S.c2_stream(rng.randint(0, 400), seed=s, start=s * 1000).tobytes()
        elif k == 1:
            w = S.c5_stream(rng, rng.randint(0, 6))
        elif k == 2:  # truncated anywhere (tail header / change / blob)
            w = S.random_stream(rng, rng.randint(1, 60), blob_p=0.2, blob_max=9000)
            w = w[:rng.randint(0, len(w))]
        elif k == 3:  # protocol error in the middle
            a = S.random_stream(rng, rng.randint(0, 20))
            w = a + b"\x03\x07ab" + S.random_stream(rng, 5)
        else:
            w = S.random_stream(rng, rng.randint(0, 80), blob_p=0.05, blob_max=20000)
        out.append(w)
    return out


@pytest.mark.parametrize("kernel", ["speculative", "exact4096", "exact8192"])
def test_many_streams(kernel):
    """300 streams in one call, on the default path and on the exact kernel at both tile sizes
    (the exact kernel's cross-tile look-back over many short streams: the wait cycle fixed in
    round 1 commit 3651cbd)."""
    import torch

    import drp_amd
    import drp_dist

    tile = 8192 if kernel == "speculative" else int(kernel[5:])
    rng = random.Random(7 + tile)
    streams = _streams(rng, 300)
    # a blob continuation at the front of some streams: decode from `entry`
    entry = [0] * len(streams)
    for s in range(4, len(streams), 7):
        pre = rng.randbytes(rng.randint(1, 5000))
        streams[s] = pre + streams[s]
        entry[s] = len(pre)
    offs = np.concatenate([[0], np.cumsum([len(w) for w in streams])]).astype(np.int64)
    wire = np.frombuffer(b"".join(streams), np.uint8)
    dev = torch.device("cuda", 0)
    wire_t = torch.from_numpy(wire.copy()).to(dev) if wire.size else torch.zeros(16, dtype=torch.uint8, device=dev)
    so_t = torch.from_numpy(offs).to(dev)
    en_t = torch.tensor(entry, dtype=torch.int64, device=dev)
    cap = int(wire.size) // 2 + 64
    outs = {"payload_off": torch.zeros(cap, dtype=torch.int64, device=dev),
            "payload_len": torch.zeros(cap, dtype=torch.int32, device=dev),
            "type": torch.zeros(cap, dtype=torch.uint8, device=dev),
            "flags": torch.zeros(cap, dtype=torch.uint8, device=dev)}
    for k in drp_amd.COLS32:
        outs[k] = torch.zeros(cap, dtype=torch.int32, device=dev)
    for k in drp_amd.COLS64:
        outs[k] = torch.zeros(cap, dtype=torch.int64, device=dev)
    rs = C.sizeof(drp_amd.StreamResult)
    res_t = torch.zeros(len(streams) * rs, dtype=torch.uint8, device=dev)
    with drp_amd.Ctx(0, tile=tile) as ctx:
        if kernel != "speculative":
            ctx.set_exact(True)
        ctx.decode_device(wire_t, so_t, en_t, outs, cap, res_t)
        stats = drp_dist.local_stats_device(ctx, res_t, so_t)
        base = drp_dist.global_index_device(ctx, stats)
    host = {k: v.cpu().numpy() for k, v in outs.items()}
    raw = res_t.cpu().numpy().tobytes()
    base = base.cpu().numpy()
    stats = stats.cpu().numpy()
    for s, w in enumerate(streams):
        r = drp_amd.StreamResult.from_buffer_copy(raw[s * rs:(s + 1) * rs])
        e = entry[s]
        ref = O.decode_batch(w[e:])
        label = f"stream {s} ({len(w)} B, entry {e})"
        assert r.frames == ref["nframes"], label
        assert r.err_code == ref["err_code"], label
        if ref["err_code"]:
            assert r.err_frame == ref["err_frame"], label
        else:
            assert r.tail_kind == ref["tail"], label
            assert r.consumed == ref["consumed"] + e, label
            assert r.blob_remaining == ref["blob_remaining"], label
        fb, n = r.frame_begin, r.frames
        assert base[s] == fb, label
        assert list(stats[s][:3]) == [r.frames, r.changes, r.blobs], label
        got_off = host["payload_off"][fb:fb + n].astype(np.int64) - offs[s] - e
        np.testing.assert_array_equal(got_off, ref["payload_off"][:n].astype(np.int64), err_msg=label)
        np.testing.assert_array_equal(host["payload_len"][fb:fb + n].astype(np.uint32),
                                      ref["payload_len"][:n], err_msg=label)
        np.testing.assert_array_equal(host["type"][fb:fb + n], ref["type"][:n], err_msg=label)
        ch = (ref["type"][:n] & 0x3F) == 1
        for k in O.COLS32 + O.COLS64 + ["flags"]:
            got = host[k][fb:fb + n].astype(ref[k].dtype)
            np.testing.assert_array_equal(got[ch], ref[k][:n][ch], err_msg=f"{label}:{k}")
