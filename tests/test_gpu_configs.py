"""GPU parity at the BASELINE.json sizes: every config the bench quotes, decoded by libdrp at
its stated size and compared with the CPU oracle (the decode.js / encode.js restatement in
oracle/) on the same bytes.

- C2: 100M Change frames (one 8.6 GB stream), every column of every frame vs the oracle
  (decode.js:144-262 + messages.Change.decode, messages/index.js:5).
- C3: ~1 GiB of C2 frames + 1 MiB blobs, one batch and 64 KiB-ragged streamed batches with
  carry (decode.js:179-202, 216-249), vs the oracle in 64 KiB writes.
- C4: 8192 independent streams (U[8192,16384] frames each) in one segmented call, every
  stream's result and columns vs the oracle run per stream, plus the global index.
- C5: 1M Changes with 4 KB values: the full encoded wire vs the oracle's encode.js
  restatement, and the full decode vs both the encoder input and the oracle's decode.

Each test frees its device memory before the next one starts.
"""
import ctypes as C
import gc
import os
import random
import sys

import numpy as np
import pytest

import _oracle as O
import _streams as S

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture()
def env():
    import torch

    import bench
    from _gpu import drp_amd
    dev = torch.device("cuda", 0)
    ctx = drp_amd.Ctx(0)
    yield torch, bench, drp_amd, dev, ctx
    ctx.close()
    gc.collect()
    torch.cuda.empty_cache()


def _same_col(got, ref, label):
    """Device column (torch, signed) vs oracle column (numpy, unsigned), bit for bit."""
    g = got.cpu().numpy()
    if g.dtype != ref.dtype:
        g = g.view(ref.dtype)
    if not np.array_equal(g, ref):
        bad = np.flatnonzero(g != ref)
        raise AssertionError(f"{label}: {bad.size} rows differ, first {bad[0]}: {g[bad[0]]} vs {ref[bad[0]]}")


def _result(drp_amd, res, s=0):
    rs = C.sizeof(drp_amd.StreamResult)
    raw = res[s * rs:(s + 1) * rs].cpu().numpy().tobytes()
    return drp_amd.StreamResult.from_buffer_copy(raw)


def test_c2_full_size(env):
    """BASELINE configs[1]: 100,000,000 frames x 86 B in one 8.6 GB stream on one GPU (the
    bench workload, same generator). The device-side property check of bench.py, then every
    column of all 100M frames against the oracle decoding the same bytes in 64 KiB writes."""
    torch, bench, drp_amd, dev, ctx = env
    n = 100_000_000
    wire = bench.c2_on_device(n, seed=1234, dev=dev)
    stream_off = torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev)
    cap = n + 64
    outs = bench.alloc_outputs(cap, dev)
    res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    ctx.decode_device(wire, stream_off, None, outs, cap, res)
    torch.cuda.synchronize(dev)
    t = ctx.timing()
    assert t.strict_reruns == 0 and t.seg_repairs == 0
    bench.verify_c2(outs, res, n, dev)
    host = wire.cpu().numpy()
    del wire
    ref = O.decode_batch(host, chunk=65536, cap=n + 16)
    assert (ref["nframes"], ref["err_code"], ref["tail"], ref["consumed"]) == (n, 0, 0, n * 86)
    for k in ["payload_off", "payload_len", "type"] + O.COLS32 + O.COLS64 + ["flags"]:
        _same_col(outs[k][:n], ref[k], f"c2:{k}")


def _device_outputs(torch, drp_amd, cap, dev):
    o = {"payload_off": torch.zeros(cap, dtype=torch.int64, device=dev),
         "payload_len": torch.zeros(cap, dtype=torch.int32, device=dev),
         "type": torch.zeros(cap, dtype=torch.uint8, device=dev),
         "flags": torch.zeros(cap, dtype=torch.uint8, device=dev)}
    for k in drp_amd.COLS32:
        o[k] = torch.zeros(cap, dtype=torch.int32, device=dev)
    for k in drp_amd.COLS64:
        o[k] = torch.zeros(cap, dtype=torch.int64, device=dev)
    return o


def _c3_wire(units=985):
    """~1.07 GB: 985 x (1000 C2 frames + one 1 MiB random blob), SURVEY §8d C3."""
    return S.c3_stream(random.Random(13), units, frames_per_unit=1000)


def _streamed(ctx, wire, sizes, cap_of):
    """Decode `wire` in batches of the cycled `sizes` through drp_decode_batch with the JS
    layer's carry (decode.js carry: header / change payload bytes re-sent, blob continuation
    via blob_remaining). Returns the delivered frames' columns, offsets made absolute, blob
    continuations dropped (the oracle's one-write decode has the whole blob as one frame)."""
    keys = ["payload_off", "payload_len", "type"] + O.COLS32 + O.COLS64 + ["flags"]
    got = {k: [] for k in keys}
    carry, brem, pos, i, batches = 0, 0, 0, 0, 0
    w = np.frombuffer(wire, np.uint8)
    while pos < len(w):
        start = pos - carry
        pos = min(len(w), pos + sizes[i % len(sizes)])
        i += 1
        batch = w[start:pos]
        g = ctx.decode_batch(batch, blob_remaining=brem, cap=cap_of(batch.size))
        batches += 1
        assert g["err_code"] == 0, g["err_code"]
        keep = (g["type"][:g["nframes"]] & 0x40) == 0
        for k in keys:
            v = g[k][:g["nframes"]][keep]
            got[k].append(v + np.uint64(start) if k == "payload_off" else v)
        carry = batch.size - g["consumed"] if g["tail"] in (1, 2) else 0
        brem = g["blob_remaining"]
    return {k: np.concatenate(v) for k, v in got.items()}, batches


def test_c3_1gib(env):
    """BASELINE configs[2]: ~1 GiB of C2 runs and 1 MiB blobs (headers and frames straddle the
    64 KiB write edges of the oracle's decode), decoded by libdrp in one batch and in ragged
    streamed batches with carry; every frame equals the oracle's."""
    torch, bench, drp_amd, dev, ctx = env
    from _gpu import assert_same
    wire = _c3_wire()
    assert len(wire) >= 1 << 30
    nexp = 985 * 1001
    ref = O.decode_batch(wire, chunk=65536, cap=nexp + 16)
    assert ref["nframes"] == nexp and ref["err_code"] == 0 and ref["tail"] == 0
    g = ctx.decode_batch(wire, cap=nexp + 16)
    assert_same(g, ref, "c3 one batch")
    sizes = [(64 << 20) - 12345, 65536 * 7 + 3, 1000003, (3 << 20) + 17, 65536, (17 << 20) + 85]
    got, batches = _streamed(ctx, wire, sizes, lambda nb: nb // 80 + 4096)
    assert batches > 50
    assert got["type"].size == nexp
    for k in ["payload_off", "payload_len"]:
        np.testing.assert_array_equal(got[k].astype(ref[k].dtype), ref[k], err_msg=f"c3 streamed:{k}")
    np.testing.assert_array_equal(got["type"] & 0x3F, ref["type"], err_msg="c3 streamed:type")
    ch = ref["type"] == 1  # (include/drp.h: Change columns of blob rows are left untouched)
    assert ch.sum() == 985 * 1000
    for k in O.COLS32 + O.COLS64 + ["flags"]:
        np.testing.assert_array_equal(got[k][ch].astype(ref[k].dtype), ref[k][ch], err_msg=f"c3 streamed:{k}")


def test_c4_8192_streams(env):
    """BASELINE configs[3] on one GPU: 8192 independent streams of U[8192,16384] C2-shaped
    frames (~100M frames, the bench's generator) in one segmented call. Every stream's result
    and every frame's columns equal the oracle decoding that stream alone (the carry resets per
    stream), and the global index from the stats scan equals the prefix of frame counts."""
    torch, bench, drp_amd, dev, ctx = env
    import drp_dist
    ns = 8192
    wire, stream_off, counts, _ = bench.c4_on_device(ns, 0, 1, dev)
    nf = int(counts.sum())
    cap = nf + 64
    outs = bench.alloc_outputs(cap, dev)
    res = torch.zeros(ns * C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    ctx.decode_device(wire, stream_off, None, outs, cap, res)
    stats = drp_dist.local_stats_device(ctx, res, stream_off)
    base = drp_dist.global_index_device(ctx, stats)
    torch.cuda.synchronize(dev)
    bench.verify_c4(outs, res, counts, base, 0, dev)
    host = wire.cpu().numpy()
    so = stream_off.cpu().numpy()
    del wire
    ref = O.alloc_outputs(nf + 16)
    fb = 0
    for s in range(ns):
        n = int(counts[s])
        view = {k: v[fb:fb + n + 1] for k, v in ref.items()}
        r = O.decode_batch(host[so[s]:so[s + 1]], chunk=65536, outs=view)
        assert (r["nframes"], r["err_code"], r["tail"]) == (n, 0, 0), s
        view["payload_off"][:n] += np.uint64(so[s])
        fb += n
    for k in ["payload_off", "payload_len", "type"] + O.COLS32 + O.COLS64 + ["flags"]:
        _same_col(outs[k][:nf], ref[k][:nf], f"c4:{k}")
    st = stats.cpu().numpy()
    np.testing.assert_array_equal(st[:, 0], counts)
    np.testing.assert_array_equal(st[:, 3], np.diff(so))


def test_c5_full_round_trip(env):
    """BASELINE configs[4] per GPU: 1,000,000 Changes (4096 B values, key U[1,256] with 2-byte
    length varints past 127, change/from/to U[0,2^32)) encoded on the GPU; the whole 4.3 GB wire
    equals the oracle's encode.js + protocol-buffers@2 restatement of the same columns, and the
    GPU decode of it equals the encoder input and the oracle's decode, every column."""
    torch, bench, drp_amd, dev, ctx = env
    n = 1_000_000
    cols, heap, frame = bench.c5_on_device(n, seed=55, dev=dev)
    W = int(frame.sum())
    out = torch.zeros(W + 64, dtype=torch.uint8, device=dev)
    foff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.encode_device(cols, heap, n, foff, out, W + 64)
    wire = out[:W]
    outs = bench.alloc_outputs(n + 64, dev)
    res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    ctx.decode_device(wire, torch.tensor([0, W], dtype=torch.int64, device=dev), None, outs, n + 64, res)
    torch.cuda.synchronize(dev)
    assert ctx.timing().strict_reruns == 0
    assert int(foff[n]) == W and torch.equal(foff[1:] - foff[:-1], frame)
    bench.verify_c5(cols, heap, wire, outs, res, n, dev, samples=64)
    hc = heap.cpu().numpy()
    cc = {k: v.cpu().numpy() for k, v in cols.items()}
    cc = {k: (v.astype(np.uint64) if k in ("key_off", "subset_off", "value_off", "change", "from", "to")
              else v.astype(np.uint32) if k.endswith("_len") else v) for k, v in cc.items()}
    host_wire = wire.cpu().numpy()
    exp = np.frombuffer(O.encode_changes(hc.tobytes(), cc), np.uint8)
    assert exp.size == W
    if not np.array_equal(host_wire, exp):
        bad = np.flatnonzero(host_wire != exp)
        raise AssertionError(f"c5 wire: {bad.size} bytes differ, first at {bad[0]}")
    ref = O.decode_batch(host_wire, chunk=65536, cap=n + 16)
    assert (ref["nframes"], ref["err_code"], ref["tail"]) == (n, 0, 0)
    for k in ["payload_off", "payload_len", "type"] + O.COLS32 + O.COLS64 + ["flags"]:
        _same_col(outs[k][:n], ref[k], f"c5:{k}")
