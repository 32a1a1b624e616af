"""GPU parity: libdrp's gfx950 decode/encode vs the oracle (decode.js / encode.js
restatement), bit-exact on every column.

Run on an MI355X:  python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
import json
import os
import random

import numpy as np
import pytest

import _oracle as O
import _streams as S

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ctx():
    from _gpu import drp_amd
    c = drp_amd.Ctx(0)
    yield c
    c.close()


def test_golden_streams(ctx):
    from _gpu import assert_same
    vecs = json.load(open(os.path.join(GOLD, "streams.json")))["vectors"]
    for v in vecs:
        wire = bytes.fromhex(v["wire"])
        assert_same(ctx.decode_batch(wire), O.decode_batch(wire), v["source"])


@pytest.mark.parametrize("kernel", ["speculative", "exact4096", "exact8192"])
@pytest.mark.parametrize("seed", range(4))
def test_random_streams(ctx, kernel, seed):
    """Both decode kernels (the tile size only applies to the exact one)."""
    from _gpu import assert_same
    if kernel != "speculative":
        ctx.set_exact(True)
        ctx.set_tile(int(kernel[5:]))
    try:
        rng = random.Random(seed)
        wire = S.random_stream(rng, 3000)
        wire = wire[:rng.randint(len(wire) // 2, len(wire))]
        assert_same(ctx.decode_batch(wire), O.decode_batch(wire), f"seed{seed}/{kernel}")
    finally:
        ctx.set_tile(0)
        ctx.set_exact(False)


def test_strict_equals_lookback(ctx):
    from _gpu import assert_same
    rng = random.Random(11)
    wire = S.random_stream(rng, 4000, blob_p=0.1, blob_max=20000)
    ref = O.decode_batch(wire)
    ctx.set_strict(True)
    try:
        assert_same(ctx.decode_batch(wire), ref, "strict")
    finally:
        ctx.set_strict(False)
    assert_same(ctx.decode_batch(wire), ref, "lookback")


def test_c2_shape(ctx):
    from _gpu import assert_same
    wire = S.c2_stream(200_000, seed=5).tobytes()
    g = ctx.decode_batch(wire)
    assert g["nframes"] == 200_000 and g["err_code"] == 0 and g["tail"] == 0
    assert_same(g, O.decode_batch(wire, chunk=65536), "c2")


def test_c5_shape(ctx):
    from _gpu import assert_same
    wire = S.c5_stream(random.Random(9), 3000)
    assert_same(ctx.decode_batch(wire), O.decode_batch(wire, chunk=65536), "c5")


def test_c3_shape(ctx):
    from _gpu import assert_same
    wire = S.c3_stream(random.Random(4), 3, frames_per_unit=1000)
    g = ctx.decode_batch(wire)
    assert g["nframes"] == 3003
    assert_same(g, O.decode_batch(wire, chunk=65536), "c3")


@pytest.mark.parametrize("seed", range(3))
def test_errors_and_tails(ctx, seed):
    """Protocol errors (decode.js:159-161) and policy errors injected at frame boundaries."""
    from _gpu import assert_same
    rng = random.Random(100 + seed)
    base = S.random_stream(rng, 800)
    bad = [b"\x03\x07ab", b"\x00\x01", b"\x80" * 10 + b"\x01\x01", b"\x01\x01",
           S.frame(b"\x12\x05k"), S.frame(b"\x12\x01k\x18\x01\x20\x02\x28\x03\x3b")]
    for b in bad:
        cut = rng.randint(0, len(base))
        r0 = O.decode_batch(base[:cut])
        if r0["tail"] == 3:
            continue
        cut = r0["consumed"]
        wire = base[:cut] + b + base
        assert_same(ctx.decode_batch(wire), O.decode_batch(wire), repr(b))


def test_batches_with_carry(ctx):
    """Split a stream into batches at random points and carry state like the JS layer; every
    frame's offset, length, type and Change columns equal the oracle's one-write decode."""
    from _gpu import COL_KEYS, stream_decode
    rng = random.Random(21)
    wire = S.random_stream(rng, 2000, blob_p=0.1, blob_max=5000)
    ref = O.decode_batch(wire)
    frames, err = stream_decode(ctx, wire, [rng.choice([1, 7, 100, 4096, 30000]) for _ in range(4000)])
    assert err is None
    got = [f for f in frames if not (f["type"] & 0x40)]  # blob continuations merge into their blob
    assert len(got) == ref["nframes"]
    for k, f in enumerate(got):
        assert (f["type"] & 0x3F, f["off"], f["len"]) == \
            (int(ref["type"][k]) & 0x3F, int(ref["payload_off"][k]), int(ref["payload_len"][k])), k
        if f["type"] & 0x3F == 1:
            assert [f[c] for c in COL_KEYS] == [int(ref[c][k]) for c in COL_KEYS], k


def _random_cols(rng, n):
    heap = bytearray()
    cols = {k: [] for k in ["key_off", "key_len", "subset_off", "subset_len", "value_off",
                            "value_len", "change", "from", "to", "flags"]}
    for _ in range(n):
        for name, b in [("key", rng.randbytes(rng.randint(0, 300))),
                        ("value", rng.randbytes(rng.choice([0, 3, 64, 4096]))),
                        ("subset", rng.randbytes(rng.randint(0, 4)))]:
            cols[name + "_off"].append(len(heap))
            cols[name + "_len"].append(len(b))
            heap += b
        cols["change"].append(rng.randint(0, 2**53 - 1))
        cols["from"].append(rng.randint(0, 2**32 - 1))
        cols["to"].append(rng.randint(0, 127))
        cols["flags"].append((1 if rng.random() < 0.3 else 0) | (2 if rng.random() < 0.9 else 0))
    dt = {"key_off": np.uint64, "subset_off": np.uint64, "value_off": np.uint64,
          "key_len": np.uint32, "subset_len": np.uint32, "value_len": np.uint32,
          "change": np.uint64, "from": np.uint64, "to": np.uint64, "flags": np.uint8}
    return bytes(heap), {k: np.array(v, dtype=dt[k]) for k, v in cols.items()}


def test_encode_matches_oracle(ctx):
    heap, c = _random_cols(random.Random(3), 3000)
    g = ctx.encode_batch(heap, c)
    assert g == O.encode_changes(heap, c)
    d = ctx.decode_batch(g)
    assert d["nframes"] == 3000 and d["err_code"] == 0
    np.testing.assert_array_equal(d["change"], c["change"])
    np.testing.assert_array_equal(d["from"], c["from"])
    np.testing.assert_array_equal(d["flags"], c["flags"])


@pytest.mark.parametrize("shape", ["c2", "c3", "c5", "random"])
def test_speculative_matches_exact(ctx, shape):
    """The default decode (speculate-and-verify kernels) and the exact kernel give identical
    columns; on clean C2-shaped streams the prediction must hold everywhere (no exact re-run)."""
    from _gpu import assert_same
    rng = random.Random(77)
    wire = {"c2": lambda: S.c2_stream(300_000, seed=8).tobytes(),
            "c3": lambda: S.c3_stream(rng, 2, frames_per_unit=1000),
            "c5": lambda: S.c5_stream(rng, 2000),
            "random": lambda: S.random_stream(rng, 5000, blob_p=0.05, blob_max=30000)}[shape]()
    spec = ctx.decode_batch(wire)
    reruns = ctx.timing().strict_reruns
    ctx.set_exact(True)
    try:
        exact = ctx.decode_batch(wire)
        assert ctx.timing().strict_reruns == 0
    finally:
        ctx.set_exact(False)
    assert_same(spec, exact, shape)
    assert_same(spec, O.decode_batch(wire, chunk=65536), shape)
    if shape == "c2":
        assert reruns == 0, "prediction failed on a clean C2 stream"


def test_c5_device_round_trip(ctx):
    """C5 shape through the device entry points: drp_encode_device -> drp_decode_device; frame
    sizes match the encode.js layout, decoded columns equal the encoder input, sampled key and
    value bytes equal the heap (the same checks bench.py --workload c5 runs at full size)."""
    import ctypes as C
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from _gpu import drp_amd
    dev = torch.device("cuda", 0)
    n = 20_000
    cols, heap, frame = bench.c5_on_device(n, seed=3, dev=dev)
    W = int(frame.sum())
    out = torch.zeros(W + 64, dtype=torch.uint8, device=dev)
    foff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.encode_device(cols, heap, n, foff, out, W + 64)
    outs = bench.alloc_outputs(n + 64, dev)
    res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    wire = out[:W]
    ctx.decode_device(wire, torch.tensor([0, W], dtype=torch.int64, device=dev), None, outs, n + 64, res)
    torch.cuda.synchronize(dev)
    assert int(foff[n]) == W and torch.equal(foff[1:] - foff[:-1], frame)
    bench.verify_c5(cols, heap, wire, outs, res, n, dev, samples=64)
    # and the wire equals the CPU restatement of encode.js on the same columns
    hc = heap.cpu().numpy()
    cc = {k: v.cpu().numpy() for k, v in cols.items()}
    cc = {k: (v.astype(np.uint64) if k in ("key_off", "subset_off", "value_off", "change", "from", "to")
              else v.astype(np.uint32) if k.endswith("_len") else v) for k, v in cc.items()}
    assert wire.cpu().numpy().tobytes() == O.encode_changes(hc.tobytes(), cc)


def test_c3_many_blobs(ctx):
    """C3 shape at 40 MiB: 1 MiB random blobs between C2 runs; every column bit-exact vs the
    oracle's 64 KiB-chunked decode, and neither a repair nor a fallback changes the result."""
    from _gpu import assert_same
    wire = S.c3_stream(random.Random(12), 40, frames_per_unit=1000)
    g = ctx.decode_batch(wire)
    assert g["nframes"] == 40 * 1001 and g["err_code"] == 0
    assert_same(g, O.decode_batch(wire, chunk=65536), "c3x40")


def test_c5_predicted_without_repairs():
    """A 200K-Change C5 stream (random 4 KB values, keys of 1..256 bytes) is predicted without a
    single miss: no repair pass, no exact re-run (C5's long frames are strong by structure,
    DESIGN.md "Long frames"), and the decode is bit-exact with the encoder's input. The repair
    passes themselves are exercised by the shadow streams of test_gpu_cascade.py."""
    import ctypes as C
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from _gpu import drp_amd
    dev = torch.device("cuda", 0)
    n = 200_000
    # a ctx of its own: the structural check of long frames is chosen from the ctx's previous
    # decodes (dense streams leave it off), and this one decodes C5 from the start
    ctx = drp_amd.Ctx(0)
    cols, heap, frame = bench.c5_on_device(n, seed=55, dev=dev)
    W = int(frame.sum())
    out = torch.zeros(W + 64, dtype=torch.uint8, device=dev)
    foff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.encode_device(cols, heap, n, foff, out, W + 64)
    outs = bench.alloc_outputs(n + 64, dev)
    res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    wire = out[:W]
    ctx.decode_device(wire, torch.tensor([0, W], dtype=torch.int64, device=dev), None, outs, n + 64, res)
    torch.cuda.synchronize(dev)
    t = ctx.timing()
    print(f"repair passes {t.spec_repairs}, exact re-runs {t.strict_reruns}")
    bench.verify_c5(cols, heap, wire, outs, res, n, dev, samples=64)
    ctx.close()
    assert t.strict_reruns == 0 and t.spec_repairs == 0, (t.spec_repairs, t.strict_reruns)


def test_stream_ends_not_relisted():
    """The same C2 frames as 1 and as 512 streams cut at frame boundaries: the records-only check
    relists about as many tiles either way. (Threads past a stream's end used to get the chain's
    end as a wrapped entry byte that read as a restart, so every stream's last tile went to the
    full re-walk: C4 relisted 11909 tiles instead of ~4000.) Results stay exact (bench.verify_c4
    checks the frame table against the generator)."""
    import ctypes as C

    import torch

    import bench
    from _gpu import drp_amd
    dev = torch.device("cuda", 0)
    n, fb = 2_000_000, 86
    wire = bench.c2_on_device(n, seed=77, dev=dev)
    outs = bench.alloc_outputs(n + 64, dev)
    res = torch.zeros(512 * C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    relisted = {}
    with drp_amd.Ctx(0) as ctx:
        for s in (1, 512):
            per = n // s
            cuts = [i * per * fb for i in range(s)] + [wire.numel()]
            so = torch.tensor(cuts, dtype=torch.int64, device=dev)
            ctx.decode_device(wire, so, None, outs, n + 64, res)
            torch.cuda.synchronize()
            t = ctx.timing()
            assert t.strict_reruns == 0
            relisted[s] = t.verify_relisted
            off = outs["payload_off"][:n].cpu().numpy()
            np.testing.assert_array_equal(off, np.arange(n, dtype=np.int64) * fb + 2)
    assert relisted[512] <= relisted[1] + 64, relisted


def test_c5_after_c2_on_one_context():
    """native.js pools contexts across streams, so a C5 stream can land on a context whose last
    decode was dense C2, which turned claims_fast's long-frame check off: that decode then relies
    on the repair passes (and segmented repair). It must still be bit-exact with the encoder's
    input and never fall back to the exact kernel; the next decode on the context has the check
    back on and needs no repair."""
    import ctypes as C
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from _gpu import drp_amd
    dev = torch.device("cuda", 0)
    ctx = drp_amd.Ctx(0)
    nc2 = 2_000_000
    w2 = bench.c2_on_device(nc2, seed=9, dev=dev)
    o2 = bench.alloc_outputs(nc2 + 64, dev)
    r2 = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    for _ in range(2):  # (the first decode of a context runs the check; the second one does not)
        ctx.decode_device(w2, torch.tensor([0, w2.numel()], dtype=torch.int64, device=dev), None, o2, nc2 + 64, r2)
    torch.cuda.synchronize(dev)
    bench.verify_c2(o2, r2, nc2, dev)
    del w2, o2
    n = 200_000
    cols, heap, frame = bench.c5_on_device(n, seed=56, dev=dev)
    W = int(frame.sum())
    out = torch.zeros(W + 64, dtype=torch.uint8, device=dev)
    foff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.encode_device(cols, heap, n, foff, out, W + 64)
    outs = bench.alloc_outputs(n + 64, dev)
    res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    wire = out[:W]
    so = torch.tensor([0, W], dtype=torch.int64, device=dev)
    reps = []
    for _ in range(2):
        outs["change"].fill_(0)
        ctx.decode_device(wire, so, None, outs, n + 64, res)
        torch.cuda.synchronize(dev)
        t = ctx.timing()
        reps.append((t.spec_repairs, t.seg_repairs, t.strict_reruns))
        bench.verify_c5(cols, heap, wire, outs, res, n, dev, samples=64)
    ctx.close()
    print(f"C5 after C2 (repairs, segmented, exact): {reps}")
    assert reps[0][2] == 0 and reps[1] == (0, 0, 0), reps


def test_encode_rejects_out_of_range_rows(ctx):
    """A row whose key/subset/value range leaves the heap is DRP_E_INVAL, not a device fault
    (drp.h: every call returns a code)."""
    from _gpu import drp_amd
    heap, c = _random_cols(random.Random(4), 50)
    for col, bad in [("key_off", len(heap) + 1), ("value_len", len(heap) + 1), ("subset_off", 2**64 - 2)]:
        cc = {k: v.copy() for k, v in c.items()}
        cc["flags"][17] |= 3  # subset and value present: their ranges are checked
        cc[col][17] = bad
        with pytest.raises(drp_amd.DrpError) as e:
            ctx.encode_batch(heap, cc)
        assert e.value.rc == drp_amd.DRP_E_INVAL, col
    assert ctx.encode_batch(heap, c) == O.encode_changes(heap, c)  # the context is still usable


def test_encode_max_width_varints(ctx):
    """change/from/to at 2^64 - 1 (10-byte varints) beside a value: 39 bytes of field prefixes
    in one frame, equal to the oracle's encoding (the C ABI takes any uint64)."""
    heap, c = _random_cols(random.Random(5), 64)
    for k in ["change", "from", "to"]:
        c[k][:] = np.uint64(2**64 - 1)
    c["flags"][:] |= 2
    assert ctx.encode_batch(heap, c) == O.encode_changes(heap, c)


@pytest.mark.parametrize("shape", ["tiny", "c1", "c5", "mixed", "edge"])
def test_encode_write_paths_match_oracle(ctx, shape):
    """The encode write covers the output with 64 KiB blocks (drp_encode.hip): a block touching
    at most ENC_FMAX frames is written chunk by chunk (16-byte copies out of the heap, chunks that
    mix segments piece by piece, listed in LDS), a denser one frame by frame. Frames of ~10 bytes
    (dense blocks), C1-sized ones (dense at 64 KiB), 4 KB values (whole copies), ~500-byte frames
    with short keys, subsets and long varints (the most mixed chunks a block can hold, around
    ENC_FMAX frames a block), and all of them interleaved, written at every alignment of the
    output pointer: the wire
    equals the oracle's encode.js + protocol-buffers@2 restatement byte for byte, and the bytes
    around it are untouched."""
    import torch
    rng = np.random.default_rng({"tiny": 1, "c1": 2, "c5": 3, "mixed": 4, "edge": 5}[shape])
    n = {"tiny": 40_000, "c1": 20_000, "c5": 2_000, "mixed": 30_000, "edge": 20_000}[shape]
    kind = {"tiny": np.zeros(n, int), "c1": np.ones(n, int), "c5": np.full(n, 2),
            "mixed": rng.integers(0, 3, n), "edge": np.full(n, 3)}[shape]
    if shape == "mixed":  # runs of each kind, so dense and sparse blocks alternate
        kind = np.repeat(rng.integers(0, 3, n // 500 + 1), 500)[:n]
    kl = np.select([kind == 0, kind == 1, kind == 2], [rng.integers(0, 3, n), 32, rng.integers(1, 257, n)],
                   rng.integers(0, 40, n)).astype(np.uint32)
    vl = np.select([kind == 0, kind == 1, kind == 2], [0, 64, 4096], rng.integers(380, 460, n)).astype(np.uint32)
    sub = (rng.random(n) < {"mixed": 0.3, "edge": 0.5}.get(shape, 0.0))
    sl = np.where(sub, rng.integers(0, 200 if shape == "mixed" else 40, n), 0).astype(np.uint32)
    flags = (sub.astype(np.uint8) | np.where((kind > 0) | (rng.random(n) < 0.5), 2, 0).astype(np.uint8))
    row = kl.astype(np.uint64) + sl + vl
    base = np.cumsum(row) - row
    heap = rng.integers(0, 256, int(row.sum()) + 16, dtype=np.uint8)
    nums = rng.integers(0, 1 << 40, (3, n), dtype=np.uint64)
    if shape in ("mixed", "edge"):
        nums[:, ::7] = np.uint64(2**64 - 1)
    cols = {"key_off": base, "key_len": kl, "subset_off": base + kl, "subset_len": sl,
            "value_off": base + kl + sl, "value_len": vl, "change": nums[0], "from": nums[1], "to": nums[2],
            "flags": flags}
    exp = O.encode_changes(heap.tobytes(), cols)
    dev = torch.device("cuda", 0)
    ct = {k: torch.from_numpy(v.astype(np.int64) if v.dtype == np.uint64 else
                              (v.astype(np.int32) if v.dtype == np.uint32 else v)).to(dev) for k, v in cols.items()}
    ht = torch.from_numpy(heap).to(dev)
    foff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    W = len(exp)
    for shift in ([0, 1, 7, 15] if shape not in ("mixed", "edge") else range(16)):
        buf = torch.full((W + 64,), 0xA5, dtype=torch.uint8, device=dev)
        ctx.encode_device(ct, ht, n, foff, buf[16 + shift:], W + 32)
        torch.cuda.synchronize(dev)
        got = buf.cpu().numpy()
        assert int(foff[n]) == W
        assert got[16 + shift:16 + shift + W].tobytes() == exp, (shape, shift)
        assert (got[:16 + shift] == 0xA5).all() and (got[16 + shift + W:] == 0xA5).all(), (shape, shift)


def test_stage_fetch_pieces_and_continuations(ctx):
    """drp_decode_stage + drp_decode_fetch (the N-API path): rows fetched in pieces equal the
    one-call decode; a leading blob continuation of every length mod 16 (its bytes are not
    staged to HBM: the device stream starts at the aligned offset after it) gives the oracle's
    frames at the right absolute offsets; a change frame cut by the batch end reports its full
    size (drp_carry.frame_bytes) for the O(n) carry."""
    from _gpu import assert_same
    rng = random.Random(31)
    wire = S.random_stream(rng, 1500, blob_p=0.1, blob_max=3000)
    full = ctx.decode_batch(wire)
    for pieces in (1, 3, 7):
        st = ctx.decode_staged(wire, pieces=pieces)
        assert_same({k: (v[:len(full["type"])] if hasattr(v, "shape") else v) for k, v in st.items()}, full,
                    f"pieces{pieces}")
    for brem in list(range(1, 40)) + [4095, 4096, 4097, 65537]:
        w = rng.randbytes(brem) + wire
        g = ctx.decode_staged(w, blob_remaining=brem)
        r = O.decode_batch(w, blob_remaining=brem)
        assert_same({k: (v[:len(r["type"])] if hasattr(v, "shape") else v) for k, v in g.items()}, r, f"brem{brem}")
    f = S.frame(S.change_payload(b"k" * 40, 1, 2, 3, value=rng.randbytes(5000)))
    for cut in (3, 100, len(f) - 1):  # (1 or 2 bytes: the header itself is incomplete)
        g = ctx.decode_staged(wire + f[:cut])
        assert g["tail"] == 2 and g["frame_bytes"] == len(f) and g["consumed"] == len(wire), cut


@pytest.mark.parametrize("shape", ["c2", "c5", "random"])
def test_cut_streams_edge_tiles(shape):
    """One wire cut into ~150 streams at arbitrary bytes (no cut on a frame boundary): every stream
    enters mid-frame (its entry is the first frame start, as the JS carry passes it) and ends in a
    cut frame, so nearly every first and last tile is a stream-edge tile, which spec_claims runs in
    the fast claims form (DRP_EDGE_FAST) with the stream's bounds. Rows, counts and tails equal the
    oracle's decode of each stream's bytes from its entry; no exact re-run."""
    import ctypes as C

    import sys

    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from _gpu import drp_amd
    dev = torch.device("cuda", 0)
    rng = random.Random(404)
    wire = {"c2": lambda: S.c2_stream(60_000, seed=6).tobytes(),
            "c5": lambda: S.c5_stream(rng, 1200),
            "random": lambda: S.random_stream(rng, 20_000, blob_p=0.02, blob_max=20000)}[shape]()
    whole = O.decode_batch(wire)
    assert whole["err_code"] == 0
    ends = whole["payload_off"].astype(np.int64) + whole["payload_len"].astype(np.int64)
    starts = np.concatenate([[0], ends[:-1]])  # frame k starts where frame k - 1's payload ends
    cuts = sorted(rng.sample(range(1, len(wire)), 149))
    cuts = [0] + [c for c in cuts if int(np.searchsorted(starts, c, "left")) < len(starts) and
                  starts[np.searchsorted(starts, c, "left")] != c] + [len(wire)]
    cuts = sorted(set(cuts))
    entry = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        j = int(np.searchsorted(starts, a, "left"))
        entry.append(min(int(starts[j]) if j < len(starts) else b, b) - a)
    ns = len(cuts) - 1
    cap = len(starts) + 64
    outs = bench.alloc_outputs(cap, dev)
    res = torch.zeros(ns * C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    w = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).to(dev)
    so = torch.tensor(cuts, dtype=torch.int64, device=dev)
    en = torch.tensor(entry, dtype=torch.int64, device=dev)
    with drp_amd.Ctx(0) as ctx:
        for _ in range(2):  # (the second decode with the long-frame check chosen from the first)
            ctx.decode_device(w, so, en, outs, cap, res)
            torch.cuda.synchronize()
            t = ctx.timing()
            print(f"{shape}: {ns} streams, repairs {t.spec_repairs}, relisted {t.verify_relisted}, "
                  f"seg {t.seg_repairs}, exact {t.strict_reruns}")
            assert t.strict_reruns == 0
            rs = (drp_amd.StreamResult * ns).from_buffer_copy(res.cpu().numpy().tobytes())
            off = outs["payload_off"].cpu().numpy()
            ln = outs["payload_len"].cpu().numpy()
            ty = outs["type"].cpu().numpy()
            for s, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
                e = a + entry[s]
                r = O.decode_batch(wire[e:b])
                f0, nf = rs[s].frame_begin, rs[s].frames
                assert (nf, rs[s].err_code, rs[s].tail_kind) == (r["nframes"], r["err_code"], r["tail"]), (s, a, b)
                np.testing.assert_array_equal(off[f0:f0 + nf], r["payload_off"].astype(np.int64) + e)
                np.testing.assert_array_equal(ln[f0:f0 + nf], r["payload_len"])
                np.testing.assert_array_equal(ty[f0:f0 + nf], r["type"])
