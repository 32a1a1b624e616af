"""GPU: pass-through of in-batch blob payloads (drp_set_blob_skip). Host batches
staged in pieces that resume after each blob they end inside decode exactly like whole-batch
staging and the oracle (decode.js:171-202: blob payload bytes are only sliced, never parsed),
while most blob bytes never reach HBM."""
import random

import numpy as np
import pytest

import _oracle as O
import _streams as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from _gpu import drp_amd
    c = drp_amd.Ctx(0)
    yield c
    c.set_blob_skip(drp_amd.BLOB_SKIP_AUTO)
    c.close()


def _streamed(ctx, wire, sizes):
    """Host batches of the cycled sizes with the JS layer's carry; returns the delivered
    frames (absolute offsets, blob continuations dropped), and the bytes staged / skipped."""
    keys = ["payload_off", "payload_len", "type"] + O.COLS32 + O.COLS64 + ["flags"]
    got = {k: [] for k in keys}
    carry, brem, pos, i, staged, skipped = 0, 0, 0, 0, 0, 0
    w = np.frombuffer(wire, np.uint8)
    while pos < len(w):
        start = pos - carry
        pos = min(len(w), pos + sizes[i % len(sizes)])
        i += 1
        batch = w[start:pos]
        g = ctx.decode_batch(batch, blob_remaining=brem, cap=batch.size // 2 + 4096)
        t = ctx.timing()
        staged += t.h2d_bytes
        skipped += t.h2d_skipped
        assert g["err_code"] == 0, g["err_code"]
        keep = (g["type"][:g["nframes"]] & 0x40) == 0
        for k in keys:
            v = g[k][:g["nframes"]][keep]
            got[k].append(v + np.uint64(start) if k == "payload_off" else v)
        carry = batch.size - g["consumed"] if g["tail"] in (1, 2) else 0
        brem = g["blob_remaining"]
    return {k: np.concatenate(v) for k, v in got.items()}, staged, skipped


def _check(got, ref):
    assert got["type"].size == ref["nframes"]
    for k in ["payload_off", "payload_len"]:
        np.testing.assert_array_equal(got[k].astype(ref[k].dtype), ref[k], err_msg=k)
    np.testing.assert_array_equal(got["type"] & 0x3F, ref["type"], err_msg="type")
    ch = ref["type"] == 1
    for k in O.COLS32 + O.COLS64 + ["flags"]:
        np.testing.assert_array_equal(got[k][ch].astype(ref[k].dtype), ref[k][ch], err_msg=k)


@pytest.mark.parametrize("mode", ["always", "auto"])
def test_c3_blob_payloads_skip_hbm(ctx, mode):
    """C3-shaped stream (1000 C2 frames + one 1 MiB blob per unit, ~113 MB) in ragged host
    batches of 4-17 MiB: every frame equals the oracle's. ALWAYS: at most 25% of the wire is
    staged into HBM (the blobs' payloads stay in host memory). AUTO on flat batches: the blobs
    are too dense for pieces (~150 us of host time each against ~20 us to DMA a 1 MiB blob), so
    after a few probe pieces the rest of each batch is staged whole (drp_api.hip kPieceBudget)."""
    from _gpu import drp_amd
    wire = S.c3_stream(random.Random(5), 100, frames_per_unit=1000)
    ref = O.decode_batch(wire, chunk=65536, cap=100 * 1001 + 16)
    assert ref["nframes"] == 100 * 1001 and ref["err_code"] == 0
    ctx.set_blob_skip(drp_amd.BLOB_SKIP_ALWAYS if mode == "always" else drp_amd.BLOB_SKIP_AUTO)
    sizes = [(16 << 20) + 12345, (4 << 20) + 7, (9 << 20) + 1, (17 << 20) + 85]
    got, staged, skipped = _streamed(ctx, wire, sizes)
    _check(got, ref)
    print(f"{mode}: staged {staged} B ({staged / len(wire):.1%} of the wire), skipped {skipped} B")
    if mode == "always":
        assert staged <= len(wire) // 4, (staged, len(wire))
    else:
        assert staged >= len(wire) // 2, (staged, len(wire))
    assert staged + skipped >= len(wire) * 9 // 10


def test_off_stages_everything(ctx):
    from _gpu import drp_amd
    wire = S.c3_stream(random.Random(6), 12, frames_per_unit=300)
    ctx.set_blob_skip(drp_amd.BLOB_SKIP_OFF)
    got, staged, skipped = _streamed(ctx, wire, [(5 << 20) + 3])
    _check(got, O.decode_batch(wire, chunk=65536))
    # (blob continuations into the next batch are pass-through in every mode)
    assert skipped == 0 and staged >= len(wire) // 2, (skipped, staged, len(wire))


@pytest.mark.parametrize("seed", range(4))
def test_random_streams_in_pieces(ctx, seed):
    """Mixed streams (blobs of 0..200 KB, id-0 headers, wide varints, subsets) decoded in
    blob-skipping pieces from host batches of 1-3 MiB: pieces end inside headers, Change frames
    and blobs of every size, and the result is the oracle's."""
    from _gpu import drp_amd
    rng = random.Random(100 + seed)
    wire = S.random_stream(rng, 40000, blob_p=0.02, blob_max=200000)
    ctx.set_blob_skip(drp_amd.BLOB_SKIP_ALWAYS)
    got, staged, skipped = _streamed(ctx, wire, [(1 << 20) + 17, (3 << 20) + 5, (2 << 20) + 999])
    _check(got, O.decode_batch(wire, chunk=65536))
    assert skipped > 0


def test_error_inside_a_later_piece(ctx):
    """A protocol error after several skipped blobs ends the batch at the right frame."""
    from _gpu import drp_amd
    rng = random.Random(9)
    wire = S.c3_stream(rng, 6, frames_per_unit=200, blob_len=300000) + S.varint(5) + b"\x07" + b"abcd"
    ctx.set_blob_skip(drp_amd.BLOB_SKIP_ALWAYS)
    g = ctx.decode_batch(wire)
    r = O.decode_batch(wire)
    from _gpu import assert_same
    assert_same(g, r, "error after pieces")
    assert r["err_code"] == 1  # 'Protocol error, unknown type: 7'
    assert ctx.timing().h2d_skipped > 0
