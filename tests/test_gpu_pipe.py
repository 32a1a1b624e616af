"""GPU: pipelined staging of large flat batches in page-locked memory (drp_api.hip, drp_ctx::pipe_chunk).
The DMA engine copies the batch in 128 MiB chunks on the ctx's copy stream while the compute
stream decodes one piece per chunk; pieces resume at the frame a chunk edge cut and jump the
blobs they end inside (decode.js:179-202: blob payloads are only sliced). Every frame, the carry
and the error must equal the oracle's whole-batch decode, and the staged rows stay one piece
(payload offsets shifted on the device), so the device-built key text works too."""
import random

import numpy as np
import pytest

import _oracle as O
import _streams as S

pytestmark = pytest.mark.gpu

MiB = 1 << 20


@pytest.fixture(params=["32", "128"])
def ctx(request, monkeypatch):
    """A ctx pipelining in 32 MiB chunks (many piece edges) or in the default 128 MiB ones
    (DRP_PIPE_CHUNK is read when the ctx opens)."""
    from _gpu import drp_amd
    monkeypatch.setenv("DRP_PIPE_CHUNK", request.param)
    c = drp_amd.Ctx(0)
    c.pipe_chunk = int(request.param) << 20
    yield c
    c.close()


def _pinned(wire):
    import torch
    t = torch.empty(len(wire), dtype=torch.uint8, pin_memory=True)
    a = t.numpy()
    a[:] = np.frombuffer(wire, np.uint8)
    return t, a


def _key_text(wire, r, rows):
    """The oracle's ASCII keys of the well-formed Change rows end to end, and each row's position."""
    ty, fl = r["type"][:rows] & 0x3F, r["flags"][:rows]
    ok = np.flatnonzero((ty == 1) & ((fl & 4) == 0))
    ok = ok[ok < r["nframes"]]
    kp, parts, tot, last = np.zeros(rows, np.uint32), [], 0, 0
    for k in ok:
        po, ko, kl = int(r["payload_off"][k]), int(r["key_off"][k]), int(r["key_len"][k])
        key = wire[po + ko:po + ko + kl]
        kp[last:k + 1] = tot
        last = k + 1
        if key.isascii():
            parts.append(key)
            tot += len(key)
    kp[last:] = tot
    return kp, b"".join(parts)


def test_pipelined_c3_batches(ctx):
    """A 283 MB C3-shaped batch (1000 C2 frames + one 1 MiB blob per unit) from pinned memory:
    the first decode probes in blob-skipping pieces and pipelines the rest, the next ones
    pipeline the whole batch; all equal the oracle, and the key text built on the device too."""
    from _gpu import assert_same
    wire = S.c3_stream(random.Random(31), 250, frames_per_unit=1000)
    nexp = 250 * 1001
    ref = O.decode_batch(wire, cap=nexp + 16)
    assert ref["nframes"] == nexp and ref["err_code"] == 0
    assert len(wire) >= 2 * ctx.pipe_chunk
    t, a = _pinned(wire)
    for k in range(3):
        g = ctx.decode_batch(a, cap=nexp + 16)
        assert_same(g, ref, f"c3 pinned #{k}")
        tm = ctx.timing()
        assert tm.h2d_bytes + tm.h2d_skipped >= len(wire) * 9 // 10, (k, tm.h2d_bytes, tm.h2d_skipped)
    o = ctx.decode_staged(a, keys=True)
    assert o["nframes"] == nexp
    kp, text = _key_text(wire, ref, nexp)
    assert o["key_text"] == text
    np.testing.assert_array_equal(o["kp"], kp)
    del t


def _long_frames_wire(rng):
    """C2 runs, a 150 MB blob and a Change with a 70 MB value (each spans chunk edges), mixed
    random frames (blobs up to 200 KB, id-0 headers, wide varints)."""
    big_value = S.frame(S.change_payload(b"big-value-key", 7, 8, 9, value=rng.randbytes(70 * MiB)))
    return (S.c2_stream(200000, seed=41).tobytes() + S.frame(rng.randbytes(150 * MiB), 2) + big_value
            + S.random_stream(rng, 60000, blob_p=0.02, blob_max=200000))


@pytest.mark.parametrize("case", ["whole", "carried", "cut_blob", "bad_type", "bad_change"])
def test_pipelined_long_frames_carry_and_errors(ctx, case):
    """Frames longer than a chunk, a leading blob continuation, a batch that ends inside a blob,
    and protocol errors in a later chunk (unknown type; a malformed Change, whose row is
    delivered) through the pipelined pieces, vs the oracle's whole-batch decode."""
    from _gpu import assert_same, drp_amd
    rng = random.Random(["whole", "carried", "cut_blob", "bad_type", "bad_change"].index(case) + 50)
    wire = _long_frames_wire(rng)
    brem = 0
    if case == "carried":
        brem = 3 * MiB + 5
        wire = rng.randbytes(brem) + wire
    elif case == "cut_blob":
        wire += S.varint(40 * MiB + 1) + b"\x02" + rng.randbytes(5 * MiB)
    elif case == "bad_type":
        wire = wire + S.varint(5) + b"\x07abcd" + S.c2_stream(1000, seed=5).tobytes()
    elif case == "bad_change":
        wire = wire + S.frame(b"\xff\xff\xff", 1) + S.c2_stream(1000, seed=6).tobytes()
    assert len(wire) >= 2 * ctx.pipe_chunk
    ref = O.decode_batch(wire, blob_remaining=brem, cap=2_000_000)
    assert ref["nframes"] < 1_999_000
    t, a = _pinned(wire)
    ctx.set_blob_skip(drp_amd.BLOB_SKIP_OFF)  # (straight to the pipelined whole-batch staging)
    try:
        g = ctx.decode_batch(a, blob_remaining=brem, cap=2_000_000)
        assert_same(g, ref, f"{case} pinned")
        assert ctx.timing().h2d_skipped == 0
        ctx.set_blob_skip(drp_amd.BLOB_SKIP_AUTO)
        g = ctx.decode_batch(a, blob_remaining=brem, cap=2_000_000)
        assert_same(g, ref, f"{case} pinned auto")
    finally:
        ctx.set_blob_skip(drp_amd.BLOB_SKIP_AUTO)
    del t


@pytest.mark.parametrize("block", [False, True])
def test_pipelined_stage_then_fetch(ctx, block):
    """drp_decode_stage of a pipelined batch, then the staged rows fetched later: in three
    drp_decode_fetch calls, or as one drp_decode_fetch_block_ex with f64 columns; the key text
    (drp_decode_fetch_keys) when the rows are one staged range (a fresh ctx's first batch probes in
    pieces first: then it may decline, as for any batch staged in pieces)."""
    wire = S.c3_stream(random.Random(37), 250, frames_per_unit=1000)
    nexp = 250 * 1001
    ref = O.decode_batch(wire, cap=nexp + 16)
    t, a = _pinned(wire)
    for k in range(2):
        o = ctx.decode_staged(a, pieces=3, block=block, f64=block, keys=True)
        assert (o["nframes"], o["err_code"], o["consumed"]) == (nexp, 0, len(wire))
        for c in ["payload_off", "payload_len", "type"]:
            np.testing.assert_array_equal(o[c].astype(np.float64 if block and c == "payload_off" else ref[c].dtype),
                                          ref[c].astype(np.float64) if block and c == "payload_off" else ref[c],
                                          err_msg=f"#{k}:{c}")
        ch = ref["type"] == 1
        for c in O.COLS32:
            np.testing.assert_array_equal(o[c][ch], ref[c][ch], err_msg=f"#{k}:{c}")
        # (keys=True adds the key flags, DRP_F_KEY_ASCII | DRP_F_KEY_UTF8: C2 keys are ASCII)
        np.testing.assert_array_equal(o["flags"][ch] & 0x0F, ref["flags"][ch], err_msg=f"#{k}:flags")
        assert np.all(o["flags"][ch] & 0x30 == 0x30)
        for c in O.COLS64:
            np.testing.assert_array_equal(o[c][ch].astype(np.float64) if block else o[c][ch],
                                          ref[c][ch].astype(np.float64) if block else ref[c][ch], err_msg=f"#{k}:{c}")
        if k == 1 or o["key_text"] is not None:
            kp, text = _key_text(wire, ref, nexp)
            assert o["key_text"] == text
            np.testing.assert_array_equal(o["kp"], kp)
    del t
