"""GPU: drp_decode_fetch_block (the N-API addon's fetch: every column of a staged batch packed on
the device in the caller's block layout, one transfer) returns exactly what drp_decode_fetch
writes into separate columns, for whole and chunked batches, blob-skipping pieces (payload
offsets shifted per piece), a carried blob continuation (row 0 set on the host), a malformed
Change row and the key hash column."""
import random

import numpy as np
import pytest

import _streams as S

pytestmark = pytest.mark.gpu

KEYS = ["payload_off", "payload_len", "type", "key_off", "key_len", "subset_off", "subset_len", "value_off",
        "value_len", "change", "from", "to", "flags"]


@pytest.fixture(scope="module")
def ctx():
    from _gpu import drp_amd
    c = drp_amd.Ctx(0)
    yield c
    c.set_blob_skip(drp_amd.BLOB_SKIP_AUTO)
    c.close()


def _same(ctx, wire, **kw):
    a = ctx.decode_staged(wire, **kw)
    b = ctx.decode_staged(wire, block=True, **kw)
    for k in ["nframes", "err_code", "err_frame", "consumed", "tail", "blob_remaining"]:
        assert a[k] == b[k], k
    rows = a["type"].size
    assert rows == b["type"].size
    for k in KEYS[:3]:
        np.testing.assert_array_equal(b[k], a[k], err_msg=k)
    ch = (a["type"] & 0x3F) == 1  # (a blob row's Change columns are unspecified)
    for k in KEYS[3:] + (["key_hash"] if kw.get("key_hash") else []):
        np.testing.assert_array_equal(b[k][ch], a[k][ch], err_msg=k)
    return a


def test_c2_whole_and_chunked(ctx):
    w = S.c2_stream(20000, seed=4).tobytes()
    a = _same(ctx, w)
    assert a["nframes"] == 20000
    rng = random.Random(2)
    cuts = sorted(rng.sample(range(1, len(w)), 40))
    chunks = [w[i:j] for i, j in zip([0] + cuts, cuts + [len(w)])]
    _same(ctx, chunks)


def test_blob_pieces_and_carried_blob(ctx):
    from _gpu import drp_amd
    ctx.set_blob_skip(drp_amd.BLOB_SKIP_ALWAYS)
    try:
        w = S.c3_stream(random.Random(5), 3, frames_per_unit=300, blob_len=1 << 20)
        a = _same(ctx, w)
        assert ctx.timing().h2d_skipped > 0  # (pieces: payload offsets shifted per piece)
        # a batch that starts inside a blob: its continuation is row 0, set on the host
        _same(ctx, w[1000:], blob_remaining=5000)
    finally:
        ctx.set_blob_skip(drp_amd.BLOB_SKIP_AUTO)
    assert a["nframes"] > 900


def test_malformed_change_and_key_hash(ctx):
    good = S.c2_stream(50, seed=8).tobytes()
    bad = S.frame(b"\x12\x02ab\x18")  # key, then a change field with no varint: malformed
    a = _same(ctx, good + bad + good)
    assert a["err_code"] != 0 and a["type"].size == a["nframes"] + 1
    _same(ctx, S.c2_stream(3000, seed=9).tobytes(), key_hash=True)
