"""GPU parity for the on-GPU key post-processing (decode.js:210-213): the key hash
column is XXH64 (seed 0) of the key bytes (checked against python-xxhash) and the key flags
say whether the bytes are ASCII / well-formed UTF-8 (checked against Python's strict UTF-8
decoder), on both decode paths and on the staged (N-API) path; the other columns are
unchanged by it."""
import random

import numpy as np
import pytest
import xxhash

import _oracle as O
import _streams as S

pytestmark = pytest.mark.gpu

KEYS = [b"", b"key", b"0123456789", b"a" * 31, b"a" * 32, b"b" * 33, b"c" * 100, b"d" * 300,
        "été".encode(), "日本語キー".encode(), "🙂 emoji".encode(), b"\xc0\x80", b"\xed\xa0\x80",
        b"\xf4\x90\x80\x80", b"\xe2\x82", b"ok\xff", b"\x80abc", b"\xf0\x9f\x99", "ok".encode() + b"\xc3",
        b"\xef\xbf\xbf", b"\xf4\x8f\xbf\xbf", b"\xe0\xa0\x80", b"\xe0\x9f\xbf"]


def _stream(rng, n):
    parts = []
    for i in range(n):
        k = KEYS[i % len(KEYS)] if i < 4 * len(KEYS) else rng.randbytes(rng.randint(0, 80))
        if rng.random() < 0.3:
            k = bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(rng.randint(0, 70)))
        parts.append(S.frame(S.change_payload(k, i, 1, 2, value=rng.randbytes(rng.randint(0, 90)))))
        if rng.random() < 0.05:
            parts.append(S.frame(rng.randbytes(rng.randint(0, 500)), 2))
    return b"".join(parts)


def _expect(wire, r):
    for k in range(r["nframes"]):
        if r["type"][k] & 0x3F != 1:
            continue
        po = int(r["payload_off"][k])
        key = wire[po + int(r["key_off"][k]):po + int(r["key_off"][k]) + int(r["key_len"][k])]
        try:
            key.decode("utf-8")
            utf8 = True
        except UnicodeDecodeError:
            utf8 = False
        yield k, xxhash.xxh64_intdigest(key), (0x10 if key.isascii() else 0) | (0x20 if utf8 else 0)


@pytest.fixture(scope="module")
def ctx():
    from _gpu import drp_amd
    c = drp_amd.Ctx(0)
    yield c
    c.close()


@pytest.mark.parametrize("kernel", ["speculative", "exact8192", "staged"])
def test_key_hash_and_flags(ctx, kernel):
    from _gpu import assert_same
    wire = _stream(random.Random(17), 3000)
    ref = O.decode_batch(wire)
    if kernel == "exact8192":
        ctx.set_exact(True)
    try:
        if kernel == "staged":
            g = ctx.decode_staged(wire, pieces=3, key_hash=True)
        else:
            g = ctx.decode_batch(wire, key_hash=True)
    finally:
        ctx.set_exact(False)
    n = len(ref["type"])
    g = {k: (v[:n] if hasattr(v, "shape") else v) for k, v in g.items()}
    base = dict(g)
    base["flags"] = g["flags"] & 0x0F
    assert_same(base, ref, kernel)
    checked = 0
    for k, h, fl in _expect(wire, ref):
        assert int(g["key_hash"][k]) == h, (kernel, k)
        assert int(g["flags"][k]) & 0x30 == fl, (kernel, k, int(g["flags"][k]), fl)
        checked += 1
    assert checked > 2500


def test_key_post_off_by_default(ctx):
    """Without a key_hash column nothing is computed: flags carry only the codec bits."""
    wire = _stream(random.Random(3), 500)
    g = ctx.decode_batch(wire)
    ch = (g["type"] & 0x3F) == 1  # (blob rows' Change columns are unspecified)
    assert int(np.max(g["flags"][ch])) < 0x10


def _key_text(wire, r, rows):
    """The oracle's ASCII keys of the Change rows end to end, and each row's position (as the
    addon's key text: rows whose key is ASCII and whose Change is well formed)."""
    kp, parts, tot = np.zeros(rows, np.uint32), [], 0
    for k in range(rows):
        kp[k] = tot
        if k >= r["nframes"] or r["type"][k] & 0x3F != 1 or r["flags"][k] & 4:
            continue
        po = int(r["payload_off"][k])
        key = wire[po + int(r["key_off"][k]):po + int(r["key_off"][k]) + int(r["key_len"][k])]
        if key.isascii():
            parts.append(key)
            tot += len(key)
    return kp, b"".join(parts)


@pytest.mark.parametrize("chunked", [False, True])
def test_fetch_keys_builds_the_key_text_on_the_device(ctx, chunked):
    """drp_decode_fetch_keys (the N-API addon's key text): every ASCII key end to end, built on
    the device from the staged batch, equals the oracle's; positions per row too."""
    from _gpu import drp_amd
    wire = _stream(random.Random(23), 4000)
    r = O.decode_batch(wire)
    arg = [wire[i:i + 65536] for i in range(0, len(wire), 65536)] if chunked else wire
    ctx.set_blob_skip(drp_amd.BLOB_SKIP_OFF)  # (one piece: the whole batch stays on the device)
    try:
        o = ctx.decode_staged(arg, keys=True)
        assert o["nframes"] == r["nframes"]
        kp, text = _key_text(wire, r, o["nframes"])
        assert o["key_text"] == text
        np.testing.assert_array_equal(o["kp"], kp)
        ctx.set_blob_skip(drp_amd.BLOB_SKIP_ALWAYS)  # pieces: the caller builds the text on the host
        o = ctx.decode_staged(arg, keys=True)
        assert o["nframes"] == r["nframes"] and (o["key_text"] is None or o["key_text"] == text)
    finally:
        ctx.set_blob_skip(drp_amd.BLOB_SKIP_AUTO)
