"""GPU: the two emit kernels (drp_decode_spec.hip). emit_tiles<true> decodes Change payloads in
decode_change_fast's shapes (one-byte field tags, varints of 1..5 bytes) and lists any tile with
another shape; emit_tiles<false> re-emits those tiles with the general decoder. Streams here mix
both shapes inside the same tiles (and dense tiles past the 512-frame list), so every tile kind
goes through one of the two paths; results must equal the oracle's (protocol-buffers@2 decoding
as restated in oracle/; these shapes are parity-pinned by the oracle only)."""
import random

import pytest

import _oracle as O
import _streams as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from _gpu import drp_amd
    c = drp_amd.Ctx(0)
    yield c
    c.close()


def _odd_payload(rng):
    """A Change payload outside the fast shapes: wide varints, a two-byte (non-minimal) tag,
    non-minimal lengths, unknown fields of each wire type, a repeated field, or a missing one."""
    key = bytes(rng.choice(b"abcdefghij") for _ in range(rng.randint(1, 30)))
    kind = rng.randrange(7)
    if kind == 0:  # change/from/to past 2^35: 6..8-byte varints
        return S.change_payload(key, rng.randint(2**35, 2**53 - 1), rng.randint(0, 2**53 - 1), 7)
    if kind == 1:  # the key tag as a two-byte varint (0x92 0x00 = 0x12)
        p = S.change_payload(key, 1, 2, 3)
        return b"\x92\x00" + p[1:]
    if kind == 2:  # a non-minimal length varint for the key
        return b"\x12" + bytes([0x80 | len(key), 0x00]) + key + b"\x18\x01\x20\x02\x28\x03"
    if kind == 3:  # unknown fields (numbers 9..12) of wire types 0, 2, 5 and 1
        return (S.change_payload(key, 4, 5, 6) + b"\x48\x96\x01" + b"\x52\x03abc" + b"\x5d\x01\x02\x03\x04" +
                b"\x61" + bytes(8))
    if kind == 4:  # a repeated field (the last one wins)
        return S.change_payload(key, 1, 2, 3) + b"\x18\x09"
    if kind == 5:  # a required field missing: a payload error at this frame
        return b"\x12" + S.varint(len(key)) + key + b"\x18\x01\x20\x02"
    return S.change_payload(key, rng.randint(0, 2**32 - 1), 1, 2, value=rng.randbytes(rng.randint(0, 3000)))


def _mixed(seed, nframes, odd_p, small_p=0.0):
    rng = random.Random(seed)
    parts = []
    for i in range(nframes):
        r = rng.random()
        if r < odd_p:
            parts.append(S.frame(_odd_payload(rng)))
        elif r < odd_p + small_p:
            parts.append(S.frame(b"", 2) if rng.random() < 0.5 else S.varint(rng.randint(0, 5)) + b"\x00")
        else:
            key = b"%010d" % i
            parts.append(S.frame(S.change_payload(key, i % 100 + 1, i % 128, (i + 1) % 128, rng.randbytes(64))))
    return b"".join(parts)


@pytest.mark.parametrize("seed,odd_p,small_p", [(1, 0.002, 0.0), (2, 0.05, 0.0), (3, 0.5, 0.0), (4, 0.01, 0.6), (5, 0.01, 0.99)])
def test_fast_and_general_emit_mix(ctx, seed, odd_p, small_p):
    from _gpu import assert_same
    wire = _mixed(seed, 40000, odd_p, small_p)
    assert_same(ctx.decode_batch(wire), O.decode_batch(wire), f"mix {seed}/{odd_p}/{small_p}")
