"""GPU parity on inputs built to reach the decode kernel's rare paths (drp_decode.hip):

- tiles with more live positions than the load-balanced parse holds (PCAP): every byte
  position of a run of 0x01/0x02 bytes can start a header, so the DP parses per lane;
- dense 2-byte frames (64 frames per lane): the lane walks and the emission loop at their
  maximum trip counts;
- an entry that is none of the keys Y_{t-1}: a blob longer than a tile lands in the middle of
  a later tile, so phase 2 walks that tile serially;
- mixtures of the above with ordinary Change frames, cut at arbitrary points.
Each is compared bit-exact with the oracle on both decode paths.
"""
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


def _blob(n, fill=None, rng=None):
    body = bytes([fill]) * n if fill is not None else rng.randbytes(n)
    return S.varint(n + 1) + b"\x02" + body


def _cases():
    rng = random.Random(5)
    c2 = S.c2_stream(400, seed=3).tobytes()
    dense = b"\x01\x02" * 20000                         # empty blobs: 2 B per frame, all live
    ones = b"\x01\x01" * 9000                           # empty Change payloads (missing fields)
    yield "dense_blobs", dense
    yield "dense_then_c2", dense + c2
    yield "c2_dense_c2", c2 + b"\x01\x02" * 6000 + c2
    yield "c2_then_empty_changes", c2 + ones  # a REQUIRED error after 400 frames
    yield "zero_blob_spans_tiles", c2 + _blob(20000, fill=0) + c2       # zero bytes: every position live
    yield "ones_blob_spans_tiles", c2 + _blob(30011, fill=1) + c2 + _blob(9000, fill=2) + c2
    yield "random_blob_lands_midtile", c2 + _blob(12345, rng=rng) + c2 + _blob(8191, rng=rng) + c2
    mix = b"".join([c2[:86 * 50], _blob(17000, fill=0), b"\x01\x02" * 3000, c2[:86 * 70],
                    _blob(5000, rng=rng), S.random_stream(rng, 300, blob_p=0.2, blob_max=9000)])
    yield "mix", mix
    yield "mix_cut", mix[:len(mix) - 777]


CASES = list(_cases())


@pytest.mark.parametrize("kernel", ["speculative", "exact4096", "exact8192"])
@pytest.mark.parametrize("name", [n for n, _ in CASES])
def test_adversarial(ctx, kernel, name):
    """The default path (speculate, repair, fall back) and the exact kernel at both of its
    tile sizes (the speculative kernels have one fixed 8 KiB tile)."""
    from _gpu import assert_same
    wire = dict(CASES)[name]
    if kernel != "speculative":
        ctx.set_exact(True)
        ctx.set_tile(int(kernel[5:]))
    try:
        assert_same(ctx.decode_batch(wire), O.decode_batch(wire), f"{name}/{kernel}")
    finally:
        ctx.set_tile(0)
        ctx.set_exact(False)
