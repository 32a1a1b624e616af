"""GPU: the measurement modes leave the decode unchanged. With DRP_STATS=1 (kernel counters) a
decode that also takes the density sample and the per-frame records clears nine regions in its
prologue; the decode must still equal the oracle (decode.js:144-262) and the stats-free run."""
import random

import pytest

import _oracle as O
import _streams as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stats", ["0", "1"])
def test_stats_mode_decodes_as_the_oracle(monkeypatch, stats):
    from _gpu import assert_same, drp_amd
    if stats == "1":
        monkeypatch.setenv("DRP_STATS", "1")
    monkeypatch.setenv("DRP_WALK_MIN", "512")  # (the density sample and the hop walkers at this size)
    wire = S.c3_stream(random.Random(41), 12, frames_per_unit=1000, blob_len=300000)
    ref = O.decode_batch(wire, cap=12 * 1001 + 16)
    c = drp_amd.Ctx(0)
    c.set_blob_skip(drp_amd.BLOB_SKIP_OFF)  # (one whole-batch decode of 570 tiles)
    try:
        for k in range(2):
            g = c.decode_batch(wire, cap=12 * 1001 + 16)
            assert_same(g, ref, f"DRP_STATS={stats} #{k}")
    finally:
        c.close()
