"""GPU parity of the hop walkers (drp_walk.hip, the claims kernel of large sparse batches) against
the oracle. Every context here forces the walkers for batches of any size (DRP_CLAIMS=hop,
read by drp_open), so a test's small input runs them with one tile per region; the default
path takes them from DRP_WALK_MIN tiles on when frames average more than 512 bytes
(test_gpu_configs.py's full-size C5).

The walkers only predict: verify_lite / verify_counts prove every claim on the exact chain, so a
wrong prediction costs repair passes, never a wrong row. The parity tests below compare rows;
the prediction tests count the repairs on the shapes the bench runs.
"""
import ctypes as C
import json
import os
import random

import numpy as np
import pytest

import _oracle as O
import _streams as S

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# the claims form under test (DRP_CLAIMS): "hop" (the hop walkers) or "fast" (claims_fast)
WALKERS = os.environ.get("DRP_TEST_WALKERS", "hop")


def walk_ctx(**env):
    from _gpu import drp_amd
    keep = {k: os.environ.get(k) for k in ["DRP_CLAIMS", "DRP_WALK_MIN", *env]}
    os.environ.update({"DRP_CLAIMS": WALKERS, "DRP_WALK_MIN": "0", **env})
    try:
        return drp_amd.Ctx(0)
    finally:
        for k, v in keep.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def ctx():
    c = walk_ctx()
    c.set_blob_skip(0)  # (whole batches: the walkers see every tile of the input)
    yield c
    c.close()


def test_golden_streams(ctx):
    from _gpu import assert_same
    for v in json.load(open(os.path.join(GOLD, "streams.json")))["vectors"]:
        wire = bytes.fromhex(v["wire"])
        assert_same(ctx.decode_batch(wire), O.decode_batch(wire), v["source"])


@pytest.mark.parametrize("seed", range(6))
def test_random_streams(ctx, seed):
    """Blobs up to 20 KB, type-0 frames, long keys, subsets and 8-byte numbers, cut anywhere."""
    from _gpu import assert_same
    rng = random.Random(seed)
    wire = S.random_stream(rng, 6000, blob_p=0.08, blob_max=20000)
    wire = wire[:rng.randint(len(wire) // 2, len(wire))]
    assert_same(ctx.decode_batch(wire), O.decode_batch(wire), f"seed{seed}")


@pytest.mark.parametrize("seed", range(3))
def test_errors_and_tails(ctx, seed):
    """A protocol or policy error mid-stream ends the chain the walker follows: its claims past
    the error are predictions that the exact walk then corrects."""
    from _gpu import assert_same
    rng = random.Random(200 + seed)
    base = S.random_stream(rng, 3000)
    for b in [b"\x03\x07ab", b"\x00\x01", b"\x80" * 10 + b"\x01\x01", b"\x01\x01", S.frame(b"\x12\x05k")]:
        cut = O.decode_batch(base[:rng.randint(0, len(base))])["consumed"]
        wire = base[:cut] + b + base
        assert_same(ctx.decode_batch(wire), O.decode_batch(wire), repr(b))


@pytest.mark.parametrize("shape", ["c2", "c3", "c5", "shadow"])
def test_shapes(ctx, shape):
    from _gpu import assert_same
    rng = random.Random(31)
    wire = {"c2": lambda: S.c2_stream(300_000, seed=8).tobytes(),
            "c3": lambda: S.c3_stream(rng, 3, frames_per_unit=1000),
            "c5": lambda: S.c5_stream(rng, 3000),
            "shadow": lambda: S.shadow_stream(300, period=8192, change_every=3)}[shape]()
    assert_same(ctx.decode_batch(wire), O.decode_batch(wire, chunk=65536), shape)


@pytest.mark.parametrize("shape", ["c2", "c5", "random"])
def test_predictions_hold(shape):
    """On the bench's shapes the walkers' claims are the exact chain's: no repair pass, and the
    records-only check relists only the regions' first tiles whose sync is not the chain's first
    frame (a few per mille; a few per cent on random streams with long blobs)."""
    from _gpu import assert_same
    rng = random.Random(77)
    wire = {"c2": lambda: S.c2_stream(400_000, seed=9).tobytes(),
            "c5": lambda: S.c5_stream(rng, 8000),
            "random": lambda: S.random_stream(rng, 60_000)}[shape]()
    c = walk_ctx()
    try:
        c.set_blob_skip(0)
        g = c.decode_batch(wire)
        t = c.timing()
    finally:
        c.close()
    ntiles = len(wire) // 8192 + 1
    print(f"{shape}: {ntiles} tiles, repairs {t.spec_repairs}, relisted {t.verify_relisted}")
    assert_same(g, O.decode_batch(wire, chunk=65536), shape)
    assert t.spec_repairs == 0 and t.strict_reruns == 0 and t.seg_repairs == 0, (t.spec_repairs, t.seg_repairs)
    # (random streams: a region starting in a blob whose header is more than SY_MERGE bytes
    # before the first shaped Change is entered at that Change, and its first tile relisted)
    assert t.verify_relisted <= ntiles // (20 if shape == "random" else 50) + 8, t.verify_relisted


def test_cut_streams():
    """~150 streams cut at arbitrary bytes (edge tiles to spec_claims, interior tiles to the
    walkers, a region never crossing a stream), decoded on the device: rows equal the oracle's."""
    import torch
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from _gpu import drp_amd
    dev = torch.device("cuda", 0)
    rng = random.Random(505)
    wire = S.random_stream(rng, 40_000, blob_p=0.02, blob_max=30000)
    whole = O.decode_batch(wire)
    ends = whole["payload_off"].astype(np.int64) + whole["payload_len"].astype(np.int64)
    starts = np.concatenate([[0], ends[:-1]])
    cuts = sorted(set([0] + rng.sample(range(1, len(wire)), 149) + [len(wire)]))
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
    c = walk_ctx()
    try:
        c.decode_device(w, so, en, outs, cap, res)
        torch.cuda.synchronize()
        t = c.timing()
    finally:
        c.close()
    assert t.strict_reruns == 0
    rs = np.frombuffer(res.cpu().numpy().tobytes(), np.uint8).reshape(ns, -1)
    row = 0
    for s in range(ns):
        a, b = cuts[s] + entry[s], cuts[s + 1]
        ref = O.decode_batch(wire[a:b])
        r = drp_amd.StreamResult.from_buffer_copy(rs[s].tobytes())
        assert (r.frames, r.err_code, r.tail_kind) == (ref["nframes"], ref["err_code"], ref["tail"]), s
        n = ref["nframes"]
        off = outs["payload_off"][row:row + n].cpu().numpy() - cuts[s]
        np.testing.assert_array_equal(off - entry[s], ref["payload_off"].astype(np.int64), err_msg=f"stream {s}")
        np.testing.assert_array_equal(outs["payload_len"][row:row + n].cpu().numpy().astype(np.uint32),
                                      ref["payload_len"], err_msg=f"stream {s}")
        row += n
