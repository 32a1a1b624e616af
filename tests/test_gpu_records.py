"""GPU parity of claims_fast's per-frame records and the record emission (fast_records ->
verify_lite's tile_recok -> emit_recs, drp_decode_spec.hip) against the oracle: contexts opened
with DRP_CREC=1 take the record path for every tile whose frames are in the record's shape, and
the wire-reading emission for the others (subsets, wide numbers, blob-heavy or cut tiles), so
the rows must equal the oracle's whatever the mix."""
import os
import random

import numpy as np
import pytest

import _oracle as O
import _streams as S

pytestmark = pytest.mark.gpu


def rec_ctx(on=True):
    from _gpu import drp_amd
    keep = os.environ.get("DRP_CREC")
    os.environ["DRP_CREC"] = "1" if on else "0"
    try:
        return drp_amd.Ctx(0)
    finally:
        if keep is None:
            os.environ.pop("DRP_CREC", None)
        else:
            os.environ["DRP_CREC"] = keep


@pytest.fixture(scope="module")
def ctx():
    c = rec_ctx()
    c.set_blob_skip(0)
    yield c
    c.close()


@pytest.mark.parametrize("shape", ["c2", "c2_wide", "c3", "c5", "random", "shadow"])
def test_record_path_rows(ctx, shape):
    from _gpu import assert_same
    rng = random.Random(91)
    wire = {"c2": lambda: S.c2_stream(400_000, seed=12).tobytes(),
            # numbers of 2..5 bytes: the general field parse of the record decode
            "c2_wide": lambda: b"".join(S.frame(S.change_payload(b"key%07d" % i, 1000 + i * 37, i * 7919, 2 ** 31 + i,
                                                                 value=bytes(rng.randrange(256) for _ in range(40))))
                                        for i in range(30000)),
            "c3": lambda: S.c3_stream(rng, 3, frames_per_unit=1000),
            "c5": lambda: S.c5_stream(rng, 3000),
            "random": lambda: S.random_stream(rng, 40_000),
            "shadow": lambda: S.shadow_stream(300, period=8192, change_every=3)}[shape]()
    assert_same(ctx.decode_batch(wire), O.decode_batch(wire, chunk=65536), shape)


def test_record_path_on_device_c2():
    """A 4M-frame C2 stream decoded on the device with and without records: every column equal."""
    import ctypes as C
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from _gpu import drp_amd
    dev = torch.device("cuda", 0)
    n = 4_000_000
    wire = bench.c2_on_device(n, seed=21, dev=dev)
    so = torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev)
    got = []
    for on in (True, False):
        c = rec_ctx(on)
        try:
            outs = bench.alloc_outputs(n + 64, dev)
            res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
            c.decode_device(wire, so, None, outs, n + 64, res)
            torch.cuda.synchronize()
            t = c.timing()
            assert t.spec_repairs == 0 and t.strict_reruns == 0
            got.append({k: v[:n].cpu().numpy() for k, v in outs.items()})
        finally:
            c.close()
    for k in got[0]:
        np.testing.assert_array_equal(got[0][k], got[1][k], err_msg=k)
    assert int(got[0]["type"].min()) == 1 and int(got[0]["change"][12345]) == (12345 % 100) + 1
