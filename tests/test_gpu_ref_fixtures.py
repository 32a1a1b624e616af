"""GPU replay of tests/golden/ref_framing.json (events recorded from the unmodified reference
decode.js / encode.js): libdrp, fed write by write through the C ABI with the JS Decoder's
carry discipline, delivers exactly the reference's events for every recorded write pattern
(every two-write split of the small streams, 64 KiB edges splitting a blob header at each
offset), and every delivered Change's columns equal the oracle codec on its payload."""
import pytest

from test_ref_fixtures import FIX, case_wire, check_events, patterns

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from _gpu import drp_amd
    c = drp_amd.Ctx(0)
    yield c
    c.close()


@pytest.mark.parametrize("name", [c["name"] for c in FIX["decode"]])
def test_libdrp_replays_reference_decode(ctx, name):
    from _gpu import stream_events
    c = next(c for c in FIX["decode"] if c["name"] == name)
    wire = case_wire(c)
    stride = 1 if len(wire) <= 400 else 11  # every split point of the small streams
    for p in patterns(c, wire, every_split_stride=stride):
        check_events(c, stream_events(ctx, wire, p))
