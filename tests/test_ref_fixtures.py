"""Replay of tests/golden/ref_framing.json: framing behaviour recorded from the UNMODIFIED
reference (decode.js / encode.js required in place by tests/golden/make_ref_fixtures.py).

CPU: the oracle (oracle/drp_oracle.c) reproduces every recorded decode (for every write
pattern the fixture was recorded with, including every two-write split) and, assembled in the
reference's blob/change order, every recorded encoder output. The GPU replays live in
tests/test_gpu_ref_fixtures.py."""
import hashlib
import json
import os

import numpy as np
import pytest

import _oracle as O
import _streams as S

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "ref_framing.json")))
BIG = 256
MESSAGES = {1: "Protocol error, unknown type: {}"}


def _digest_hex(b):
    h = b.hex()
    if len(h) <= BIG:
        return {"hex": h}
    return {"len": len(b), "sha256": hashlib.sha256(b).hexdigest()}


def events_digest(ev):
    return hashlib.sha256(json.dumps(ev, sort_keys=True, separators=(",", ":")).encode()).hexdigest()


def events_from_table(wire, r, nbytes=None):
    """Normalised reference-style events from a decoded frame table (oracle or libdrp):
    change -> payload bytes, blob -> delivered bytes (+ ended), then error or finish."""
    ev = []
    n = len(wire)
    for k in range(r["nframes"]):
        off, ln, t = int(r["payload_off"][k]), int(r["payload_len"][k]), int(r["type"][k])
        if t & 0x3F == 1:
            ev.append(dict(t="change", **_digest_hex(wire[off:off + ln])))
        else:
            ev.append(dict(t="blob", ended=not (t & 0x80), **_digest_hex(wire[off:min(n, off + ln)])))
    if r["err_code"]:
        ev.append({"t": "error", "message": MESSAGES[r["err_code"]].format(r["err_detail"])})
    else:
        ev.append({"t": "finish", "changes": r["changes"], "blobs": r["blobs"],
                   "bytes": n if nbytes is None else nbytes})
    return ev


def c1_wire_oracle():
    return reference_order_encode(S.c1_ops())


def case_wire(c):
    if "wire" in c:
        return bytes.fromhex(c["wire"])
    fn, args = c["recipe"]["fn"], c["recipe"]["args"]
    w = c1_wire_oracle() if fn == "c1_wire_ref" else getattr(S, fn)(*args)
    assert len(w) == c["wire_len"] and hashlib.sha256(w).hexdigest() == c["wire_sha256"], c["name"]
    return w


def check_events(c, ev):
    if "events" in c:
        assert ev == c["events"], c["name"]
    else:
        assert len(ev) == c["n_events"], (c["name"], len(ev), c["n_events"])
        assert ev[:4] == c["events_head"] and ev[-4:] == c["events_tail"], c["name"]
        assert events_digest(ev) == c["events_sha256"], c["name"]


def patterns(c, wire, every_split_stride=1):
    pats = [list(p) for p in c["writes"]]
    if c["every_split"]:
        pats += [[k, 0] for k in range(1, len(wire), every_split_stride)]
    return pats


@pytest.mark.parametrize("name", [c["name"] for c in FIX["decode"]])
def test_oracle_replays_reference_decode(name):
    c = next(c for c in FIX["decode"] if c["name"] == name)
    wire = case_wire(c)
    for p in patterns(c, wire):
        r = O.decode_batch(wire, writes=p)
        check_events(c, events_from_table(wire, r))


# ---- encoder: reference order of a synchronous call sequence (encode.js:77-117) -----------
def reference_order(ops):
    """Frames in the order encode.js emits them for ops issued in one tick: changes go out at
    once until the first blob is opened; blobs serialise in creation order; changes issued
    while a blob is open are queued and flushed after the last open blob finishes."""
    pre, blobs, queued, opened = [], [], [], False
    for o in ops:
        if o["op"] == "change":
            (queued if opened else pre).append(o)
        elif o["op"] == "blob":
            opened = True
            blobs.append(o)
    return pre + blobs + queued


def _val(x):
    return bytes.fromhex(x) if isinstance(x, str) else x


def encode_rows(rows):
    heap, cols = bytearray(), {k: [] for k in ["key_off", "key_len", "subset_off", "subset_len", "value_off",
                                               "value_len", "change", "from", "to", "flags"]}
    for o in rows:
        key = o["key"].encode()
        sub = o.get("subset")
        val = o.get("value")
        fl = 0
        cols["key_off"].append(len(heap)); cols["key_len"].append(len(key)); heap += key
        if sub is not None:
            sb = sub.encode()
            cols["subset_off"].append(len(heap)); cols["subset_len"].append(len(sb)); heap += sb; fl |= 1
        else:
            cols["subset_off"].append(0); cols["subset_len"].append(0)
        if val is not None:
            vb = _val(val)
            cols["value_off"].append(len(heap)); cols["value_len"].append(len(vb)); heap += vb; fl |= 2
        else:
            cols["value_off"].append(0); cols["value_len"].append(0)
        for k in ["change", "from", "to"]:
            cols[k].append(o[k])
        cols["flags"].append(fl)
    dt = {"key_len": np.uint32, "subset_len": np.uint32, "value_len": np.uint32, "flags": np.uint8}
    return bytes(heap), {k: np.array(v, dtype=dt.get(k, np.uint64)) for k, v in cols.items()}


def reference_order_encode(ops):
    out = bytearray()
    for o in reference_order(ops):
        if o["op"] == "change":
            heap, cols = encode_rows([o])
            out += O.encode_changes(heap, cols)
        else:
            out += S.varint(o["len"] + 1) + b"\x02" + b"".join(_val(w) for w in o["writes"])
    return bytes(out)


@pytest.mark.parametrize("name", sorted(FIX["encode"]))
def test_oracle_replays_reference_encode(name):
    c = FIX["encode"][name]
    if "recipe" in c:
        wire = reference_order_encode(S.c1_ops())
        assert len(wire) == c["wire_len"] and hashlib.sha256(wire).hexdigest() == c["wire_sha256"]
    else:
        assert reference_order_encode(c["ops"]).hex() == c["wire"]
        assert c["bytes"] == len(c["wire"]) // 2


def test_c1_reference_counters():
    c = FIX["encode"]["c1"]
    assert (c["changes"], c["blobs"], c["bytes"]) == (10000, 1, c["wire_len"])
