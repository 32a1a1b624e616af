"""Helpers for GPU tests: load the libdrp binding (never a fallback)."""
import os
import sys

import torch  # noqa: E402

# torch's HIP runtime initialises before libdrp's (the order bench.py uses): a process that
# loads libdrp first then fails torch's lazy device init ("no ROCm-capable device")
if torch.cuda.is_available():
    torch.cuda.init()

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dat-replication-protocol_amd", "python"))
import drp_amd  # noqa: E402,F401

import numpy as np  # noqa: E402

import _oracle as O  # noqa: E402

CMP_KEYS = ["payload_off", "payload_len", "type"]
COL_KEYS = O.COLS32 + O.COLS64 + ["flags"]


def assert_same(g, r, label=""):
    """Bit-exact comparison of a libdrp decode with the oracle."""
    for k in ["nframes", "err_code", "err_detail", "consumed", "tail", "blob_remaining"]:
        assert g[k] == r[k], (label, k, g[k], r[k])
    if r["err_code"]:
        assert g["err_frame"] == r["err_frame"], (label, "err_frame", g["err_frame"], r["err_frame"])
    n = len(r["type"])
    assert len(g["type"]) == n, (label, "rows", len(g["type"]), n)
    for k in CMP_KEYS:
        np.testing.assert_array_equal(g[k], r[k], err_msg=f"{label}:{k}")
    ch = (r["type"] & 0x3F) == 1
    for k in COL_KEYS:
        np.testing.assert_array_equal(g[k][ch], r[k][ch], err_msg=f"{label}:{k}")


def stream_decode(ctx, wire, writes):
    """Feed `wire` to libdrp in the cycled write sizes `writes` (0 = the rest) the way the JS
    Decoder does (dat-replication-protocol_amd/decode.js): an incomplete header / change payload
    is carried into the next batch, an open blob continues via blob_remaining. Returns the
    delivered frames as dicts with absolute offsets, the counters and the error (or None)."""
    carry, brem, pos, k, base = b"", 0, 0, 0, 0
    frames, err = [], None
    while pos < len(wire):
        n = writes[k % len(writes)] or len(wire)
        k += 1
        chunk = wire[pos:pos + n]
        batch = carry + chunk
        base = pos - len(carry)
        pos += len(chunk)
        g = ctx.decode_batch(batch, blob_remaining=brem)
        for i in range(g["nframes"]):
            f = {"type": int(g["type"][i]), "off": base + int(g["payload_off"][i]),
                 "len": int(g["payload_len"][i]), "batch_end": base + len(batch)}
            if f["type"] & 0x3F == 1:
                f.update({c: int(g[c][i]) for c in COL_KEYS})
            frames.append(f)
        if g["err_code"]:
            err = (g["err_code"], g["err_detail"])
            break
        carry = batch[g["consumed"]:] if g["tail"] in (1, 2) else b""
        brem = g["blob_remaining"]
    return frames, err


def stream_events(ctx, wire, writes):
    """Reference-style events (tests/test_ref_fixtures.events_from_table format) of a streamed
    libdrp decode: change payloads, blobs assembled across batches, then error or finish. Also
    checks every change frame's columns against the oracle codec on its payload."""
    from test_ref_fixtures import MESSAGES, _digest_hex
    frames, err = stream_decode(ctx, wire, writes)
    ev, changes, blobs, cur = [], 0, 0, None
    for f in frames:
        if f["type"] & 0x3F == 1:
            p = wire[f["off"]:f["off"] + f["len"]]
            c = O.change_decode(p)
            for col, v in [("key_off", c.key_off), ("key_len", c.key_len), ("subset_off", c.subset_off),
                           ("subset_len", c.subset_len), ("value_off", c.value_off),
                           ("value_len", c.value_len), ("change", c.change), ("from", c.from_),
                           ("to", c.to), ("flags", c.flags)]:
                assert f[col] == v, (col, f[col], v)
            ev.append(dict(t="change", **_digest_hex(p)))
            changes += 1
            continue
        if not f["type"] & 0x40:  # a new blob (not the continuation of an open one)
            cur = {"data": bytearray(), "ended": False}
            ev.append(cur)
            blobs += 1
        cur["data"] += wire[f["off"]:min(f["batch_end"], f["off"] + f["len"])]
        if not f["type"] & 0x80:
            cur["ended"] = True
    out = []
    for e in ev:
        out.append(e if "t" in e else dict(t="blob", ended=e["ended"], **_digest_hex(bytes(e["data"]))))
    if err:
        out.append({"t": "error", "message": MESSAGES[err[0]].format(err[1])})
    else:
        out.append({"t": "finish", "changes": changes, "blobs": blobs, "bytes": len(wire)})
    return out
