"""CPU: pin the oracle (the decode.js / protocol-buffers@2 restatement) to the golden
fixtures — google.protobuf codec vectors and the /root/reference/test/basic.js known
answers — and check the restatement's chunk-split invariance."""
import json
import os
import random

import numpy as np
import pytest

import _oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)["vectors"]


CODEC = load("change_codec.json")
STREAMS = load("streams.json")


@pytest.mark.parametrize("i", range(len(CODEC)))
def test_change_decode_matches_protobuf(i):
    v = CODEC[i]
    p = bytes.fromhex(v["payload"])
    c = O.change_decode(p)
    assert c.err == 0, v["source"]
    assert p[c.key_off:c.key_off + c.key_len].hex() == v["key"]
    assert bool(c.flags & 1) == v["has_subset"]
    assert bool(c.flags & 2) == v["has_value"]
    if v["has_subset"]:
        assert p[c.subset_off:c.subset_off + c.subset_len].hex() == v["subset"]
    if v["has_value"]:
        assert p[c.value_off:c.value_off + c.value_len].hex() == v["value"]
    assert (c.change, c.from_, c.to) == (v["change"], v["from"], v["to"])


@pytest.mark.parametrize("i", [i for i, v in enumerate(CODEC) if v["canonical"]])
def test_change_encode_matches_protobuf(i):
    v = CODEC[i]
    subset = bytes.fromhex(v["subset"]) if v["has_subset"] else None
    value = bytes.fromhex(v["value"]) if v["has_value"] else None
    got = O.change_encode(subset, bytes.fromhex(v["key"]), v["change"], v["from"], v["to"], value)
    assert got.hex() == v["payload"], v["source"]


def check_stream(v, r, wire):
    exp = v["frames"]
    assert r["nframes"] == len(exp), v["source"]
    for k, f in enumerate(exp):
        assert r["type"][k] & 0x3F == f["type"]
        off, ln = int(r["payload_off"][k]), int(r["payload_len"][k])
        if f["type"] == 2:
            assert wire[off:off + ln].hex() == f["blob"]
        else:
            p = wire[off:off + ln]
            assert p[r["key_off"][k]:r["key_off"][k] + r["key_len"][k]].hex() == f["key"]
            assert (int(r["change"][k]), int(r["from"][k]), int(r["to"][k])) == \
                (f["change"], f["from"], f["to"])
            assert bool(r["flags"][k] & 2) == f["has_value"]
            assert bool(r["flags"][k] & 1) == f["has_subset"]
            if f["has_value"]:
                vo, vl = int(r["value_off"][k]), int(r["value_len"][k])
                assert p[vo:vo + vl].hex() == f["value"]
    assert r["err_code"] == v["err_code"]
    if v["err_code"]:
        assert r["err_frame"] == v["err_frame"]
        assert r["err_detail"] == v.get("err_detail", r["err_detail"])
    else:
        assert r["tail"] == v["tail"]
        assert r["consumed"] == v["consumed"]


@pytest.mark.parametrize("i", range(len(STREAMS)))
@pytest.mark.parametrize("chunk", [0, 1, 2, 3, 7, 64, 255])
def test_stream_known_answers(i, chunk):
    v = STREAMS[i]
    wire = bytes.fromhex(v["wire"])
    check_stream(v, O.decode_batch(wire, chunk=chunk), wire)


def random_stream(rng, nframes, blob_every=0, blob_max=300):
    """Wire bytes built from codec golden payloads + blob frames."""
    parts = []
    canon = [v for v in CODEC]
    for i in range(nframes):
        if blob_every and i % blob_every == blob_every - 1:
            b = rng.randbytes(rng.randint(1, blob_max))
            parts.append(bytes(_hdr(len(b), 2)) + b)
        else:
            p = bytes.fromhex(rng.choice(canon)["payload"])
            parts.append(bytes(_hdr(len(p), 1)) + p)
    return b"".join(parts)


def _hdr(plen, typ):
    out = bytearray()
    n = plen + 1
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    out.append(typ)
    return out


@pytest.mark.parametrize("seed", range(6))
def test_oracle_chunk_invariance(seed):
    """The restated decode.js delivers identical frames for every chunking."""
    rng = random.Random(seed)
    wire = random_stream(rng, 60, blob_every=7)
    cut = rng.randint(0, len(wire))
    wire = wire[:cut]  # random truncation exercises every tail kind
    ref = O.decode_batch(wire)
    for chunk in [1, 2, 3, 5, 17, 64, 1000]:
        r = O.decode_batch(wire, chunk=chunk)
        for k in ["nframes", "err_code", "consumed", "tail", "blob_remaining", "changes", "blobs"]:
            assert r[k] == ref[k], (k, chunk)
        for k in O.COLS32 + O.COLS64 + ["payload_off", "payload_len", "type", "flags"]:
            np.testing.assert_array_equal(r[k], ref[k])


def test_encode_decode_round_trip():
    rng = random.Random(7)
    heap = bytearray()
    cols = {k: [] for k in ["key_off", "key_len", "subset_off", "subset_len", "value_off",
                            "value_len", "change", "from", "to", "flags"]}
    for i in range(500):
        key = rng.randbytes(rng.randint(0, 200))
        val = rng.randbytes(rng.randint(0, 300))
        sub = rng.randbytes(rng.randint(0, 5))
        fl = (1 if rng.random() < 0.3 else 0) | (2 if rng.random() < 0.8 else 0)
        for name, b in [("key", key), ("value", val), ("subset", sub)]:
            cols[name + "_off"].append(len(heap))
            cols[name + "_len"].append(len(b))
            heap += b
        cols["change"].append(rng.randint(0, 2**53 - 1))
        cols["from"].append(rng.randint(0, 300))
        cols["to"].append(rng.randint(0, 2**32))
        cols["flags"].append(fl)
    dt = {"key_off": np.uint64, "subset_off": np.uint64, "value_off": np.uint64,
          "key_len": np.uint32, "subset_len": np.uint32, "value_len": np.uint32,
          "change": np.uint64, "from": np.uint64, "to": np.uint64, "flags": np.uint8}
    c = {k: np.array(v, dtype=dt[k]) for k, v in cols.items()}
    wire = O.encode_changes(bytes(heap), c)
    r = O.decode_batch(wire, chunk=4096)
    assert r["nframes"] == 500 and r["err_code"] == 0 and r["tail"] == 0
    for i in range(500):
        p = wire[int(r["payload_off"][i]):int(r["payload_off"][i]) + int(r["payload_len"][i])]
        ko = int(r["key_off"][i])
        assert p[ko:ko + int(r["key_len"][i])] == bytes(heap[c["key_off"][i]:c["key_off"][i] + c["key_len"][i]])
        assert int(r["change"][i]) == int(c["change"][i])
        assert int(r["flags"][i]) == int(c["flags"][i])


def test_policy_errors():
    good = bytes.fromhex(STREAMS[0]["wire"])
    # L = 0 on a change frame (policy DRP_ERR_LEN)
    r = O.decode_batch(good + b"\x00\x01" + good)
    assert (r["nframes"], r["err_code"], r["err_frame"]) == (1, 2, 1)
    # 11-byte header varint (policy DRP_ERR_VARINT)
    r = O.decode_batch(good + b"\x80" * 10 + b"\x01\x01")
    assert (r["nframes"], r["err_code"]) == (1, 3)
    # empty change payload: required fields missing (policy DRP_ERR_REQUIRED)
    r = O.decode_batch(good + b"\x01\x01" + good)
    assert (r["nframes"], r["err_code"], r["err_frame"]) == (1, 5, 1)
    # truncated field inside a complete frame (policy DRP_ERR_CHANGE)
    r = O.decode_batch(b"\x04\x01\x12\x05k")
    assert (r["nframes"], r["err_code"]) == (0, 4)
    # empty blob (L = 1) is fine
    r = O.decode_batch(b"\x01\x02" + good)
    assert r["nframes"] == 2 and r["type"][0] == 2 and r["payload_len"][0] == 0
