"""Generate tests/golden/ref_framing.json by running the UNMODIFIED reference in place.

Runs /root/reference/{decode,encode}.js (required where they lie) under Node with the
restated dependency shims in oracle/ref_js/shims (varint@3, and a protocol-buffers@2 stand-in
whose Change.decode passes the payload bytes through), so every expectation below is what the
reference's own framing code produced: frame boundaries, change payload bytes, blob data,
chunk-edge reassembly, the type-0 / type>=3 / truncated-EOF behaviour, and the encoder's
header bytes and blob/change ordering. Codec parity (Change fields) is pinned separately by
tests/golden/change_codec.json (google.protobuf vectors).

This container only: the reference never travels; the GPU box replays the committed JSON.
    python tests/golden/make_ref_fixtures.py [--check]
"""
import argparse
import hashlib
import json
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _streams as S  # noqa: E402

RUN = os.path.join(ROOT, "oracle", "ref_js", "ref_run.js")
SHIMS = os.path.join(ROOT, "oracle", "ref_js", "shims")
OUT = os.path.join(HERE, "ref_framing.json")
BIG = 256  # hex longer than this is stored as length + sha256


def node(args, env_extra=None):
    env = dict(os.environ, NODE_PATH=SHIMS, NODE_NO_WARNINGS="1")
    env.update(env_extra or {})
    return json.loads(subprocess.check_output(["node", RUN] + args, env=env, text=True, timeout=600))


def digest_hex(h):
    if len(h) <= BIG:
        return {"hex": h}
    b = bytes.fromhex(h)
    return {"len": len(b), "sha256": hashlib.sha256(b).hexdigest()}


def norm(events):
    out = []
    for e in events:
        if e["t"] == "change":
            out.append(dict(t="change", **digest_hex(e["payload"])))
        elif e["t"] == "blob":
            out.append(dict(t="blob", ended=e["ended"], **digest_hex(e["data"])))
        else:
            out.append(e)
    return out


def ref_decode_multi(wire, patterns):
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(wire)
        path = f.name
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(patterns, f)
        ppath = f.name
    try:
        return [norm(e) for e in node(["decode-multi", path, ppath])]
    finally:
        os.unlink(path)
        os.unlink(ppath)


def decode_case(name, wire, patterns, every_split=False, recipe=None):
    """Events of the reference for each write pattern; all patterns must agree (the reference
    is chunk-invariant on these inputs), so one event list is stored."""
    pats = list(patterns)
    if every_split:
        pats += [[k, 0] for k in range(1, len(wire))]
    evs = ref_decode_multi(wire, pats)
    ev = evs[0]
    for p, e in zip(pats, evs):
        if e != ev:
            raise SystemExit(f"{name}: reference events differ between write patterns {pats[0]} and {p}")
    case = {"name": name, "writes": patterns, "every_split": every_split}
    if recipe is None:
        case["wire"] = wire.hex()
        case["events"] = ev
    else:  # large: the wire is regenerated from its recipe, the events pinned by a digest
        case["recipe"] = recipe
        case["wire_len"] = len(wire)
        case["wire_sha256"] = hashlib.sha256(wire).hexdigest()
        case["n_events"] = len(ev)
        case["events_sha256"] = events_digest(ev)
        case["events_head"], case["events_tail"] = ev[:4], ev[-4:]
    return case


def events_digest(ev):
    """sha256 of the canonical JSON of a normalised event list (tests/test_ref_fixtures.py)."""
    return hashlib.sha256(json.dumps(ev, sort_keys=True, separators=(",", ":")).encode()).hexdigest()


def ops_json(ops):
    out = []
    for o in ops:
        o = dict(o)
        if "value" in o and o["value"] is not None:
            o["value"] = o["value"].hex()
        if "writes" in o:
            o["writes"] = [w.hex() for w in o["writes"]]
        out.append(o)
    return out


def ref_encode(ops):
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(ops_json(ops), f)
        path = f.name
    try:
        return node(["encode", path])
    finally:
        os.unlink(path)


GOOD = bytes.fromhex("130112036b65791801200028013205") + b"hello"  # test/basic.js:21-27 frame
BLOB = S.frame(b"hello world", 2)


def encode_cases():
    ch = lambda k, c, f, t, v=None, s=None: dict(op="change", key=k, change=c, **{"from": f}, to=t,
                                                  **({"value": v} if v is not None else {}),
                                                  **({"subset": s} if s is not None else {}))
    blob = lambda data, ln=None: {"op": "blob", "len": ln or len(data), "writes": [data[:5], data[5:]]}
    return {
        # test/basic.js:5-30, :32-51, :86-126 call sequences
        "basic_change": [ch("key", 1, 0, 1, b"hello"), {"op": "finalize"}],
        "basic_blob": [blob(b"hello world"), {"op": "finalize"}],
        "basic_blob_then_change": [blob(b"hello world"), ch("key", 1, 0, 1, b"hello"), {"op": "finalize"}],
        # ordering: changes before a blob precede it; changes after an open blob wait for it;
        # two blobs serialise in creation order
        "interleave": [ch("a", 1, 2, 3), blob(b"0123456789"), ch("b", 4, 5, 6, b""), blob(b"xyz"),
                       ch("c", 7, 8, 9, b"v" * 200, "sub"), {"op": "finalize"}],
        # field widths: empty/absent value, subset, keys >= 128 B, numbers up to 2^53 - 1
        "widths": [ch("k" * 130, 2**32 - 1, 2**21, 127, bytes(range(256)) * 2),
                   ch("", 0, 0, 0, None, ""), ch("été", 2**53 - 1, 2**31, 2**31 - 1, b"\x00"),
                   {"op": "finalize"}],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true", help="regenerate and compare, do not write")
    args = ap.parse_args()
    cases = []
    small = [[0], [1], [2], [3], [7], [64], [65536]]
    cases.append(decode_case("basic_frames", GOOD + BLOB + GOOD, small, every_split=True))
    for seed in range(4):
        r = random.Random(100 + seed)
        w = S.random_stream(r, 30, blob_p=0.15, blob_max=200, zero_p=0.08, big_key_p=0.1,
                            subset_p=0.3, value_max=150)
        cases.append(decode_case(f"mixed_{seed}", w, small, every_split=True))
    # id 0: the frame's header is consumed and its declared length ignored (decode.js:146-149)
    cases.append(decode_case("type0", GOOD + bytes([0x05, 0x00]) + GOOD + bytes([0x81, 0x01, 0x00]) + BLOB,
                             small, every_split=True))
    # id >= 3: 'Protocol error, unknown type: N' after the earlier frames (decode.js:159-161)
    for t in (3, 7, 0x80, 0xFF):
        cases.append(decode_case(f"type_{t}", GOOD + BLOB + bytes([0x03, t, 0x61, 0x62]) + GOOD, small,
                                 every_split=True))
    # truncated final frames are dropped silently (partial blobs are delivered as far as they go)
    for nm, tail in [("hdr", bytes([0x85])), ("hdr2", bytes([0x85, 0x80])), ("change", GOOD[:9]),
                     ("change_hdr_only", GOOD[:2]), ("blob", bytes([101, 2]) + bytes(range(40)))]:
        cases.append(decode_case(f"truncated_{nm}", GOOD + BLOB + tail, small, every_split=True))
    # a blob header split at every byte offset around a 64 KiB write edge (C3)
    for j in range(7):
        w = S.c3_edge_stream(j)
        cases.append(decode_case(f"c3_edge_{j}", w, [[65536], [65536, 1], [4096]],
                                 recipe={"fn": "c3_edge_stream", "args": [j]}))
    # a larger mixed stream in 64 KiB writes
    w = S.random_stream_seeded(2024, 3000)
    cases.append(decode_case("mixed_large", w, [[65536], [1000], [65536, 17]],
                             recipe={"fn": "random_stream_seeded", "args": [2024, 3000]}))

    enc = {}
    for name, ops in encode_cases().items():
        r = ref_encode(ops)
        enc[name] = {"ops": ops_json(ops), "wire": r["wire"], "changes": r["changes"], "blobs": r["blobs"],
                     "bytes": r["bytes"]}
    c1 = ref_encode(S.c1_ops())
    wire = bytes.fromhex(c1["wire"])
    enc["c1"] = {"recipe": {"fn": "c1_ops", "args": []}, "wire_len": len(wire),
                 "wire_sha256": hashlib.sha256(wire).hexdigest(), "changes": c1["changes"],
                 "blobs": c1["blobs"], "bytes": c1["bytes"], "drains": c1["drains"]}
    # and the reference decoder's view of the C1 wire
    cases.append(decode_case("c1_wire", wire, [[65536], [1000]], recipe={"fn": "c1_wire_ref", "args": []}))

    doc = {"generated_by": "tests/golden/make_ref_fixtures.py (reference decode.js/encode.js required in "
                           "place, node " + subprocess.check_output(["node", "--version"], text=True).strip()
                           + ", shims oracle/ref_js/shims, codec passthrough)",
           "decode": cases, "encode": enc}
    text = json.dumps(doc, indent=None, sort_keys=True, separators=(",", ":")) + "\n"
    if args.check:
        old = open(OUT).read()
        print("identical" if old == text else "DIFFERENT")
        sys.exit(0 if old == text else 1)
    with open(OUT, "w") as f:
        f.write(text)
    print(f"wrote {OUT}: {len(cases)} decode cases, {len(enc)} encode cases, {len(text)} bytes")


if __name__ == "__main__":
    main()
