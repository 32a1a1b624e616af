"""Generate tests/golden/ref_acks.json: the reference's write-acknowledgement order.

Runs the UNMODIFIED reference (/root/reference/decode.js, required in place under Node with
the restated dependency shims of oracle/ref_js/shims) through tests/js/ack_driver.js on small
seeded streams: every change and blob handler acknowledges on a later turn, writes are issued
at once ('burst', the stream buffers them) or each from the previous write's callback ('paced'),
and the log records how write callbacks interleave with the handlers (decode.js:89-99,
144-169). tests/test_js_api.py replays the same cases through this package's Decoder.

This container only: the reference never travels; the GPU box reads the committed JSON.
    python tests/golden/make_ack_fixtures.py
"""
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
OUT = os.path.join(HERE, "ref_acks.json")


def wire_for(seed, n):
    """Change frames of 60..90 bytes and blobs of <= 40 payload bytes: with writes of >= 100
    bytes every write completes a frame, so every write callback follows an acknowledgement."""
    rng = random.Random(seed)
    out = b""
    for i in range(n):
        if rng.random() < 0.15:
            out += S.frame(bytes(rng.randrange(256) for _ in range(rng.randrange(0, 41))), typ=2)
        else:
            key = ("k%06d" % rng.randrange(10 ** 6)).encode()
            value = bytes(rng.randrange(256) for _ in range(rng.randrange(30, 56)))
            out += S.frame(S.change_payload(key, rng.randrange(1, 1000), rng.randrange(128), rng.randrange(128), value))
    return out


CASES = [("burst_100", 1, 300, [100], "burst"), ("burst_mixed", 2, 400, [100, 173, 256, 1000], "burst"),
         ("burst_big", 3, 500, [4096], "burst"), ("paced_100", 4, 200, [100, 131], "paced"),
         ("paced_big", 5, 300, [2048, 700], "paced")]


def error_cases():
    """Protocol errors whose header straddles two writes: the reference raises
    'unknown type' in the write that holds the type byte (decode.js:144-169, 251-262), after the
    write before it has been acknowledged. A 2-byte length varint split after its first byte, and
    the type byte alone at the start of the next write; plus the same header inside one write."""
    prefix = wire_for(6, 30)
    bad = bytes([0xC8, 0x01, 0x07]) + b"junk" * 5
    wire = prefix + bad
    P = len(prefix)
    out = []
    for name, sizes in [("err_split_varint", [P + 1, 100]), ("err_split_type", [P + 2, 100]),
                        ("err_one_write", [P + 3, 100]), ("err_small_writes", [97, 13])]:
        for pattern in ("burst", "paced"):
            out.append((name + "_" + pattern, wire, sizes, pattern))
    return out


def main():
    cases = []
    todo = [(name, wire_for(seed, n), sizes, pattern) for name, seed, n, sizes, pattern in CASES] + error_cases()
    for name, wire, sizes, pattern in todo:
        with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
            f.write(wire)
            path = f.name
        try:
            env = dict(os.environ, NODE_PATH=SHIMS, NODE_NO_WARNINGS="1")
            log = json.loads(subprocess.check_output(["node", RUN, "acks", path, ",".join(map(str, sizes)), pattern],
                                                     env=env, text=True, timeout=300))
        finally:
            os.unlink(path)
        cases.append({"name": name, "wire": wire.hex(), "sizes": sizes, "pattern": pattern, "log": log})
        print(name, len(wire), "bytes,", len(log), "events")
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_ack_fixtures.py", "cases": cases}, f)


if __name__ == "__main__":
    main()
