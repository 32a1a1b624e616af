"""Generate tests/golden/ref_throws.json: how the reference surfaces a Change its codec rejects.

Runs the UNMODIFIED reference (/root/reference/decode.js, required in place under Node with the
restated dependency shims of oracle/ref_js/shims; DRP_REF_CODEC=strict makes the protocol-buffers
shim throw Error('Decoded message is not valid') for a payload missing a required field, as the
generated decoder does) through tests/js/throw_driver.js: a few Change frames, one without its
`to` field, more Change frames; every handler acknowledges on a later turn; writes issued at once
('burst') or each from the previous write's callback ('paced'). The log records the deliveries,
acknowledgements, write callbacks, and where the exception surfaced: out of write() (throw<k>),
out of a callback the stream ran (uncaught), or as an event. tests/test_js_api.py replays the
cases through this package's Decoder.

This container only: the reference never travels; the GPU box reads the committed JSON.
    python tests/golden/make_throw_fixtures.py
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _streams as S  # noqa: E402

RUN = os.path.join(ROOT, "oracle", "ref_js", "ref_run.js")
SHIMS = os.path.join(ROOT, "oracle", "ref_js", "shims")
OUT = os.path.join(HERE, "ref_throws.json")


def wire_and_cut():
    good = [S.frame(S.change_payload(b"key%07d" % i, i + 1, i, i + 1, value=b"v" * 20)) for i in range(6)]
    bad = S.frame(b"\x12\x03bad\x18\x01\x20\x02")  # key, change, from; no `to` (schema.proto:5, required)
    return b"".join(good[:3]) + bad + b"".join(good[3:]), sum(len(g) for g in good[:3])


def cases():
    wire, P = wire_and_cut()
    out = []
    for name, sizes in [("one_write", [len(wire)]), ("writes_40", [40]), ("bad_starts_write_1", [P, 100]),
                        ("bad_inside_write_1", [P + 5, 100]), ("bad_ends_write_0", [P + 8, 100])]:
        for pattern in ("burst", "paced"):
            out.append((name + "_" + pattern, wire, sizes, pattern))
    return out


def main():
    res = []
    for name, wire, sizes, pattern in cases():
        with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
            f.write(wire)
            path = f.name
        try:
            env = dict(os.environ, NODE_PATH=SHIMS, NODE_NO_WARNINGS="1", DRP_REF_CODEC="strict")
            log = json.loads(subprocess.check_output(["node", RUN, "throws", path, ",".join(map(str, sizes)), pattern],
                                                     env=env, text=True, timeout=120))
        finally:
            os.unlink(path)
        res.append({"name": name, "wire": wire.hex(), "sizes": sizes, "pattern": pattern, "log": log})
        print(name, log[-3:])
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_throw_fixtures.py", "cases": res}, f)


if __name__ == "__main__":
    main()
