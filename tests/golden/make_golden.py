#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run once in the build container:  python tests/golden/make_golden.py

Sources of truth (nothing here imports or runs /root/reference, whose JS
dependencies varint@3 / protocol-buffers@2 are absent from the image):

* Change codec vectors: google.protobuf 7.35.1 — an independent implementation of
  the proto2 wire format — over a schema identical to
  /root/reference/messages/schema.proto:1-8 (Change{subset=1,key=2,change=3,from=4,
  to=5,value=6}). Serialisation writes fields in field-number order, which is also
  the protocol-buffers@2 order; parsing is last-wins with unknown fields skipped.
* Framing: README.md:63-71 (varint length | id byte | payload), with the length
  counting the id byte (encode.js:124-137 `varint.encode(len+1)`); varints are
  produced with google.protobuf's own varint encoder.
* Stream vectors: the inputs and expected outputs of /root/reference/test/basic.js
  (the four tape tests), transcribed as data.

Outputs: tests/golden/change_codec.json, tests/golden/streams.json
"""
import json
import os
import random

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
from google.protobuf.internal import encoder as pb_encoder

HERE = os.path.dirname(os.path.abspath(__file__))


def change_class():
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "drp_schema.proto"
    fdp.package = "drp"
    fdp.syntax = "proto2"
    m = fdp.message_type.add()
    m.name = "Change"
    F = descriptor_pb2.FieldDescriptorProto
    for name, num, typ, label in [
        ("subset", 1, F.TYPE_STRING, F.LABEL_OPTIONAL),
        ("key", 2, F.TYPE_STRING, F.LABEL_REQUIRED),
        ("change", 3, F.TYPE_UINT32, F.LABEL_REQUIRED),
        ("from", 4, F.TYPE_UINT32, F.LABEL_REQUIRED),
        ("to", 5, F.TYPE_UINT32, F.LABEL_REQUIRED),
        ("value", 6, F.TYPE_BYTES, F.LABEL_OPTIONAL),
    ]:
        f = m.field.add()
        f.name, f.number, f.type, f.label = name, num, typ, label
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("drp.Change"))


Change = change_class()


def varint(n):
    return pb_encoder._VarintBytes(n)


def make_msg(subset, key, change, frm, to, value):
    c = Change()
    if subset is not None:
        c.subset = subset
    c.key = key
    c.change = change
    setattr(c, "from", frm)
    c.to = to
    if value is not None:
        c.value = value
    return c


def fields_of(payload):
    """Decode with google.protobuf and return the expected column view."""
    c = Change()
    c.ParseFromString(payload)
    out = {
        "has_subset": c.HasField("subset"),
        "subset": c.subset.encode("utf-8").hex() if c.HasField("subset") else "",
        "key": c.key.encode("utf-8").hex(),
        "change": c.change,
        "from": getattr(c, "from"),
        "to": c.to,
        "has_value": c.HasField("value"),
        "value": c.value.hex() if c.HasField("value") else "",
    }
    return out


def rand_text(rng, n, alphabet="abcdefghijklmnopqrstuvwxyz0123456789"):
    return "".join(rng.choice(alphabet) for _ in range(n))


def codec_vectors():
    rng = random.Random(20140901)
    vecs = []
    # test/basic.js:21-27 input
    vecs.append(("test/basic.js:21-27", make_msg(None, "key", 1, 0, 1, b"hello")))
    # example.js / README usage shapes
    vecs.append(("README.md:28-34", make_msg(None, "some-row-key", 0, 0, 1, b"some binary value")))
    # presence corner cases
    vecs.append(("empty key", make_msg(None, "", 0, 0, 0, None)))
    vecs.append(("empty value present", make_msg(None, "k", 5, 6, 7, b"")))
    vecs.append(("empty subset present", make_msg("", "k", 5, 6, 7, b"v")))
    vecs.append(("subset present", make_msg("users", "k", 1, 2, 3, b"v")))
    vecs.append(("unicode key", make_msg("subé", "clé☃", 9, 8, 7, b"\x00\xff")))
    # varint width boundaries of the numbers (uint32 range: google.protobuf caps at 2^32-1)
    for v in [0, 1, 127, 128, 16383, 16384, 2097151, 2097152, 268435455, 268435456, 2**31 - 1,
              2**31, 2**32 - 1]:
        vecs.append((f"numbers {v}", make_msg(None, "n", v, v, v, b"x")))
    # length-varint boundaries of key / value
    for L in [0, 1, 126, 127, 128, 129, 255, 256, 16383, 16384]:
        vecs.append((f"key len {L}", make_msg(None, rand_text(rng, L), 1, 2, 3, b"v")))
        vecs.append((f"value len {L}", make_msg(None, "k", 1, 2, 3, rng.randbytes(L))))
    # random
    for i in range(200):
        subset = None if rng.random() < 0.6 else rand_text(rng, rng.randint(0, 20))
        value = None if rng.random() < 0.15 else rng.randbytes(rng.choice([0, 1, 5, 64, 200, 700]))
        key = rand_text(rng, rng.randint(0, 300))
        nums = [rng.choice([rng.randint(0, 127), rng.randint(0, 2**14), rng.randint(0, 2**32 - 1)])
                for _ in range(3)]
        vecs.append((f"random {i}", make_msg(subset, key, *nums, value)))
    out = []
    for src, msg in vecs:
        payload = msg.SerializeToString()
        out.append({"source": src, "payload": payload.hex(), "canonical": True, **fields_of(payload)})

    # Non-canonical payloads that a proto2 parser must accept; google.protobuf gives the
    # expected view (same semantics as the generated JS decoder for these cases:
    # last-wins duplicates, unknown fields skipped by wire type, overlong varints).
    def raw(*parts):
        return b"".join(parts)

    tag = lambda num, wt: varint((num << 3) | wt)
    s = lambda b: varint(len(b)) + b
    nc = [
        ("fields reversed", raw(tag(6, 2), s(b"val"), tag(5, 0), varint(3), tag(4, 0), varint(2),
                                tag(3, 0), varint(1), tag(2, 2), s(b"key"))),
        ("duplicate key last wins", raw(tag(2, 2), s(b"first"), tag(3, 0), varint(1), tag(4, 0),
                                        varint(2), tag(5, 0), varint(3), tag(2, 2), s(b"second"))),
        ("duplicate numbers last wins", raw(tag(2, 2), s(b"k"), tag(3, 0), varint(1), tag(3, 0),
                                            varint(99), tag(4, 0), varint(2), tag(5, 0), varint(3),
                                            tag(4, 0), varint(77))),
        ("unknown varint field", raw(tag(2, 2), s(b"k"), tag(7, 0), varint(123456), tag(3, 0),
                                     varint(1), tag(4, 0), varint(2), tag(5, 0), varint(3))),
        ("unknown fixed64 field", raw(tag(9, 1), b"\x01" * 8, tag(2, 2), s(b"k"), tag(3, 0),
                                      varint(1), tag(4, 0), varint(2), tag(5, 0), varint(3))),
        ("unknown fixed32 field", raw(tag(2, 2), s(b"k"), tag(3, 0), varint(1), tag(15, 5),
                                      b"\x02" * 4, tag(4, 0), varint(2), tag(5, 0), varint(3))),
        ("unknown bytes field", raw(tag(2, 2), s(b"k"), tag(3, 0), varint(1), tag(4, 0), varint(2),
                                    tag(100, 2), s(b"ignored" * 30), tag(5, 0), varint(3))),
        ("overlong varint number", raw(tag(2, 2), s(b"k"), tag(3, 0), b"\x81\x80\x80\x00",
                                       tag(4, 0), b"\x80\x00", tag(5, 0), b"\xff\xff\xff\xff\x0f")),
        ("overlong length varint", raw(tag(2, 2), b"\x83\x80\x00" + b"abc", tag(3, 0), varint(1),
                                       tag(4, 0), varint(2), tag(5, 0), varint(3))),
        ("duplicate value last wins", raw(tag(2, 2), s(b"k"), tag(3, 0), varint(1), tag(4, 0),
                                          varint(2), tag(5, 0), varint(3), tag(6, 2), s(b"a"),
                                          tag(6, 2), s(b"bb"))),
    ]
    for src, payload in nc:
        out.append({"source": src, "payload": payload.hex(), "canonical": False, **fields_of(payload)})
    return out


def frame(payload, typ=1):
    return varint(len(payload) + 1) + bytes([typ]) + payload


def stream_vectors():
    """Known answers of /root/reference/test/basic.js plus README framing examples."""
    basic = make_msg(None, "key", 1, 0, 1, b"hello").SerializeToString()
    expect_basic = {"type": 1, "key": b"key".hex(), "change": 1, "from": 0, "to": 1,
                    "has_value": True, "value": b"hello".hex(), "has_subset": False, "subset": ""}
    vecs = []
    # test/basic.js:5-30 encode + decode changes
    w = frame(basic)
    vecs.append({"source": "test/basic.js:5-30", "wire": w.hex(), "frames": [expect_basic],
                 "err_code": 0, "tail": 0, "consumed": len(w)})
    # test/basic.js:32-51 encode + decode blob: e.blob(11) + 'hello ' + 'world'
    w = varint(12) + b"\x02" + b"hello world"
    vecs.append({"source": "test/basic.js:32-51", "wire": w.hex(),
                 "frames": [{"type": 2, "blob": b"hello world".hex()}],
                 "err_code": 0, "tail": 0, "consumed": len(w)})
    # test/basic.js:53-84 mixed blobs: b1(11) 'hello '+'world', b2(11) 'HELLO '+'WORLD '
    # (12 bytes written into an 11-byte blob; encode.js does not validate the length).
    # Blobs serialise in creation order (encode.js:87-95); the trailing 0x20 is an
    # incomplete header, dropped silently at EOF (decode.js:135-142).
    w = varint(12) + b"\x02" + b"hello world" + varint(12) + b"\x02" + b"HELLO WORLD "
    vecs.append({"source": "test/basic.js:53-84", "wire": w.hex(),
                 "frames": [{"type": 2, "blob": b"hello world".hex()},
                            {"type": 2, "blob": b"HELLO WORLD".hex()}],
                 "err_code": 0, "tail": 1, "consumed": len(w) - 1})
    # test/basic.js:86-126 blob and changes: change issued while the blob is open is
    # queued behind it (encode.js:104-107, :95)
    w = varint(12) + b"\x02" + b"hello world" + frame(basic)
    vecs.append({"source": "test/basic.js:86-126", "wire": w.hex(),
                 "frames": [{"type": 2, "blob": b"hello world".hex()}, expect_basic],
                 "err_code": 0, "tail": 0, "consumed": len(w)})
    # example.js:1-53 sequence (three changes, one blob between)
    ex = make_msg(None, "lol1", 1, 0, 1, b"val").SerializeToString()
    ex2 = make_msg(None, "lol", 1, 0, 1, b"val").SerializeToString()
    w = frame(ex) + frame(ex2) + varint(12) + b"\x02" + b"hello world" + frame(ex2)
    exp = lambda k: {"type": 1, "key": k.hex(), "change": 1, "from": 0, "to": 1, "has_value": True,
                     "value": b"val".hex(), "has_subset": False, "subset": ""}
    vecs.append({"source": "example.js:1-53", "wire": w.hex(),
                 "frames": [exp(b"lol1"), exp(b"lol"), {"type": 2, "blob": b"hello world".hex()},
                            exp(b"lol")],
                 "err_code": 0, "tail": 0, "consumed": len(w)})
    # decode.js:159-161 unknown type after one good frame
    w = frame(basic) + varint(3) + b"\x07" + b"ab" + frame(basic)
    vecs.append({"source": "decode.js:159-161 unknown type", "wire": w.hex(),
                 "frames": [expect_basic], "err_code": 1, "err_detail": 7, "err_frame": 1})
    # decode.js:146-149 id 0: header consumed, declared length ignored
    w = varint(5) + b"\x00" + frame(basic)
    vecs.append({"source": "decode.js:146-149 type 0", "wire": w.hex(), "frames": [expect_basic],
                 "err_code": 0, "tail": 0, "consumed": len(w)})
    # truncated final frame: dropped at EOF (decode.js:135-142)
    full = frame(basic)
    w = full + full[:-1]
    vecs.append({"source": "decode.js:135-142 truncated final frame", "wire": w.hex(),
                 "frames": [expect_basic], "err_code": 0, "tail": 2, "consumed": len(full)})
    return vecs


def main():
    codec = codec_vectors()
    streams = stream_vectors()
    known = frame(make_msg(None, "key", 1, 0, 1, b"hello").SerializeToString()).hex()
    # SURVEY.md §0 known-answer frame
    assert known == "130112036b65791801200028013205" + b"hello".hex(), known
    with open(os.path.join(HERE, "change_codec.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "protobuf": "google.protobuf 7.35.1",
                   "vectors": codec}, f, indent=0)
    with open(os.path.join(HERE, "streams.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "vectors": streams}, f, indent=1)
    print(f"{len(codec)} codec vectors, {len(streams)} stream vectors")


if __name__ == "__main__":
    main()
