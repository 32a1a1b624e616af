"""Synthetic replication streams shaped like BASELINE.json's configs (seeded)."""
import random

import numpy as np


def varint(n):
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def change_payload(key, change, frm, to, value=None, subset=None):
    """protocol-buffers@2 field order (schema.proto:1-8): subset?, key, change, from, to, value?"""
    p = bytearray()
    if subset is not None:
        p += b"\x0a" + varint(len(subset)) + subset
    p += b"\x12" + varint(len(key)) + key
    p += b"\x18" + varint(change) + b"\x20" + varint(frm) + b"\x28" + varint(to)
    if value is not None:
        p += b"\x32" + varint(len(value)) + value
    return bytes(p)


def frame(payload, typ=1):
    return varint(len(payload) + 1) + bytes([typ]) + payload


def c2_stream(nframes, seed=1, start=0):
    """C2: exactly 86 B/frame: key = 10-digit i, change=(i%100)+1, from=i%128, to=(i+1)%128,
    64 random value bytes."""
    i = np.arange(start, start + nframes, dtype=np.int64)
    a = np.zeros((nframes, 86), np.uint8)
    a[:, 0] = 85
    a[:, 1] = 1
    a[:, 2] = 0x12
    a[:, 3] = 10
    for k in range(10):
        a[:, 4 + k] = 48 + (i // 10 ** (9 - k)) % 10
    a[:, 14] = 0x18
    a[:, 15] = (i % 100) + 1
    a[:, 16] = 0x20
    a[:, 17] = i % 128
    a[:, 18] = 0x28
    a[:, 19] = (i + 1) % 128
    a[:, 20] = 0x32
    a[:, 21] = 64
    rng = np.random.default_rng(seed)
    a[:, 22:] = rng.integers(0, 256, size=(nframes, 64), dtype=np.uint8)
    return a.reshape(-1)


def random_stream(rng, nframes, blob_p=0.05, blob_max=3000, zero_p=0.01, big_key_p=0.05,
                  subset_p=0.2, value_max=300):
    parts = []
    for _ in range(nframes):
        r = rng.random()
        if r < blob_p:
            b = rng.randbytes(rng.randint(0, blob_max))
            parts.append(frame(b, 2))
        elif r < blob_p + zero_p:
            parts.append(varint(rng.randint(0, 300)) + b"\x00")  # id 0: header only
        else:
            klen = rng.randint(128, 300) if rng.random() < big_key_p else rng.randint(0, 40)
            key = bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz0123456789") for _ in range(klen))
            val = None if rng.random() < 0.1 else rng.randbytes(rng.randint(0, value_max))
            sub = rng.randbytes(rng.randint(0, 8)) if rng.random() < subset_p else None
            nums = [rng.choice([rng.randint(0, 127), rng.randint(0, 2**21), rng.randint(0, 2**32 - 1),
                                rng.randint(0, 2**53 - 1)]) for _ in range(3)]
            parts.append(frame(change_payload(key, *nums, value=val, subset=sub)))
    return b"".join(parts)


def c5_stream(rng, nframes):
    """C5-shaped: 4096 B values, key length U[1,256], change/from/to U[0,2^32)."""
    parts = []
    for _ in range(nframes):
        key = rng.randbytes(rng.randint(1, 256))
        nums = [rng.randint(0, 2**32 - 1) for _ in range(3)]
        parts.append(frame(change_payload(key, *nums, value=rng.randbytes(4096))))
    return b"".join(parts)


def c3_stream(rng, units, frames_per_unit=1000, blob_len=1 << 20, seed=3):
    """C3-shaped: repeating [frames_per_unit C2 frames + one blob of blob_len random bytes]."""
    out = []
    for u in range(units):
        out.append(c2_stream(frames_per_unit, seed=seed + u, start=u * frames_per_unit).tobytes())
        out.append(frame(rng.randbytes(blob_len), 2))
    return b"".join(out)


C1_ALPHABET = b"abcdefghijklmnopqrstuvwxyz0123456789"


def c1_changes(n=10000, seed=11):
    """C1: n Changes, key 32 random [a-z0-9] chars, change=i+1, from=i, to=i+1,
    value 64 random bytes (seeded)."""
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, len(C1_ALPHABET), size=(n, 32))
    vals = rng.integers(0, 256, size=(n, 64), dtype=np.uint8)
    alpha = np.frombuffer(C1_ALPHABET, np.uint8)
    return [{"key": alpha[keys[i]].tobytes().decode(), "change": i + 1, "from": i, "to": i + 1,
             "value": vals[i].tobytes()} for i in range(n)]


C1_BLOB = b"hello world\n"


def c1_ops(n=10000, blob_after=5000, seed=11):
    """The C1 encoder call sequence: changes 0..blob_after-1, then e.blob(12) written with
    "hello world\\n" and ended, then the remaining changes (issued while the blob is still
    open, so encode.js:104-107 queues them behind it)."""
    ch = c1_changes(n, seed)
    ops = [dict(op="change", **c) for c in ch[:blob_after]]
    ops.append({"op": "blob", "len": len(C1_BLOB), "writes": [C1_BLOB]})
    ops += [dict(op="change", **c) for c in ch[blob_after:]]
    ops.append({"op": "finalize"})
    return ops


def c3_edge_stream(j, blob_len=70000, tail_frames=40, seed=21):
    """A C2 prefix padded so that a blob header (3-byte varint + id) starts j bytes before the
    64 KiB write edge, then the blob payload and more C2 frames (C3's chunk-edge case)."""
    pre = c2_stream(760, seed=seed).tobytes()  # 65360 bytes
    target = 65536 - j - len(pre)
    # a change frame of exactly `target` bytes: 2 header bytes + key/number fields + value
    vlen = target
    while len(frame(change_payload(b"pad", 1, 2, 3, value=bytes(vlen)))) > target:
        vlen -= 1
    pad = frame(change_payload(b"pad", 1, 2, 3, value=(bytes(range(256)) * (vlen // 256 + 1))[:vlen]))
    assert len(pad) == target, (len(pad), target)
    rng = np.random.default_rng(seed + j)
    blob = frame(rng.integers(0, 256, size=blob_len, dtype=np.uint8).tobytes(), 2)
    return pre + pad + blob + c2_stream(tail_frames, seed=seed + 100, start=760).tobytes()


def random_stream_seeded(seed, nframes):
    """random_stream with a fresh seeded generator (fixture recipes)."""
    return random_stream(random.Random(seed), nframes, blob_p=0.05, blob_max=5000, subset_p=0.2)


def shadow_stream(nframes, period=8192, shadow_at=100, small=10, seed=7, change_every=0):
    """Adversarial for the speculative decode: two valid framings that never merge. Real blob
    frames of `period` bytes; inside each payload, at `shadow_at`, a shadow chain of one
    `small`-byte blob frame and one blob frame of `period - small` bytes, so the shadow chain
    repeats with the same period, one frame denser than the real one. Every tile then holds a
    strong, denser chain the prediction prefers, consistent from tile to tile: a miss cascade.
    change_every > 0 makes every n-th real frame a Change frame (key + value) instead of a blob."""
    out = bytearray(np.random.default_rng(seed).integers(0, 256, size=nframes * period, dtype=np.uint8).tobytes())
    sh_small = varint(small - 1) + b"\x02"  # (small <= 128: a one-byte length)
    sh_big_len = period - small
    kb = len(varint(sh_big_len))
    sh_big = varint(sh_big_len - kb) + b"\x02"
    for i in range(nframes):
        r = i * period
        if change_every and i % change_every == 0:
            key = b"k%09d" % i
            head = b"\x12" + varint(len(key)) + key + b"\x18\x01\x20\x02\x28\x03"
            vlen = period - len(varint(period - 3)) - 1 - len(head) - 3
            pay = head + b"\x32" + varint(vlen)
            kr = len(varint(period - 3))
            hdr = varint(period - kr) + b"\x01"
            assert len(hdr) + len(pay) + vlen == period, (len(hdr), len(pay), vlen)
            out[r:r + len(hdr) + len(pay)] = hdr + pay
        else:
            kr = len(varint(period - 2))
            hdr = varint(period - kr) + b"\x02"
            out[r:r + len(hdr)] = hdr
        s = r + shadow_at
        out[s:s + len(sh_small)] = sh_small
        out[s + small:s + small + len(sh_big)] = sh_big
    return bytes(out)


def shadow_stream_np(nframes, period, shadow_at, small, seed=7):
    """shadow_stream for blob frames only, vectorised (GB-sized inputs): every period-byte row
    holds the real blob header at 0 and the shadow chain's two headers at shadow_at and
    shadow_at + small over random payload bytes."""
    a = np.random.default_rng(seed).integers(0, 256, size=(nframes, period), dtype=np.uint8)
    kr = len(varint(period - 2))
    hdr = varint(period - kr) + b"\x02"
    sh_small = varint(small - 1) + b"\x02"
    sh_big_len = period - small
    sh_big = varint(sh_big_len - len(varint(sh_big_len))) + b"\x02"
    for off, h in [(0, hdr), (shadow_at, sh_small), (shadow_at + small, sh_big)]:
        a[:, off:off + len(h)] = np.frombuffer(h, np.uint8)
    return a.reshape(-1)
