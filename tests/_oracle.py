"""ctypes access to the CPU parity oracle (oracle/_build/liboracle.so).

Test infrastructure only: the oracle is the checker, never the thing measured.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "liboracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ROOT, "oracle", "drp_oracle.c")
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        _lib = C.CDLL(LIB)
        _lib.oracle_change_decode.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p]
        _lib.oracle_change_decode.restype = C.c_int
        _lib.oracle_change_encode.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p,
                                              C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64,
                                              C.c_void_p, C.c_uint32, C.c_int, C.c_void_p]
        _lib.oracle_change_encode.restype = C.c_uint64
        _lib.oracle_encode_changes.argtypes = [C.c_void_p, C.c_uint64] + [C.c_void_p] * 11
        _lib.oracle_encode_changes.restype = C.c_uint64
        _lib.oracle_blob_header.argtypes = [C.c_uint64, C.c_void_p]
        _lib.oracle_blob_header.restype = C.c_int
        _lib.oracle_decode_batch.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64,
                                             C.c_uint64] + [C.c_void_p] * 14
        _lib.oracle_decode_batch.restype = C.c_int
        _lib.oracle_decode_writes.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_uint64,
                                              C.c_uint64] + [C.c_void_p] * 14
        _lib.oracle_decode_writes.restype = C.c_int
    return _lib


class OracleChange(C.Structure):
    _fields_ = [("key_off", C.c_uint32), ("key_len", C.c_uint32), ("subset_off", C.c_uint32),
                ("subset_len", C.c_uint32), ("value_off", C.c_uint32), ("value_len", C.c_uint32),
                ("change", C.c_uint64), ("from_", C.c_uint64), ("to", C.c_uint64),
                ("flags", C.c_uint8), ("err", C.c_uint32)]


def change_decode(payload: bytes):
    buf = C.create_string_buffer(payload, max(1, len(payload)))
    c = OracleChange()
    lib().oracle_change_decode(buf, len(payload), C.byref(c))
    return c


def change_encode(subset, key, change, frm, to, value):
    """subset/value: bytes or None (absent). Returns payload bytes."""
    hs, hv = subset is not None, value is not None
    sb, vb = subset or b"", value or b""
    n = lib().oracle_change_encode(sb, len(sb), hs, key, len(key), change, frm, to, vb, len(vb),
                                   hv, None)
    out = C.create_string_buffer(max(1, n))
    lib().oracle_change_encode(sb, len(sb), hs, key, len(key), change, frm, to, vb, len(vb), hv,
                               out)
    return out.raw[:n]


COLS32 = ["key_off", "key_len", "subset_off", "subset_len", "value_off", "value_len"]
COLS64 = ["change", "from", "to"]


def alloc_outputs(cap):
    o = {"payload_off": np.zeros(cap, np.uint64), "payload_len": np.zeros(cap, np.uint32),
         "type": np.zeros(cap, np.uint8), "flags": np.zeros(cap, np.uint8)}
    for k in COLS32:
        o[k] = np.zeros(cap, np.uint32)
    for k in COLS64:
        o[k] = np.zeros(cap, np.uint64)
    return o


def decode_batch(wire, chunk=0, blob_remaining=0, cap=None, outs=None, writes=None):
    """Run the decode.js restatement over `wire` written in `chunk`-byte pieces (or in the
    cycled list of piece sizes `writes`, 0 = the rest)."""
    if outs is not None:
        cap = len(outs["type"])
    if cap is None:
        cap = len(wire) // 2 + 2
    w = np.frombuffer(wire, np.uint8) if len(wire) else np.zeros(1, np.uint8)
    o = outs if outs is not None else alloc_outputs(cap)
    meta = np.zeros(9, np.uint64)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    cols = [p(o["payload_off"]), p(o["payload_len"]), p(o["type"]), p(o["key_off"]), p(o["key_len"]),
            p(o["subset_off"]), p(o["subset_len"]), p(o["value_off"]), p(o["value_len"]), p(o["change"]),
            p(o["from"]), p(o["to"]), p(o["flags"]), p(meta)]
    if writes is not None:
        ws = np.ascontiguousarray(writes, dtype=np.uint64)
        rc = lib().oracle_decode_writes(p(w), len(wire), p(ws), len(ws), blob_remaining, cap, *cols)
    else:
        rc = lib().oracle_decode_batch(p(w), len(wire), chunk, blob_remaining, cap, *cols)
    assert rc == 0, rc
    n = int(meta[0])
    # a malformed Change (err 4/5) stays in the table at index err_frame
    keep = n + (1 if int(meta[2]) in (4, 5) else 0)
    res = {k: v[:keep] for k, v in o.items()}
    res.update(nframes=n, err_frame=int(meta[1]), err_code=int(meta[2]), err_detail=int(meta[3]),
               consumed=int(meta[4]), tail=int(meta[5]), blob_remaining=int(meta[6]),
               changes=int(meta[7]), blobs=int(meta[8]))
    return res


def encode_changes(heap: bytes, cols: dict):
    """cols: numpy arrays key_off(u64) key_len(u32) subset_off subset_len value_off value_len
    change from to (u64) flags(u8). Returns wire bytes (encode.js framing)."""
    n = len(cols["key_len"])
    h = np.frombuffer(heap, np.uint8) if len(heap) else np.zeros(1, np.uint8)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    args = [p(np.ascontiguousarray(cols[k])) for k in
            ["key_off", "key_len", "subset_off", "subset_len", "value_off", "value_len", "change",
             "from", "to", "flags"]]
    total = lib().oracle_encode_changes(p(h), n, *args, None)
    out = np.zeros(max(1, total), np.uint8)
    lib().oracle_encode_changes(p(h), n, *args, p(out))
    return out[:total].tobytes()
