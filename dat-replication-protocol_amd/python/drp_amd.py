"""ctypes binding of libdrp (include/drp.h) for the Python test suite and bench.py.

The product host layer is the Node module in this package (index.js / decode.js /
encode.js over the N-API addon); this module exposes the same C ABI to Python so the
parity tests and the benchmark call exactly the code the addon calls. It loads the
in-tree lib/libdrp.so and raises if it is missing: there is no CPU fallback.
"""
import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("DRP_LIB") or os.path.join(PKG, "lib", "libdrp.so")
if not os.path.isabs(LIB_PATH):  # (an A/B build named relative to the repo root: exp/<name>/libdrp.so)
    LIB_PATH = os.path.join(os.path.dirname(PKG), LIB_PATH)

DRP_OK, DRP_E_INVAL, DRP_E_HIP, DRP_E_NOMEM, DRP_E_CAPACITY, DRP_E_NODEV = 0, -1, -2, -3, -4, -5
TYPE_CHANGE, TYPE_BLOB, FRAME_CONT, FRAME_PARTIAL = 1, 2, 0x40, 0x80
F_SUBSET, F_VALUE, F_BAD, F_MISSING, F_KEY_ASCII, F_KEY_UTF8 = 1, 2, 4, 8, 0x10, 0x20
ERR_NONE, ERR_TYPE, ERR_LEN, ERR_VARINT, ERR_CHANGE, ERR_REQUIRED = 0, 1, 2, 3, 4, 5
TAIL_NONE, TAIL_HEADER, TAIL_CHANGE, TAIL_BLOB = 0, 1, 2, 3

EXPORTS = [
    "drp_abi_version", "drp_open", "drp_close", "drp_stream", "drp_synchronize",
    "drp_last_timing", "drp_set_tile", "drp_set_strict", "drp_set_exact", "drp_set_key_post",
    "drp_set_blob_skip", "drp_decode_scratch_bytes",
    "drp_decode_device", "drp_decode_batch", "drp_decode_stage", "drp_decode_stage_v", "drp_decode_fetch", "drp_decode_fetch_block",
    "drp_decode_fetch_block_ex", "drp_decode_fetch_keys",
    "drp_encode_size", "drp_encode_device",
    "drp_encode_batch", "drp_index_scan", "drp_stream_stats_from_results", "drp_device",
    "drp_comm_id", "drp_comm_init_rank", "drp_comm_init_all", "drp_comm_destroy",
    "drp_index_allgather", "drp_index_allgather_multi", "drp_index_allgather_host", "drp_device_count",
    "drp_host_alloc", "drp_host_free",
]
KEY_POST_OFF, KEY_POST_HASH, KEY_POST_FLAGS = 0, 1, 2
BLOB_SKIP_OFF, BLOB_SKIP_AUTO, BLOB_SKIP_ALWAYS = 0, 1, 2
DRP_E_COMM = -7
COMM_ID_BYTES = 128

P = C.c_void_p
U64, U32 = C.c_uint64, C.c_uint32


class Frames(C.Structure):
    _fields_ = [("payload_off", P), ("payload_len", P), ("type", P)]


class Changes(C.Structure):
    _fields_ = [(k, P) for k in ["key_off", "key_len", "subset_off", "subset_len", "value_off",
                                 "value_len", "change", "from_", "to", "flags", "key_hash"]]


class ChangeSrc(C.Structure):
    _fields_ = [(k, P) for k in ["key_off", "key_len", "subset_off", "subset_len", "value_off",
                                 "value_len", "change", "from_", "to", "flags"]]


class Carry(C.Structure):
    _fields_ = [("blob_remaining", U64), ("consumed", U64), ("tail_kind", U32), ("reserved", U32),
                ("frame_bytes", U64)]


class StreamResult(C.Structure):
    _fields_ = [("frame_begin", U64), ("frames", U64), ("changes", U64), ("blobs", U64),
                ("consumed", U64), ("blob_remaining", U64), ("err_frame", U64), ("err_code", U32),
                ("err_detail", U32), ("tail_kind", U32), ("reserved", U32), ("tail_frame_bytes", U64)]


class StreamStats(C.Structure):
    _fields_ = [("frames", U64), ("changes", U64), ("blobs", U64), ("wire_bytes", U64)]


class Chunk(C.Structure):
    _fields_ = [("bytes", P), ("n", U64)]


class Timing(C.Structure):
    _fields_ = [("decode_ms", C.c_float), ("finalize_ms", C.c_float), ("total_ms", C.c_float),
                ("strict_reruns", U32), ("spec_repairs", U32), ("exact_retries", U32), ("verify_relisted", U32),
                ("seg_repairs", U32), ("reserved", U32), ("h2d_ms", C.c_float), ("d2h_ms", C.c_float),
                ("h2d_bytes", U64), ("h2d_skipped", U64), ("host_copied", U64)]


_lib = None


def lib():
    """Load lib/libdrp.so (raises OSError if it was not built: no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"libdrp not built: {LIB_PATH} missing (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        L.drp_abi_version.restype = C.c_int
        L.drp_open.argtypes = [C.c_int, C.POINTER(P)]
        L.drp_close.argtypes = [P]
        L.drp_close.restype = None
        L.drp_stream.argtypes = [P]
        L.drp_stream.restype = P
        L.drp_synchronize.argtypes = [P]
        L.drp_last_timing.argtypes = [P, C.POINTER(Timing)]
        L.drp_set_tile.argtypes = [P, U32]
        L.drp_set_strict.argtypes = [P, C.c_int]
        L.drp_set_exact.argtypes = [P, C.c_int]
        L.drp_set_key_post.argtypes = [P, C.c_int]
        L.drp_set_blob_skip.argtypes = [P, C.c_int]
        L.drp_decode_scratch_bytes.argtypes = [P, U64, U64]
        L.drp_decode_scratch_bytes.restype = U64
        L.drp_decode_device.argtypes = [P, P, U64, P, P, U64, C.POINTER(Frames),
                                        C.POINTER(Changes), U64, P]
        L.drp_decode_batch.argtypes = [P, P, U64, C.POINTER(Carry), C.POINTER(Frames),
                                       C.POINTER(Changes), U64, C.POINTER(U64), C.POINTER(U64),
                                       C.POINTER(U32), C.POINTER(U32)]
        L.drp_decode_stage.argtypes = [P, P, U64, C.POINTER(Carry), C.POINTER(U64), C.POINTER(U64),
                                       C.POINTER(U32), C.POINTER(U32)]
        L.drp_decode_stage_v.argtypes = [P, C.POINTER(Chunk), U64, C.POINTER(Carry), C.POINTER(U64), C.POINTER(U64),
                                         C.POINTER(U32), C.POINTER(U32)]
        L.drp_decode_fetch.argtypes = [P, C.POINTER(Frames), C.POINTER(Changes), U64, U64]
        L.drp_decode_fetch_block.argtypes = [P, P, U64, C.POINTER(U64), U64, U64]
        L.drp_decode_fetch_block_ex.argtypes = [P, P, U64, C.POINTER(U64), U64, U64, U32]
        L.drp_decode_fetch_keys.argtypes = [P, U64, U64, P, P, U64, C.POINTER(U64)]
        L.drp_encode_size.argtypes = [P, C.POINTER(ChangeSrc), U64, C.POINTER(U64)]
        L.drp_encode_device.argtypes = [P, C.POINTER(ChangeSrc), P, U64, U64, P, P, U64]
        L.drp_encode_batch.argtypes = [P, C.POINTER(ChangeSrc), P, U64, U64, P, U64,
                                       C.POINTER(U64)]
        L.drp_index_scan.argtypes = [P, P, U64, P]
        L.drp_stream_stats_from_results.argtypes = [P, P, P, U64, P]
        L.drp_device.argtypes = [P]
        L.drp_comm_id.argtypes = [P]
        L.drp_comm_init_rank.argtypes = [P, P, C.c_int, C.c_int, C.POINTER(P)]
        L.drp_comm_init_all.argtypes = [C.POINTER(P), C.c_int, C.POINTER(P)]
        L.drp_comm_destroy.argtypes = [P]
        L.drp_comm_destroy.restype = None
        L.drp_index_allgather.argtypes = [P, P, P, U64, P, P]
        L.drp_index_allgather_multi.argtypes = [C.POINTER(P), C.POINTER(P), C.c_int, C.POINTER(P), U64,
                                                C.POINTER(P), C.POINTER(P)]
        L.drp_index_allgather_host.argtypes = [C.POINTER(P), C.POINTER(P), C.c_int, C.POINTER(P), U64, P, P]
        L.drp_device_count.argtypes = [C.POINTER(C.c_int)]
        for f in ["drp_open", "drp_synchronize", "drp_last_timing", "drp_set_tile",
                  "drp_set_strict", "drp_set_exact", "drp_set_key_post", "drp_set_blob_skip", "drp_decode_device",
                  "drp_decode_batch",
                  "drp_decode_stage", "drp_decode_stage_v", "drp_decode_fetch", "drp_encode_size",
                  "drp_encode_device", "drp_encode_batch", "drp_index_scan",
                  "drp_stream_stats_from_results", "drp_device", "drp_comm_id", "drp_comm_init_rank",
                  "drp_comm_init_all", "drp_index_allgather", "drp_index_allgather_multi",
                  "drp_index_allgather_host", "drp_device_count"]:
            getattr(L, f).restype = C.c_int
        _lib = L
    return _lib


class DrpError(RuntimeError):
    def __init__(self, fn, rc):
        super().__init__(f"{fn} failed with {rc}")
        self.rc = rc


def _chk(fn, rc):
    if rc != DRP_OK:
        raise DrpError(fn, rc)


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


COLS32 = ["key_off", "key_len", "subset_off", "subset_len", "value_off", "value_len"]
COLS64 = ["change", "from", "to"]


def alloc_host_outputs(cap, key_hash=False):
    o = {"payload_off": np.zeros(cap, np.uint64), "payload_len": np.zeros(cap, np.uint32),
         "type": np.zeros(cap, np.uint8), "flags": np.zeros(cap, np.uint8)}
    if key_hash:
        o["key_hash"] = np.zeros(cap, np.uint64)
    for k in COLS32:
        o[k] = np.zeros(cap, np.uint32)
    for k in COLS64:
        o[k] = np.zeros(cap, np.uint64)
    return o


def _structs(o, ptr):
    fr = Frames(ptr(o["payload_off"]), ptr(o["payload_len"]), ptr(o["type"]))
    co = Changes(*[ptr(o[k]) for k in COLS32], ptr(o["change"]), ptr(o["from"]), ptr(o["to"]),
                 ptr(o["flags"]), ptr(o["key_hash"]) if o.get("key_hash") is not None else None)
    return fr, co


class Ctx:
    """One libdrp context (device + HIP stream + scratch)."""

    def __init__(self, device=0, tile=0):
        self.L = lib()
        h = P()
        _chk("drp_open", self.L.drp_open(device, C.byref(h)))
        self.h = h
        if tile:
            _chk("drp_set_tile", self.L.drp_set_tile(self.h, tile))

    def close(self):
        if self.h:
            self.L.drp_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def stream(self):
        return self.L.drp_stream(self.h)

    # libdrp launches on its own non-blocking HIP stream: work torch queued on its current
    # stream (allocations, fills, copies producing our inputs) must be ordered before a
    # libdrp call, and torch must not read libdrp outputs before libdrp's stream is done.
    def _ext(self, dev):
        import torch
        ext = getattr(self, "_ext_stream", None)
        if ext is None or ext.device != dev:
            ext = torch.cuda.ExternalStream(self.stream, device=dev)
            self._ext_stream = ext
        return ext

    def order_after_torch(self, t):
        """libdrp's stream waits for the work queued so far on torch's current stream (nothing
        to do when torch's current stream is libdrp's own, e.g. under torch.cuda.stream(...))."""
        import torch
        ext, cur = self._ext(t.device), torch.cuda.current_stream(t.device)
        if cur.cuda_stream != ext.cuda_stream:
            ext.wait_stream(cur)

    def order_torch_after(self, t):
        """torch's current stream waits for the work queued so far on libdrp's stream."""
        import torch
        ext, cur = self._ext(t.device), torch.cuda.current_stream(t.device)
        if cur.cuda_stream != ext.cuda_stream:
            cur.wait_stream(ext)

    def set_strict(self, on):
        _chk("drp_set_strict", self.L.drp_set_strict(self.h, 1 if on else 0))

    def set_exact(self, on):
        """Force the exact decode kernel (else: speculate-and-verify with exact fallback)."""
        _chk("drp_set_exact", self.L.drp_set_exact(self.h, 1 if on else 0))

    def set_blob_skip(self, mode):
        """Host batches: BLOB_SKIP_AUTO (default), _ALWAYS (every batch in blob-skipping
        pieces) or _OFF (every batch staged whole); results are identical."""
        _chk("drp_set_blob_skip", self.L.drp_set_blob_skip(self.h, mode))

    def set_tile(self, tile):
        _chk("drp_set_tile", self.L.drp_set_tile(self.h, tile))

    def timing(self):
        t = Timing()
        _chk("drp_last_timing", self.L.drp_last_timing(self.h, C.byref(t)))
        return t

    # ---- host-buffer batch decode (the N-API addon's path) -----------------------------
    def decode_batch(self, wire, blob_remaining=0, cap=None, key_hash=False, outs=None):
        """drp_decode_batch into host columns; key_hash=True also asks for the key hash
        column and the DRP_F_KEY_ASCII / DRP_F_KEY_UTF8 flags. outs: host columns to reuse
        (alloc_host_outputs(cap))."""
        w = np.frombuffer(bytes(wire), np.uint8) if not isinstance(wire, np.ndarray) else wire
        n = int(w.size)
        if outs is not None:
            cap = int(outs["payload_off"].size)
        elif cap is None:
            cap = n // 2 + 2
        o = outs if outs is not None else alloc_host_outputs(cap, key_hash)
        fr, co = _structs(o, _p)
        carry = Carry(blob_remaining, 0, 0, 0, 0)
        nf, ef, ec, ed = U64(), U64(), U32(), U32()
        buf = w if n else np.zeros(16, np.uint8)
        rc = self.L.drp_decode_batch(self.h, _p(buf), n, C.byref(carry), C.byref(fr), C.byref(co),
                                     cap, C.byref(nf), C.byref(ef), C.byref(ec), C.byref(ed))
        _chk("drp_decode_batch", rc)
        nframes = int(nf.value)
        keep = nframes + (1 if ec.value in (ERR_CHANGE, ERR_REQUIRED) else 0)
        res = {k: v[:keep] for k, v in o.items()}
        res.update(nframes=nframes, err_frame=int(ef.value), err_code=int(ec.value),
                   err_detail=int(ed.value), consumed=int(carry.consumed),
                   tail=int(carry.tail_kind), blob_remaining=int(carry.blob_remaining),
                   frame_bytes=int(carry.frame_bytes))
        return res

    def decode_staged(self, wire, blob_remaining=0, pieces=1, key_hash=False, block=False, f64=False, keys=False):
        """drp_decode_stage, then drp_decode_fetch of the rows in `pieces` consecutive
        fetches into host columns sized from the frame count (the N-API addon's path). `wire`
        as a list of byte strings: the batch is those chunks end to end (drp_decode_stage_v).
        block=True: one drp_decode_fetch_block of every row into one host block instead (the
        columns at 64-byte aligned offsets, as the addon lays them out); f64=True: with
        drp_decode_fetch_block_ex(DRP_FETCH_F64), payload_off / change / from / to as float64.
        keys=True: the key flags too, and drp_decode_fetch_keys' "kp" (u32 per row) and "key_text"
        (bytes; None when the batch was staged in pieces: DRP_E_INVAL)."""
        carry = Carry(blob_remaining, 0, 0, 0, 0)
        nf, ef, ec, ed = U64(), U64(), U32(), U32()
        kpost = KEY_POST_HASH if key_hash else (KEY_POST_FLAGS if keys else KEY_POST_OFF)
        _chk("drp_set_key_post", self.L.drp_set_key_post(self.h, kpost))
        if isinstance(wire, (list, tuple)):
            arrs = [np.frombuffer(bytes(c), np.uint8) if len(c) else np.zeros(1, np.uint8) for c in wire]
            ch = (Chunk * max(1, len(arrs)))(*[Chunk(_p(a), len(c)) for a, c in zip(arrs, wire)])
            _chk("drp_decode_stage_v", self.L.drp_decode_stage_v(self.h, ch, len(arrs), C.byref(carry), C.byref(nf),
                                                                 C.byref(ef), C.byref(ec), C.byref(ed)))
        else:
            w = np.frombuffer(bytes(wire), np.uint8) if not isinstance(wire, np.ndarray) else wire
            n = int(w.size)
            buf = w if n else np.zeros(16, np.uint8)
            _chk("drp_decode_stage", self.L.drp_decode_stage(self.h, _p(buf), n, C.byref(carry), C.byref(nf),
                                                             C.byref(ef), C.byref(ec), C.byref(ed)))
        rows = int(nf.value) + (1 if ec.value in (ERR_CHANGE, ERR_REQUIRED) else 0)
        if block:
            names = ["payload_off", "payload_len", "type"] + COLS32 + COLS64 + ["flags"] + (["key_hash"] if key_hash else [])
            dt = {"payload_off": np.uint64, "payload_len": np.uint32, "type": np.uint8, "flags": np.uint8,
                  "key_hash": np.uint64, **{k: np.uint32 for k in COLS32}, **{k: np.uint64 for k in COLS64}}
            if f64:
                dt.update({k: np.float64 for k in ["payload_off"] + COLS64})
            offs, at = [], 0
            for k in names:
                offs.append(at)
                at += (rows * np.dtype(dt[k]).itemsize + 8 + 63) & ~63
            blk = np.full(at + 64, 0xAB, np.uint8)
            col_off = (U64 * 14)(*(offs + [~0 & 0xFFFFFFFFFFFFFFFF] * (14 - len(offs))))
            if f64:
                _chk("drp_decode_fetch_block_ex", self.L.drp_decode_fetch_block_ex(self.h, _p(blk), at, col_off, 0, rows, 1))
            else:
                _chk("drp_decode_fetch_block", self.L.drp_decode_fetch_block(self.h, _p(blk), at, col_off, 0, rows))
            o = {k: blk[a:a + rows * np.dtype(dt[k]).itemsize].view(dt[k]) for k, a in zip(names, offs)}
            pieces = 0
        else:
            o = alloc_host_outputs(rows, key_hash)
        bounds = np.linspace(0, rows, pieces + 1).astype(np.int64)
        for a, b in zip(bounds[:-1], bounds[1:]):
            part = {k: v[a:] for k, v in o.items()}
            fr, co = _structs(part, _p)
            _chk("drp_decode_fetch", self.L.drp_decode_fetch(self.h, C.byref(fr), C.byref(co), int(a), int(b - a)))
        if keys:
            kp = np.zeros(max(rows, 1), np.uint32)
            tl = U64()
            rc = self.L.drp_decode_fetch_keys(self.h, 0, rows, _p(kp), None, 0, C.byref(tl))
            if rc == -1:  # DRP_E_INVAL: staged in pieces
                o.update(kp=None, key_text=None)
            else:
                _chk("drp_decode_fetch_keys", rc)
                text = np.zeros(max(int(tl.value), 1), np.uint8)
                _chk("drp_decode_fetch_keys", self.L.drp_decode_fetch_keys(self.h, 0, rows, _p(kp), _p(text),
                                                                           int(tl.value), C.byref(tl)))
                o.update(kp=kp[:rows], key_text=text[:int(tl.value)].tobytes())
        o.update(nframes=int(nf.value), err_frame=int(ef.value), err_code=int(ec.value), err_detail=int(ed.value),
                 consumed=int(carry.consumed), tail=int(carry.tail_kind), blob_remaining=int(carry.blob_remaining),
                 frame_bytes=int(carry.frame_bytes))
        return o

    # ---- device decode over torch tensors (bench path) --------------------------------
    def decode_device(self, wire_t, stream_off_t, entry_t, outs, cap, results_t):
        """All arguments are torch CUDA tensors (uint8 wire, int64 offsets); outs is a dict
        of column tensors; results_t is a uint8 tensor of nstreams*sizeof(StreamResult)."""
        tp = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
        fr, co = _structs(outs, tp)
        ns = stream_off_t.numel() - 1
        self.order_after_torch(wire_t)
        rc = self.L.drp_decode_device(self.h, tp(wire_t), wire_t.numel(), tp(stream_off_t),
                                      tp(entry_t), ns, C.byref(fr), C.byref(co), cap, tp(results_t))
        _chk("drp_decode_device", rc)
        self.order_torch_after(wire_t)

    # ---- encode -----------------------------------------------------------------------
    def encode_device(self, cols_t, heap_t, n, frame_off_t, out_t, cap):
        """Device encode over torch CUDA tensors (asynchronous, on this ctx's stream): cols_t
        holds the drp_change_src columns (int64 offsets, int32 lengths, int64 numbers, uint8
        flags); frame_off_t (int64, n + 1) receives the frame offsets, out_t (uint8) the wire."""
        tp = lambda t: C.c_void_p(t.data_ptr())
        src = ChangeSrc(*[tp(cols_t[k]) for k in ["key_off", "key_len", "subset_off", "subset_len",
                                                  "value_off", "value_len", "change", "from", "to",
                                                  "flags"]])
        self.order_after_torch(heap_t)
        _chk("drp_encode_device", self.L.drp_encode_device(self.h, C.byref(src), tp(heap_t), heap_t.numel(),
                                                           n, tp(frame_off_t), tp(out_t), cap))
        self.order_torch_after(heap_t)

    def encode_batch(self, heap, cols):
        n = len(cols["key_len"])
        h = np.frombuffer(bytes(heap), np.uint8) if not isinstance(heap, np.ndarray) else heap
        arrs = {k: np.ascontiguousarray(cols[k]) for k in
                ["key_off", "key_len", "subset_off", "subset_len", "value_off", "value_len",
                 "change", "from", "to", "flags"]}
        src = ChangeSrc(*[_p(arrs[k]) for k in ["key_off", "key_len", "subset_off", "subset_len",
                                                  "value_off", "value_len", "change", "from", "to",
                                                  "flags"]])
        total = U64()
        _chk("drp_encode_size", self.L.drp_encode_size(self.h, C.byref(src), n, C.byref(total)))
        out = np.zeros(max(16, int(total.value)), np.uint8)
        written = U64()
        hb = h if h.size else np.zeros(16, np.uint8)
        _chk("drp_encode_batch", self.L.drp_encode_batch(self.h, C.byref(src), _p(hb), int(h.size), n,
                                                         _p(out), int(total.value), C.byref(written)))
        return out[:int(written.value)].tobytes()


class Comm:
    """An RCCL communicator owned by libdrp (drp_comm_*): one rank per process."""

    def __init__(self, ctx, comm_id, nranks, rank):
        self.L = lib()
        h = P()
        _chk("drp_comm_init_rank", self.L.drp_comm_init_rank(ctx.h, comm_id, nranks, rank, C.byref(h)))
        self.h, self.nranks, self.rank = h, nranks, rank

    @staticmethod
    def new_id():
        buf = C.create_string_buffer(COMM_ID_BYTES)
        _chk("drp_comm_id", lib().drp_comm_id(buf))
        return buf.raw

    def allgather_index(self, ctx, local_t, global_t, base_t):
        """drp_index_allgather over torch CUDA tensors (int64 (per_rank, 4) local stats)."""
        ctx.order_after_torch(local_t)
        tp = lambda t: C.c_void_p(t.data_ptr())
        _chk("drp_index_allgather", self.L.drp_index_allgather(ctx.h, self.h, tp(local_t), local_t.shape[0],
                                                               tp(global_t), tp(base_t)))

    def close(self):
        if self.h:
            self.L.drp_comm_destroy(self.h)
            self.h = None
