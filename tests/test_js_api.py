"""The Node host layer (dat-replication-protocol_amd/{index,decode,encode}.js over the
N-API addon): reference-API round trips (test/basic.js restated) and event-level parity
with the oracle across chunkings and asynchronous callback acks."""
import hashlib
import json
import os
import random
import shutil
import subprocess
import tempfile

import pytest

import _oracle as O
import _streams as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(ROOT, "tests", "js")
NODE = shutil.which("node")

needs_node = pytest.mark.skipif(NODE is None, reason="node not installed")


@needs_node
def test_package_loads_without_gpu_use():
    """require() works and exposes the reference's entry points (index.js:1-2); the addon
    exports open/decode/encode over libdrp."""
    code = ("var p=require(%r); var a=require(%r);"
            "console.log(JSON.stringify([typeof p.encode, typeof p.decode, Object.keys(a).sort(), a.abiVersion]))"
            % (os.path.join(ROOT, "dat-replication-protocol_amd"),
               os.path.join(ROOT, "dat-replication-protocol_amd", "lib", "drp.node")))
    out = json.loads(subprocess.check_output([NODE, "-e", code], text=True, timeout=60))
    assert out == ["function", "function", ["abiVersion", "decode", "decodeSync", "deviceCount", "encode",
                                            "indexAllgather", "open"], 5]


def _enc(b, digest):
    return hashlib.sha256(b).hexdigest()[:16] if digest else b.hex()


def oracle_events(wire, digest=False):
    r = O.decode_batch(wire)
    ev = []
    for k in range(r["nframes"]):
        off, ln, t = int(r["payload_off"][k]), int(r["payload_len"][k]), int(r["type"][k])
        p = wire[off:off + ln]
        if t & 0x3F == 1:
            f = int(r["flags"][k])
            so, sl = int(r["subset_off"][k]), int(r["subset_len"][k])
            ko, kl = int(r["key_off"][k]), int(r["key_len"][k])
            vo, vl = int(r["value_off"][k]), int(r["value_len"][k])
            # the JS object carries strings; compare their UTF-8 re-encoding
            sub = p[so:so + sl].decode("utf-8", "replace").encode() if f & 1 else b""
            key = p[ko:ko + kl].decode("utf-8", "replace").encode()
            ev.append({"t": "change", "subset": _enc(sub, digest), "key": _enc(key, digest),
                       "change": int(r["change"][k]), "from": int(r["from"][k]), "to": int(r["to"][k]),
                       "value": _enc(p[vo:vo + vl], digest) if f & 2 else None})
        else:
            ev.append({"t": "blob", "data": _enc(wire[off:off + ln], digest), "len": ln})
    return r, ev


def run_js(wire, sizes, mode="", nth=0, batch=None, mock=False):
    """Events of the package's Decoder fed `wire` in the cycled write `sizes`; `batch` sets
    DRP_MAX_BATCH (a small one makes every few writes a GPU batch of their own, so frames,
    headers and blobs straddle batch edges and the decoder's carry runs)."""
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(wire)
        path = f.name
    env = dict(os.environ)
    if batch:
        env["DRP_MAX_BATCH"] = str(batch)
    if mock:  # the CPU stand-in for the addon (tests/js/mock_native.js): the JS layer alone
        env["DRP_MOCK_NATIVE"] = "1"
    try:
        out = subprocess.check_output([NODE, os.path.join(JS, "decode_events.js"), path, sizes, mode, str(nth)],
                                      text=True, timeout=150, env=env)
    finally:
        os.unlink(path)
    return json.loads(out)


def run_encode(ops, slow=False):
    from test_ref_fixtures import _val  # noqa: F401  (ops carry hex values already)
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(ops, f)
        path = f.name
    try:
        out = subprocess.check_output([NODE, os.path.join(JS, "encode_ops.js"), path] + (["slow"] if slow else []),
                                      text=True, timeout=120)
    finally:
        os.unlink(path)
    return json.loads(out)


def ops_json(ops):
    out = []
    for o in ops:
        o = dict(o)
        if o.get("value") is not None and not isinstance(o["value"], str):
            o["value"] = o["value"].hex()
        if "writes" in o:
            o["writes"] = [w if isinstance(w, str) else w.hex() for w in o["writes"]]
        out.append(o)
    return out


@pytest.mark.gpu
@needs_node
def test_reference_round_trips():
    out = subprocess.run([NODE, os.path.join(JS, "basic.js")], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.count("ok ") == 4, out.stdout


@pytest.mark.gpu
@needs_node
@pytest.mark.parametrize("sizes,mode,batch", [("65536", "", None), ("1", "", None), ("3,7,64", "", None),
                                              ("1000", "async", None), ("17,4096", "async", None),
                                              ("1000,7", "", 4096), ("3,7,64", "async", 1024),
                                              ("65536", "ticks", 65536), ("509,1", "ticks", 3000)])
def test_decoder_events_match_oracle(sizes, mode, batch):
    """Event parity with the oracle across write sizes, async acks and (batch) GPU batches of a
    few KiB, so the carry of decode.js runs: headers, Change frames and blobs cut by batch edges
    (ticks: writes spread over event-loop turns, each turn's writes one batch)."""
    rng = random.Random(len(sizes) * 31 + len(mode) + (batch or 0))
    wire = S.random_stream(rng, 300 if sizes == "1" else 1500, blob_p=0.08, blob_max=3000,
                           subset_p=0.3)
    r, exp = oracle_events(wire)
    got = run_js(wire, sizes, mode, batch=batch)
    got = [e for e in got if e["t"] != "close"]
    assert got[-1]["t"] == "finish", got[-3:]
    assert got[:-1] == exp
    assert got[-1]["changes"] == r["changes"] and got[-1]["blobs"] == r["blobs"]
    assert got[-1]["bytes"] == len(wire)


@pytest.mark.gpu
@needs_node
def test_decoder_batch_edges():
    """Crafted batch edges (DRP_MAX_BATCH=64, one write per batch): a Change frame whose header
    and payload are cut mid-way, a header cut between its varint bytes, a 2-byte-varint header
    cut after its first byte, a blob cut in its header and its payload spanning several batches,
    and a Change frame longer than a batch (collected once into its declared size, decode.js:229-247)."""
    big = S.frame(S.change_payload(b"k" * 130, 300, 2**32 - 1, 5, value=bytes(range(256)) * 2, subset=b"s"))
    parts = [S.frame(S.change_payload(b"key%d" % i, i, 0, 1, value=b"v" * (i * 7 % 50))) for i in range(12)]
    wire = (parts[0] + parts[1] + big + parts[2] + S.frame(bytes(range(200)), 2) + parts[3] +
            S.frame(b"", 2) + parts[4] + big + b"".join(parts[5:]))
    r, exp = oracle_events(wire)
    for sizes in ["64", "5,59", "1,2,3,61", "130,1"]:
        for mode in ("", "async"):
            got = [e for e in run_js(wire, sizes, mode, batch=64) if e["t"] != "close"]
            assert got[:-1] == exp, (sizes, mode)
            assert got[-1] == {"t": "finish", "changes": r["changes"], "blobs": r["blobs"], "bytes": len(wire)}


@pytest.mark.gpu
@needs_node
def test_decoder_protocol_error():
    good = bytes.fromhex("130112036b65791801200028013205") + b"hello"
    wire = good + b"\x03\x07ab" + good
    got = run_js(wire, "5")
    assert [e["t"] for e in got] == ["change", "error"]
    assert got[1]["message"] == "Protocol error, unknown type: 7"


@pytest.mark.gpu
@needs_node
def test_c1_round_trip_through_the_package():
    """BASELINE configs[0] (C1): 10,000 Changes (32-char [a-z0-9] keys, change=i+1, from=i,
    to=i+1, 64 random value bytes) with e.blob(12) "hello world\n" issued after change 5000 while
    the later changes queue behind it, through encode() with a slow consumer (push() returns
    false: the drain path of encode.js:139-151), then decode(). The encoder's bytes equal the
    reference encode.js's (fixture recorded in place) and the oracle's; the decoder's events
    equal the oracle's (reference test/basic.js:86-126 at scale)."""
    from test_ref_fixtures import FIX, reference_order_encode
    ops = S.c1_ops()
    got = run_encode(ops_json(ops), slow=True)
    ref = FIX["encode"]["c1"]
    wire = reference_order_encode(ops)
    assert hashlib.sha256(wire).hexdigest() == ref["wire_sha256"]
    assert got["sha256"] == ref["wire_sha256"] and got["len"] == ref["wire_len"]
    assert (got["changes"], got["blobs"], got["bytes"]) == (10000, 1, ref["bytes"])
    assert got["acked"] == 10001  # every change cb and the blob's finish cb ran
    assert got["pushFalse"] >= 1, "the slow consumer never made push() return false"
    r, exp = oracle_events(wire, digest=True)
    assert r["changes"] == 10000 and r["blobs"] == 1
    for sizes in ["65536", "1000,7"]:
        ev = [e for e in run_js(wire, sizes, "digest") if e["t"] != "close"]
        assert ev[:-1] == exp and ev[-1] == {"t": "finish", "changes": 10000, "blobs": 1, "bytes": len(wire)}


@pytest.mark.gpu
@needs_node
@pytest.mark.parametrize("name", ["basic_change", "basic_blob", "basic_blob_then_change", "interleave", "widths"])
def test_encoder_matches_reference_fixtures(name):
    """The package's encoder reproduces the bytes the reference encode.js wrote for the same
    call sequence (blob/change interleavings, field widths, absent/empty values, subsets)."""
    from test_ref_fixtures import FIX
    c = FIX["encode"][name]
    for slow in (False, True):
        got = run_encode(c["ops"], slow=slow)
        assert got["hex"] == c["wire"], (name, slow)
        assert (got["changes"], got["blobs"], got["bytes"]) == (c["changes"], c["blobs"], c["bytes"])


@pytest.mark.gpu
@needs_node
def test_decoder_destroy_mid_batch():
    """destroy() inside a change callback (decode.js:104-110) stops delivery at once: the events
    before it equal the oracle's, 'close' follows, nothing else is delivered and there is no
    'finish'; the GPU batch still in flight is dropped."""
    wire = S.c2_stream(5000, seed=3).tobytes() + S.random_stream(random.Random(3), 200)
    _, exp = oracle_events(wire)
    for sizes, nth in [("65536", 37), ("1000", 1), ("300000", 4999)]:
        got = run_js(wire, sizes, "destroy", nth)
        assert got[:nth] == exp[:nth], sizes
        assert got[nth:] == [{"t": "close"}], (sizes, got[nth:nth + 3])


@pytest.mark.gpu
@needs_node
def test_c3_blobs_through_the_package():
    """BASELINE configs[2] shape through the Node path: 1 MiB blobs between C2 runs in 64 KiB
    writes (blob headers and frames straddle the write edges; blob continuations pass through
    without going to HBM), asynchronous acks; every event equals the oracle's."""
    wire = S.c3_stream(random.Random(8), 3, frames_per_unit=1000)
    r, exp = oracle_events(wire, digest=True)
    for sizes, mode in [("65536", "digest"), ("65536,1,4093", "digest")]:
        got = [e for e in run_js(wire, sizes, mode) if e["t"] != "close"]
        assert got[:-1] == exp
        assert got[-1] == {"t": "finish", "changes": r["changes"], "blobs": r["blobs"], "bytes": len(wire)}


@pytest.mark.gpu
@needs_node
def test_c3_blob_payloads_stay_in_host_memory():
    """SURVEY §8 f2 through the Node path: a C3-shaped stream (100 units of 1000 C2 frames + a
    1 MiB blob, ~113 MB) in 1 MiB writes; the addon stages the decoder's batches in pieces that
    skip blob payloads, so at most 25% of the wire is copied into HBM and at most 25% is copied
    on the host (the written chunks are handed over as they are and only the staged ranges are
    gathered), every blob piece handed to the blob stream is a slice of a written chunk
    (decode.js:179-202), and every event still equals the oracle's."""
    wire = S.c3_stream(random.Random(12), 100, frames_per_unit=1000)
    r, exp = oracle_events(wire, digest=True)
    out = [e for e in run_js(wire, str(1 << 20), "h2d") if e["t"] != "close"]
    tm = out.pop()
    assert tm["t"] == "timing"
    assert out[:-1] == exp
    assert out[-1] == {"t": "finish", "changes": r["changes"], "blobs": r["blobs"], "bytes": len(wire)}
    print(f"staged {tm['h2dBytes']} B of {len(wire)} ({tm['h2dBytes'] / len(wire):.1%}), "
          f"skipped {tm['h2dSkipped']} B, copied on the host {tm['hostCopied']} B")
    assert tm["h2dBytes"] <= len(wire) // 4, tm
    # f2: the batch is never concatenated on the host; libdrp gathers only the staged ranges
    # (drp_decode_stage_v), and only frames straddling two writes are copied by the JS layer
    assert tm["hostCopied"] <= len(wire) // 4, tm
    assert tm["blobPieces"] >= r["blobs"] and tm["blobPiecesShared"] == tm["blobPieces"], tm


@pytest.mark.gpu
@needs_node
def test_held_values_survive_later_batches():
    """Change values are slices of the written chunks (no batch copy: libdrp gathers what it
    stages, drp_decode_stage_v), and the columns come back in pinned blocks the addon recycles
    (drp_napi.c colblock). Values held until the end of the stream (digested only at 'finish',
    ~40 batches later) must still hold their own bytes."""
    wire = S.c2_stream(600_000, seed=21).tobytes()
    r, exp = oracle_events(wire, digest=True)
    got = [e for e in run_js(wire, "65536", "hold", batch=1 << 20) if e["t"] != "close"]
    assert got[:-1] == exp
    assert got[-1] == {"t": "finish", "changes": r["changes"], "blobs": r["blobs"], "bytes": len(wire)}


@pytest.mark.gpu
@needs_node
def test_decoder_key_hash_option():
    """decode({keyHash: true}) (f4): every change also carries the GPU's XXH64 of its key bytes,
    equal to python-xxhash; the events are otherwise the reference's (ASCII keys go through the
    latin1 path, invalid UTF-8 keys still become U+FFFD strings like toString('utf-8'))."""
    import xxhash
    rng = random.Random(12)
    keys = [b"plain", "été".encode(), b"\xff\xfebad", b"x" * 40, b""]
    wire = b"".join(S.frame(S.change_payload(keys[i % len(keys)] + str(i).encode(), i, 0, 1, value=b"v"))
                    for i in range(500)) + S.random_stream(rng, 300)
    r, exp = oracle_events(wire)
    got = [e for e in run_js(wire, "65536", "keyhash") if e["t"] != "close"]
    assert got[-1]["t"] == "finish"
    for g, e in zip(got[:-1], exp):
        h = g.pop("keyHash", None)
        assert g == e
        if e["t"] == "change":
            assert h is not None
    # hashes of the raw key bytes (not of the decoded strings)
    hashes = [int(e["keyHash"]) for e in run_js(wire, "65536", "keyhash") if e["t"] == "change"]
    raw = []
    for k in range(r["nframes"]):
        if r["type"][k] & 0x3F == 1:
            po, ko, kl = int(r["payload_off"][k]), int(r["key_off"][k]), int(r["key_len"][k])
            raw.append(xxhash.xxh64_intdigest(wire[po + ko:po + ko + kl]))
    assert hashes == raw


@pytest.mark.gpu
@needs_node
def test_global_index_over_devices():
    """Streams sharded over the process's devices (index.js shard: contiguous blocks, as
    bench.py's C4 shards) each decode on their device ({device: k}); globalIndex() all-gathers
    the per-stream counters through libdrp's RCCL communicators (drp_index_allgather_host, one
    per device of this process) into every stream's global first-frame index. On a one-GPU box
    all shards land on device 0; the frame counts must equal the oracle's and the bases their
    prefix sums."""
    rng = random.Random(41)
    wires = [S.random_stream(rng, n, blob_p=0.05, blob_max=2000) for n in (300, 0, 1200, 57, 800)]
    code = r"""
var fs = require('fs'), p = require(%r)
var wires = JSON.parse(fs.readFileSync(process.argv[1])).map(function (h) { return Buffer.from(h, 'hex') })
var ndev = Math.max(1, p.devices())
var devs = p.shard(wires.length, ndev)
var decs = wires.map(function (w, i) { return p.decode({device: devs[i]}) })
var left = decs.length
decs.forEach(function (d, i) {
  d.on('finish', function () { if (--left === 0) done() })
  d.end(wires[i])
})
function done () {
  var g = p.globalIndex(decs, ndev)
  console.log(JSON.stringify({ndev: ndev, devs: devs, base: g.base, frames: g.frames,
    counts: decs.map(function (d) { return [d.changes, d.blobs] })}))
  process.exit(0)
}
""" % os.path.join(ROOT, "dat-replication-protocol_amd")
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump([w.hex() for w in wires], f)
        path = f.name
    try:
        # (the last line: RCCL may print its version banner first when NCCL_DEBUG is set)
        out = json.loads(subprocess.check_output([NODE, "-e", code, path], text=True, timeout=120).strip().splitlines()[-1])
    finally:
        os.unlink(path)
    frames = []
    for w, (ch, bl) in zip(wires, out["counts"]):
        r = O.decode_batch(w)
        assert (ch, bl) == (r["changes"], r["blobs"])
        frames.append(r["nframes"])
    assert out["frames"] == frames
    assert out["base"] == [sum(frames[:i]) for i in range(len(frames))]


@pytest.mark.gpu
@needs_node
def test_worker_threads_keep_their_own_state():
    """The addon's mutable state (pinned staging blocks, RCCL communicators) is per Node
    environment (drp_napi.c env_state): a worker_thread and the main thread decode (through
    pinned blocks) and all-gather at once, the worker exits (tearing down its environment), and
    the main thread decodes and all-gathers again with its own blocks and communicators."""
    rng = random.Random(43)
    wires = [S.c2_stream(40_000, seed=5).tobytes(), S.random_stream(rng, 2000, blob_p=0.05, blob_max=3000)]
    code = r"""
var fs = require('fs'), wt = require('worker_threads'), p = require(%r)
var path = wt.isMainThread ? process.argv[2] : wt.workerData.path
var wires = JSON.parse(fs.readFileSync(path)).map(function (h) { return Buffer.from(h, 'hex') })
function run (wire, cb) {
  var d = p.decode(), n = 0
  d.change(function (c, done) { n++; done() })
  d.blob(function (b, done) { b.resume(); b.on('end', done) })
  d.on('finish', function () {
    var g = p.globalIndex([d], 1)
    cb([n, d.blobs, g.frames[0]])
  })
  for (var o = 0; o < wire.length; o += 65536) d.write(wire.slice(o, o + 65536))
  d.end()
}
if (!wt.isMainThread) {
  run(wires[wt.workerData.i], function (r) { wt.parentPort.postMessage(r) })
} else {
  var out = {}
  var w = new wt.Worker(__filename, {workerData: {i: 1, path: path}})
  w.on('message', function (r) { out.worker = r })
  var left = 2
  w.on('exit', function () { if (--left === 0) after() })
  run(wires[0], function (r) { out.main = r; if (--left === 0) after() })
  function after () {
    run(wires[0], function (r) { out.again = r; console.log(JSON.stringify(out)); process.exit(0) })
  }
}
""" % os.path.join(ROOT, "dat-replication-protocol_amd")
    d = tempfile.mkdtemp()
    js, path = os.path.join(d, "wt.js"), os.path.join(d, "wires.json")
    open(js, "w").write(code)
    json.dump([w.hex() for w in wires], open(path, "w"))
    try:
        out = json.loads(subprocess.check_output([NODE, js, path], text=True, timeout=120).strip().splitlines()[-1])
    finally:
        shutil.rmtree(d)
    exp = []
    for w in wires:
        r = O.decode_batch(w)
        exp.append([r["changes"], r["blobs"], r["nframes"]])
    assert out == {"main": exp[0], "worker": exp[1], "again": exp[0]}


@pytest.mark.gpu
@needs_node
def test_encoder_input_policy():
    """Encoder.change validates synchronously, as messages.Change.encode throws inside change()
    (encode.js:102-117): key must be a string, change/from/to unsigned integers <= 2^53 - 1
    (JS Number range; the reference's varint@3 would write larger doubles inexactly), missing
    required fields throw; 2^53 - 1 is accepted. (GPU: the encoder opens its device context.)"""
    code = r"""
var enc = require(%r).encode()
var cases = [
  ['nokey', {change: 1, from: 0, to: 1}], ['numkey', {key: 5, change: 1, from: 0, to: 1}],
  ['neg', {key: 'k', change: -1, from: 0, to: 1}], ['frac', {key: 'k', change: 1.5, from: 0, to: 1}],
  ['big', {key: 'k', change: Math.pow(2, 53), from: 0, to: 1}], ['str', {key: 'k', change: '1', from: 0, to: 1}],
  ['nofrom', {key: 'k', change: 1, to: 1}], ['max', {key: 'k', change: Number.MAX_SAFE_INTEGER, from: 0, to: 1}]]
var out = {}
cases.forEach(function (c) {
  try { enc.change(c[1]); out[c[0]] = 'ok' } catch (e) { out[c[0]] = e.constructor.name + ': ' + e.message }
})
console.log(JSON.stringify(out))
process.exit(0)
""" % os.path.join(ROOT, "dat-replication-protocol_amd")
    out = json.loads(subprocess.check_output([NODE, "-e", code], text=True, timeout=60))
    assert out == {
        "nokey": "Error: key is required",
        "numkey": "TypeError: key must be a string",
        "neg": "RangeError: change must be an unsigned integer",
        "frac": "RangeError: change must be an unsigned integer",
        "big": "RangeError: change must be an unsigned integer",
        "str": "RangeError: change must be an unsigned integer",
        "nofrom": "Error: from is required",
        "max": "ok",
    }


# ---- the JS host layer on CPU: decode.js over the mock addon (tests/js/mock_native.js) ----------

@needs_node
@pytest.mark.parametrize("sizes,mode,batch", [("65536", "", None), ("3,7,64", "", None), ("1000", "async", None),
                                              ("1000,7", "", 4096), ("3,7,64", "async", 1024),
                                              ("509,1", "ticks", 3000), ("1", "", 64)])
def test_js_layer_events_match_oracle_cpu(sizes, mode, batch):
    """decode.js's batching, carry across batches (headers, Change frames, blobs cut by batch
    edges), double-buffered replay and _pending discipline, checked on CPU: the addon is replaced
    by a sequential restatement of drp_decode_stage's per-batch result, and the events must equal
    the oracle's one-write decode."""
    rng = random.Random(len(sizes) * 7 + (batch or 0))
    wire = S.random_stream(rng, 300 if sizes == "1" else 1200, blob_p=0.08, blob_max=3000, subset_p=0.3)
    r, exp = oracle_events(wire)
    got = [e for e in run_js(wire, sizes, mode, batch=batch, mock=True) if e["t"] != "close"]
    assert got[:-1] == exp
    assert got[-1] == {"t": "finish", "changes": r["changes"], "blobs": r["blobs"], "bytes": len(wire)}


@needs_node
def test_js_layer_batch_edges_cpu():
    """The crafted batch edges of test_decoder_batch_edges on CPU (mock addon)."""
    big = S.frame(S.change_payload(b"k" * 130, 300, 2**32 - 1, 5, value=bytes(range(256)) * 2, subset=b"s"))
    parts = [S.frame(S.change_payload(b"key%d" % i, i, 0, 1, value=b"v" * (i * 7 % 50))) for i in range(12)]
    wire = (parts[0] + parts[1] + big + parts[2] + S.frame(bytes(range(200)), 2) + parts[3] +
            S.frame(b"", 2) + parts[4] + big + b"".join(parts[5:]))
    r, exp = oracle_events(wire)
    for sizes in ["64", "5,59", "1,2,3,61", "130,1"]:
        for mode in ("", "async", "ticks"):
            got = [e for e in run_js(wire, sizes, mode, batch=64, mock=True) if e["t"] != "close"]
            assert got[:-1] == exp, (sizes, mode)
            assert got[-1] == {"t": "finish", "changes": r["changes"], "blobs": r["blobs"], "bytes": len(wire)}


@needs_node
@pytest.mark.parametrize("sizes,mode,batch", [("65536", "h2d", None), ("4093,1,65536", "h2d", 1 << 18),
                                              ("1000", "h2d", 4096)])
def test_js_layer_blob_pieces_are_write_slices_cpu(sizes, mode, batch):
    """SURVEY §8 f2 on CPU (mock addon): blob payloads reach the blob stream as slices of the
    written chunks, one piece per chunk a payload spans (decode.js:179-202 pushes each _write's
    part), never as slices of the coalesced batch copy; the events equal the oracle's."""
    wire = S.c3_stream(random.Random(5), 3, frames_per_unit=300, blob_len=200_000)
    r, exp = oracle_events(wire, digest=True)
    out = [e for e in run_js(wire, sizes, mode, batch=batch, mock=True) if e["t"] != "close"]
    tm = out.pop()
    assert out[:-1] == exp
    assert out[-1] == {"t": "finish", "changes": r["changes"], "blobs": r["blobs"], "bytes": len(wire)}
    assert tm["blobPieces"] > r["blobs"] and tm["blobPiecesShared"] == tm["blobPieces"], tm


@needs_node
def test_js_layer_errors_and_destroy_cpu():
    """Protocol errors end the stream after the frames before them, whatever the batching; a
    destroy() inside a change callback stops delivery (mock addon, CPU)."""
    good = bytes.fromhex("130112036b65791801200028013205") + b"hello"
    wire = good * 3 + b"\x03\x07ab" + good
    for batch in (None, 16):
        got = run_js(wire, "5", batch=batch, mock=True)
        assert [e["t"] for e in got] == ["change"] * 3 + ["error"], batch
        assert got[3]["message"] == "Protocol error, unknown type: 7"
    wire = S.c2_stream(3000, seed=3).tobytes()
    _, exp = oracle_events(wire)
    for sizes, batch, nth in [("65536", None, 37), ("1000", 4096, 1), ("300000", 65536, 2999)]:
        got = run_js(wire, sizes, "destroy", nth, batch=batch, mock=True)
        assert got[:nth] == exp[:nth] and got[nth:] == [{"t": "close"}], (sizes, batch)


@needs_node
def test_js_shard_assignment_cpu():
    """index.js shard(): contiguous device blocks differing by at most one stream, the same split
    as python/drp_dist.shard_range; the package loads without touching a GPU."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "dat-replication-protocol_amd", "python"))
    import drp_dist
    code = ("var p=require(%r); var out=[];"
            "[[10,3],[3,8],[8192,8],[8192,1],[0,4],[7,7],[100,6]].forEach(function(a){out.push(p.shard(a[0],a[1]))});"
            "console.log(JSON.stringify(out))" % os.path.join(ROOT, "dat-replication-protocol_amd"))
    out = json.loads(subprocess.check_output([NODE, "-e", code], text=True, timeout=60))
    for (n, d), got in zip([(10, 3), (3, 8), (8192, 8), (8192, 1), (0, 4), (7, 7), (100, 6)], out):
        exp = []
        for r in range(d):
            lo, hi = drp_dist.shard_range(n, d, r)
            exp += [r] * (hi - lo)
        assert got == exp, (n, d)


def _ack_cases():
    with open(os.path.join(ROOT, "tests", "golden", "ref_acks.json")) as f:
        return json.load(f)["cases"]


def run_acks(case, mock, piece=None):
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(bytes.fromhex(case["wire"]))
        path = f.name
    env = dict(os.environ)
    if mock:
        env["DRP_MOCK_NATIVE"] = "1"
    if piece:
        env["DRP_PIECE"] = str(piece)
    try:
        return json.loads(subprocess.check_output(
            [NODE, os.path.join(JS, "ack_order.js"), path, ",".join(map(str, case["sizes"])), case["pattern"]],
            text=True, timeout=120, env=env).strip().splitlines()[-1])
    finally:
        os.unlink(path)


@needs_node
@pytest.mark.parametrize("piece", [None, 1000])
def test_write_acks_follow_the_reference_cpu(piece):
    """The reference's write backpressure (decode.js:144-169): a write is acknowledged once the
    frames it completes are delivered and acknowledged, so write callbacks interleave with
    asynchronous change/blob handlers exactly as the reference's do (tests/golden/ref_acks.json,
    recorded from the reference itself by tests/golden/make_ack_fixtures.py), with writes read
    ahead into batches (DRP_PIECE=1000: many batches). JS layer over the CPU stand-in addon."""
    for case in _ack_cases():
        assert run_acks(case, mock=True, piece=piece) == case["log"], case["name"]


@pytest.mark.gpu
@needs_node
def test_write_acks_follow_the_reference():
    """As test_write_acks_follow_the_reference_cpu, through the addon and the GPU."""
    for case in _ack_cases():
        assert run_acks(case, mock=False) == case["log"], case["name"]


@needs_node
def test_high_water_mark_option():
    """decode() keeps MAX_BATCH (64 MiB) as its highWaterMark so a producer that honours write()
    runs far enough ahead to fill GPU batches (a documented divergence);
    decode({highWaterMark: 16384}) restores the reference's Writable default (decode.js:65), so
    write() returns false once 16 KiB are buffered. And the write queue never keeps a consumed
    write alive (300 distinct 64 KiB writes, each issued after the previous callback)."""
    out = json.loads(subprocess.check_output([NODE, os.path.join(JS, "hwm_queue.js"), "300", "65536"],
                                             text=True, timeout=120))
    assert out["defaultHwm"] == 64 * 1024 * 1024 and out["optionHwm"] == 16384
    assert out["writeReturns"][-1] is False, out["writeReturns"]  # (Node's Writable, as the reference's)
    assert out["retained"] == 0, out
    assert out["queueLength"] < 130, out
    assert out["changes"] > 300 * 1000, out


def _throw_cases():
    with open(os.path.join(ROOT, "tests", "golden", "ref_throws.json")) as f:
        return json.load(f)["cases"]


def run_throws(case, mock):
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(bytes.fromhex(case["wire"]))
        path = f.name
    env = dict(os.environ)
    if mock:
        env["DRP_MOCK_NATIVE"] = "1"
    try:
        return json.loads(subprocess.check_output(
            [NODE, os.path.join(JS, "throw_order.js"), path, ",".join(map(str, case["sizes"])), case["pattern"]],
            text=True, timeout=120, env=env).strip().splitlines()[-1])
    finally:
        os.unlink(path)


def _same_surfacing(got, want, name):
    """Equal logs, except that where the reference throws out of write() (the write whose bytes hold
    the rejected Change was decoded synchronously inside it), the package's exception leaves the
    GPU batch's completion callback instead: a write's bytes are decoded after write() returns."""
    assert len(got) == len(want), (name, got, want)
    for g, w in zip(got, want):
        if w.startswith("throw") and not w.startswith("throw-end") and g.startswith("uncaught:"):
            assert g.split(":", 1)[1] == w.split(":", 1)[1], (name, g, w)
        else:
            assert g == w, (name, got, want)


@needs_node
def test_codec_throw_surfaces_as_in_the_reference_cpu():
    """A Change the codec rejects (a missing required field) surfaces as the reference's
    Change.decode throw does (tests/golden/ref_throws.json, recorded from the reference with a
    strict codec shim): the same frames delivered and acknowledged before it, the same message,
    thrown out of the handler callback that resumed delivery, no 'error' or 'close' event, nothing
    delivered after it. JS layer over the CPU stand-in addon."""
    for case in _throw_cases():
        _same_surfacing(run_throws(case, mock=True), case["log"], case["name"])


@pytest.mark.gpu
@needs_node
def test_codec_throw_surfaces_as_in_the_reference():
    """As test_codec_throw_surfaces_as_in_the_reference_cpu, through the addon and the GPU."""
    for case in _throw_cases():
        _same_surfacing(run_throws(case, mock=False), case["log"], case["name"])
