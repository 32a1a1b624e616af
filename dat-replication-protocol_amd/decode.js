// Decoder: the reference's streaming decode API (decode.js:63-142 of
// mafintosh/dat-replication-protocol v4.1.2) over the gfx950 batch codec.
//
// Writes reach _write one at a time, as in the reference; the ones buffered behind the write
// being consumed (the stream's highWaterMark is MAX_BATCH unless opts.highWaterMark says otherwise) are read ahead: up to PIECE bytes of
// them form a batch, decoded on the GPU in one call on a worker thread (frame split + Change
// decode, libdrp via lib/drp.node, the written chunks handed over as they are: libdrp gathers
// the ranges it stages, so nothing is concatenated here). While one batch is replayed the next
// is decoded. The replay keeps the reference's discipline exactly: a frame is delivered while
// the write holding its last byte is consumed, a change/blob callback increments _pending and
// delivery stops while _pending > 0 (decode.js:89-99, 144-169), and a write's callback fires
// once every frame it completes has been delivered and acknowledged (decode.js:167-168), so
// the callbacks interleave as they do there (write()'s return value: opts.highWaterMark below).
//
// Carry across batches (decode.js:75-81): an incomplete header (<= 10 bytes) is prepended to
// the next batch; an incomplete Change frame is collected once into a buffer of its declared
// size (as _onchangedata fills _buffer, decode.js:229-247) and decoded when complete; the
// bytes of an open blob continue through the next batch as pass-through (never sent to HBM).
// Change values and blob pieces are slices of the written chunks (decode.js:179-202, 205-214
// slice the chunk they were given); only a frame that straddles two writes is copied.
'use strict'

var stream = require('stream')
var util = require('util')
var native = require('./native')

var FLUSH = Buffer.from([0]) // identity-compared end sentinel (decode.js:6, :125)
var MAX_BATCH = Number(process.env.DRP_MAX_BATCH) || 64 * 1024 * 1024 // bytes written ahead
var PIECE = Math.min(MAX_BATCH, Number(process.env.DRP_PIECE) || 16 * 1024 * 1024) // bytes per GPU call
var FIRST_PIECE = 1024 * 1024 // the first batch after the decoder ran dry
var MAX_FRAME = require('buffer').constants.MAX_LENGTH

var TYPE_MASK = 0x3f
var CONT = 0x40
var PARTIAL = 0x80
var KEY_ASCII = 0x10 // key flags, only set when key post-processing is on
var TAIL_HEADER = 1
var TAIL_CHANGE = 2

// --- blob payload stream handed to the user's blob handler (decode.js:8-48) ---------
function BlobStream (parent) {
  stream.Readable.call(this)
  this.destroyed = false
  this._parent = parent
  this._drain = null
  this.on('end', this._read)
}
util.inherits(BlobStream, stream.Readable)

BlobStream.prototype.destroy = function (err) {
  if (this.destroyed) return
  this.destroyed = true
  if (err) this.emit('error', err)
  this.emit('close')
  this._parent.destroy()
}

BlobStream.prototype._push = function (data, cb) {
  if (this.push(data)) return cb()
  var prev = this._drain
  this._drain = prev ? function () { prev(); cb() } : cb
}

BlobStream.prototype._end = function () {
  this.push(null)
}

BlobStream.prototype._read = function () {
  var fn = this._drain
  this._drain = null
  if (fn) fn()
}

// --- default handlers (decode.js:50-61) -------------------------------------------
function noopFinalize (cb) { cb() }
function noopChange (change, cb) { cb() }
function drainBlob (blob, cb) { blob.resume(); cb() }

var ERRORS = {
  1: function (d) { return 'Protocol error, unknown type: ' + d },
  2: function (d) { return 'Protocol error, zero length for type: ' + d },
  3: function () { return 'Protocol error, invalid length varint' },
  4: function () { return 'Protocol error, malformed change message' },
  5: function () { return 'Decoded message is not valid' }
}

// the decode result of a batch that needs no GPU call (its bytes only fill a carried frame)
var NOTHING = { n: 0, errCode: 0, tailKind: 0, consumed: 0, blobRemaining: 0, frameBytes: 0 }

// opts (not in the reference, whose constructor takes none):
//   keyHash: true  - every change object also carries keyHash, the XXH64 of its key bytes as
//                    a BigInt, computed on the GPU (drp_keys.hip)
//   device: k      - the GPU this stream decodes on (default: DRP_DEVICE or 0); independent
//                    streams are spread over a node's GPUs this way (index.js: shard)
//   codecErrors    - 'event': a Change the codec rejects destroys the stream with an 'error'
//                    event; by default it is thrown, as the reference's Change.decode throws
//                    (decode.js:210): out of write() or the handler callback that led to it
//   highWaterMark  - the Writable's highWaterMark. Default MAX_BATCH (64 MiB), a deliberate
//                    divergence from the reference (Node's default, 16 KiB): a producer that
//                    honours write()'s return value stops at the highWaterMark, and the writes
//                    buffered behind the one being consumed are all a GPU batch can read ahead.
//                    16384 restores the reference's write()/'drain' signal (batches then hold
//                    ~one write each; INTEGRATION.md)
function Decoder (opts) {
  if (!(this instanceof Decoder)) return new Decoder(opts)
  var hwm = opts && opts.highWaterMark !== undefined ? opts.highWaterMark : MAX_BATCH
  stream.Writable.call(this, { highWaterMark: hwm })
  // a Change the codec rejects: thrown, as the reference's Change.decode throws (default), or
  // emitted as an 'error' event that destroys the stream (opts.codecErrors === 'event')
  this._codecEvents = !!(opts && opts.codecErrors === 'event')
  this._broken = false
  this._keyPost = !!(opts && opts.keyHash)

  this.destroyed = false
  this.bytes = 0
  this.changes = 0
  this.blobs = 0

  this._pending = 0
  this._paused = false    // delivery stopped at a callback that has not been acknowledged

  this._onchange = noopChange
  this._onblob = drainBlob
  this._onfinalize = noopFinalize

  this._ctx = native.context(opts && opts.device)
  // read-ahead: the write being consumed and the stream's buffered writes behind it
  this._cw = null         // the write being consumed (_write's chunk) and its callback
  this._wcb = null
  this._slots = []        // writes whose last byte is in a batch, not yet consumed: {chunk, batch, end}
  this._q = []            // written chunks; [_qh, ...) not yet taken by _write
  this._qh = 0
  this._taken = 0         // of those, how many are already placed (whole or in part) in batches
  this._rest = null       // the part of a write not yet in a batch: {chunk, off}
  this._batches = []      // formed batches in order; [0] is the one delivered from
  this._inflight = null   // the batch on the GPU (worker thread)
  this._halt = false      // a batch ended in an error: nothing after it is decoded
  this._carry = null      // an incomplete frame header (<= 10 bytes)
  this._partial = null    // an incomplete Change frame of known size: {buf, filled}
  this._blobLeft = 0      // payload bytes of the open blob still to come
  this._blob = null       // the open BlobStream
  // delivery position in _batches[0]
  this._next = 0          // next frame
  this._ck = 0            // chunk holding the bytes delivered next
  this._blobPos = -1      // batch offset of the next piece of a blob row being delivered
  // ms, summed; bytes staged into HBM, blob payload bytes left in host memory, bytes copied on
  // the host (gathered for HBM, frames straddling two writes, carried frames)
  this.timing = { batches: 0, h2d: 0, gpu: 0, d2h: 0, convert: 0, replay: 0, h2dBytes: 0, h2dSkipped: 0, hostCopied: 0, d2hMax: 0, pinnedBatches: 0 }

  var self = this
  this._up = function () {
    self._pending++
    return self._down
  }
  this._down = function () {
    if (--self._pending > 0 || !self._paused) return
    self._paused = false
    self._deliver()
  }
  this._scheduled = false
  this._formFn = function () {
    self._scheduled = false
    self._form()
    self._deliver() // (a batch that only filled a carried frame needs no GPU call)
  }
}
util.inherits(Decoder, stream.Writable)

Decoder.prototype.destroy = function (err) {
  if (this.destroyed) return
  this.destroyed = true
  if (this._blob) this._blob.destroy()
  if (err) this.emit('error', err)
  this.emit('close')
}

Decoder.prototype.change = function (fn) { this._onchange = fn }
Decoder.prototype.blob = function (fn) { this._onblob = fn }
Decoder.prototype.finalize = function (fn) { this._onfinalize = fn }

Decoder.prototype._write = function (data, enc, cb) {
  var q = this._q
  // (taken slots are cleared at once: the queue must not keep consumed writes alive)
  while (this._qh < q.length && q[this._qh] !== data) q[this._qh++] = undefined // (chunks the stream refused)
  if (this._qh < q.length) q[this._qh++] = undefined
  if (this._qh >= 64 && this._qh * 2 > q.length) {
    this._q = q.slice(this._qh)
    this._qh = 0
  }
  if (data === FLUSH) { // every write before it has been consumed (decode.js:121-124)
    this._onfinalize(cb)
    return
  }
  this.bytes += data.length
  this._cw = data
  this._wcb = cb
  if (this._taken > 0) {
    this._taken-- // (read ahead into a batch already)
  } else {
    // not read ahead: a batch from it and the writes made in the same turn of the event loop
    // (a producer writes its next chunks right after this call returns)
    this._rest = { chunk: data, off: 0 }
    if (!this._scheduled) {
      this._scheduled = true
      setImmediate(this._formFn)
    }
  }
  this._deliver()
}

Decoder.prototype.end = function (data, enc, cb) {
  if (typeof data === 'function') return this.end(null, null, data)
  if (typeof enc === 'function') return this.end(data, null, enc)
  if (data) this.write(data)
  this.write(FLUSH)
  stream.Writable.prototype.end.call(this, cb)
}

// Every written chunk is also queued here (write() below) until _write takes it: the writes
// behind the one being consumed are read ahead from this queue, not from the stream's internals.
Decoder.prototype.write = function (chunk, enc, cb) {
  if (typeof chunk === 'string') chunk = Buffer.from(chunk, typeof enc === 'string' ? enc : 'utf8')
  else if (chunk instanceof Uint8Array && !Buffer.isBuffer(chunk)) {
    chunk = Buffer.from(chunk.buffer, chunk.byteOffset, chunk.byteLength)
  }
  if (Buffer.isBuffer(chunk) && !this._writableState.ended && !this.destroyed) this._q.push(chunk)
  return stream.Writable.prototype.write.call(this, chunk, typeof enc === 'string' ? null : enc, cb)
}

Decoder.prototype._bufferedFirst = function () {
  return this._q[this._qh]
}

Decoder.prototype._bufferedNext = function () {
  return this._q[this._qh + this._taken]
}

// Form the next batch: up to PIECE bytes of the unplaced writes (the rest of a write cut at a
// batch edge, then the buffered writes in order), behind the carry of the batch before, and hand
// it to the GPU. One batch is on the GPU at a time (the next one's carry depends on it).
Decoder.prototype._form = function () {
  if (this._inflight || this._halt || this.destroyed) return
  var segs = [] // {chunk, a, b, write}: bytes [a, b) of a written chunk; write: its last byte is here
  var size = 0
  // a decoder with nothing decoded to replay starts with a small batch, so its callbacks start
  // after a short GPU call; the batches behind it are decoded while it is replayed
  var piece = this._batches.length ? PIECE : Math.min(PIECE, FIRST_PIECE)
  while (size < piece) {
    var r = this._rest
    if (!r) {
      var e = this._bufferedNext()
      if (!e || e === FLUSH) break
      this._taken++
      r = this._rest = { chunk: e, off: 0 }
    }
    var take = Math.min(r.chunk.length - r.off, piece - size)
    var last = r.off + take === r.chunk.length
    segs.push({ chunk: r.chunk, a: r.off, b: r.off + take, write: last, first: r.off === 0 })
    size += take
    if (last) this._rest = null
    else r.off += take
  }
  if (!segs.length) return
  var chunks = []
  var starts = []
  var at = 0
  var slots = []
  var first = [] // the writes whose first byte is in this batch
  for (var q = 0; q < segs.length; q++) if (segs[q].first) first.push(segs[q].chunk)
  var p = this._partial
  var i = 0
  if (p) {
    // collect the rest of a Change frame of known size: each byte is copied once (a write that
    // ends inside it ends at its position in that frame's buffer, the batch's first chunk)
    while (i < segs.length && p.filled < p.buf.length) {
      var s = segs[i]
      var n = Math.min(s.b - s.a, p.buf.length - p.filled)
      s.chunk.copy(p.buf, p.filled, s.a, s.a + n)
      p.filled += n
      this.timing.hostCopied += n
      s.a += n
      if (s.a < s.b) break // (the frame ends inside this segment; the rest follows it)
      if (s.write) slots.push({ chunk: s.chunk, end: p.filled })
      i++
    }
    if (p.filled < p.buf.length) { // nothing to decode yet: these writes only fill the frame
      this._queueBatch({ chunks: [], starts: [], size: 0, res: NOTHING, tooBig: 0, first: first }, slots)
      return this._form()
    }
    this._partial = null
    chunks.push(p.buf)
    starts.push(0)
    at = p.buf.length
  } else if (this._carry) {
    chunks.push(this._carry)
    starts.push(0)
    at = this._carry.length
    this._carry = null
  }
  for (; i < segs.length; i++) {
    var g = segs[i]
    if (g.b > g.a) {
      chunks.push(g.a === 0 && g.b === g.chunk.length ? g.chunk : g.chunk.slice(g.a, g.b)) // (slices: no copy)
      starts.push(at)
      at += g.b - g.a
    }
    if (g.write) slots.push({ chunk: g.chunk, end: at })
  }
  var batch = { chunks: chunks, starts: starts, size: at, res: null, tooBig: 0, first: first }
  this._queueBatch(batch, slots)
  this._inflight = batch
  var self = this
  native.decode(this._ctx, chunks.length === 1 ? chunks[0] : chunks, this._blobLeft, function (err, res) {
    self._ondecoded(err, res, batch)
  }, this._keyPost)
}

Decoder.prototype._queueBatch = function (batch, slots) {
  this._batches.push(batch)
  for (var k = 0; k < slots.length; k++) {
    slots[k].batch = batch
    this._slots.push(slots[k])
  }
}

Decoder.prototype._ondecoded = function (err, res, batch) {
  this._inflight = null
  if (this.destroyed) return
  if (err) return this.destroy(err)
  // the carry into the next batch (decode.js:75-81) is known now, before the replay
  var tooBig = 0
  if (!res.errCode) {
    var rest = batch.size - res.consumed
    if (res.tailKind === TAIL_HEADER) {
      this._carry = this._gather(batch, res.consumed, batch.size) // copied, as into _header
    } else if (res.tailKind === TAIL_CHANGE) {
      if (res.frameBytes > MAX_FRAME) {
        tooBig = res.frameBytes // reported after the frames before it (the reference throws)
      } else {
        var buf = Buffer.allocUnsafe(res.frameBytes) // decode.js:227 allocates _buffer the same way
        this._copyOut(batch, res.consumed, batch.size, buf, 0)
        this._partial = { buf: buf, filled: rest }
      }
    }
  }
  this._blobLeft = res.blobRemaining
  if (res.errCode || tooBig) this._halt = true
  var t = res.t
  if (t) {
    var tm = this.timing
    tm.batches++
    tm.h2d += t.h2d
    tm.gpu += t.gpu
    tm.d2h += t.d2h
    if (t.d2h > tm.d2hMax) tm.d2hMax = t.d2h
    tm.pinnedBatches += t.pinnedColumns || 0
    tm.convert += t.convert
    tm.h2dBytes += t.h2dBytes || 0
    tm.h2dSkipped += t.h2dSkipped || 0
    tm.hostCopied += t.hostCopied || 0
  }
  batch.res = res
  batch.tooBig = tooBig
  this._form() // the next batch goes to the GPU before this one's callbacks run
  this._deliver()
}

// bytes [a, b) of a batch into dst at d (they may span chunks)
Decoder.prototype._copyOut = function (batch, a, b, dst, d) {
  var chunks = batch.chunks
  var starts = batch.starts
  var k = 0
  while (k + 1 < chunks.length && starts[k + 1] <= a) k++
  this.timing.hostCopied += b - a
  for (; a < b; k++) {
    var n = Math.min(b, starts[k] + chunks[k].length) - a
    chunks[k].copy(dst, d, a - starts[k], a - starts[k] + n)
    d += n
    a += n
  }
}

Decoder.prototype._gather = function (batch, a, b) {
  var out = Buffer.allocUnsafe(b - a)
  this._copyOut(batch, a, b, out, 0)
  return out
}

// Deliver frames of the front batch while no callback is outstanding, up to the end of the
// write being consumed; then acknowledge that write (decode.js:144-169).
Decoder.prototype._deliver = function () {
  if (this._broken) return // (a codec exception was thrown: see _replay)
  while (!this.destroyed && this._pending <= 0) {
    var batch = this._batches[0]
    var slot = this._slots[0]
    if (!this._cw) return // (no write being consumed: wait for _write)
    if (slot && slot.chunk === this._cw && slot.batch === batch && batch && batch.res) {
      if (!this._replay(batch, slot.end)) return
      // every frame the write completes has been delivered and acknowledged; its callback lets
      // the stream hand over the next buffered write at once, whose frames the reference then
      // delivers before this callback returns: so that batch must be decoded first
      if (this._nextOnGpu()) return // (resumed by _ondecoded)
      this._slots.shift()
      var cb = this._wcb
      this._cw = null
      this._wcb = null
      cb()
      return
    }
    if (!batch || !batch.res) return // (the write's frames are still on the GPU)
    // the write ends in a later batch: this one is delivered whole
    if (!this._replay(batch, Infinity)) return
    this._retire()
  }
}

// Is the first byte of the next buffered write still on its way (not yet decoded)?
Decoder.prototype._nextOnGpu = function () {
  if (this._halt) return false
  var e = this._bufferedFirst()
  if (!e || e === FLUSH) return false
  if (this._taken === 0) this._form() // (not read ahead yet: now)
  if (this._taken === 0) return true // (behind the batch on the GPU)
  var b = this._inflight
  return b !== null && b.first.indexOf(e) >= 0
}

Decoder.prototype._retire = function () {
  this._batches.shift()
  this._next = 0
  this._ck = 0
  this._blobPos = -1
}

// Deliver the batch's frames completed before batch offset `lim` (the end of the write being
// consumed). false: stopped at a callback not yet acknowledged, or the stream ended.
// Change frames are built inline (the hot loop: one object, one key string, one value slice per
// frame); keys the GPU flagged ASCII are substrings of the batch's key text (res.keyText: those
// keys end to end, made by the addon; the same string buf.toString('utf8', ...) would give,
// without a UTF-8 decode and a native call per key).
Decoder.prototype._replay = function (batch, lim) {
  var res = batch.res
  var n = res.n
  var type = res.type
  var off = res.off
  var len = res.len
  var flags = res.flags
  var ko = res.ko
  var kl = res.kl
  var so = res.so
  var sl = res.sl
  var vcol = res.vo
  var vl = res.vl
  var cc = res.change
  var cf = res.from
  var ct = res.to
  var keyHash = res.keyHash
  var keyText = typeof res.keyText === 'string' ? res.keyText : null
  var kp = res.kp
  var chunks = batch.chunks
  var starts = batch.starts
  var down = this._down
  var i = this._next
  var k = this._ck
  var t0 = process.hrtime()
  while (i < n && this._pending <= 0) {
    var o = off[i]
    if ((type[i] & TYPE_MASK) !== 1) {
      if (o > lim) break // (its header ends in a later write)
      this._next = i
      this._ck = k
      var r = this._deliverBlob(batch, i, lim)
      if (this._ck > k) k = this._ck
      if (r === 0) break // (the next piece is in a later write)
      if (r === 2) i++
      if (this.destroyed) break
      continue
    }
    var e = o + len[i]
    if (e > lim) break // (its last byte is in a later write)
    // messages.Change.decode result shape: {subset, key, change, from, to, value}
    while (k + 1 < chunks.length && starts[k + 1] <= o) k++
    var c = chunks[k]
    var base = starts[k]
    var inChunk = e <= base + c.length
    if (!inChunk) { // (the frame straddles two writes: its payload is copied once)
      c = this._gather(batch, o, e)
      base = o
    }
    var f = flags[i]
    var k0 = o + ko[i] - base
    var k1 = k0 + kl[i]
    var v0 = o + vcol[i] - base
    var key
    if (keyText !== null && (f & KEY_ASCII)) {
      key = keyText.substring(kp[i], kp[i] + kl[i])
    } else {
      key = c.toString('utf8', k0, k1)
    }
    var change = {
      subset: (f & 1) ? c.toString('utf8', o + so[i] - base, o + so[i] - base + sl[i]) : '',
      key: key,
      change: cc[i],
      from: cf[i],
      to: ct[i],
      value: (f & 2) ? c.slice(v0, v0 + vl[i]) : null
    }
    if (keyHash) change.keyHash = keyHash[i]
    this.changes++
    this._pending++ // released by the handler's cb (_up, decode.js:89-93)
    this._onchange(change, down) // (nothing it calls re-enters this loop: _down only resumes a paused replay)
    i++
    if (this.destroyed) break
  }
  this._next = i
  this._ck = k
  var dt = process.hrtime(t0)
  this.timing.replay += dt[0] * 1e3 + dt[1] * 1e-6
  if (this.destroyed) return false
  if (this._pending > 0) {
    this._paused = true // resumed by _down
    return false
  }
  if (i < n) return true // (the rest completes in later writes)
  if (res.errCode && this._errPos(batch) < lim) {
    var err = new Error(ERRORS[res.errCode](res.errDetail))
    if ((res.errCode === 4 || res.errCode === 5) && !this._codecEvents) {
      // a Change the codec rejects: messages.Change.decode throws inside the reference's
      // _onchangeend (decode.js:205-214), so the exception leaves whatever drove the delivery
      // (the write() that handed the bytes over, or the handler's callback that resumed it; here
      // also the GPU batch's completion) and the stream is left as it was: nothing more is
      // delivered and no event is emitted (tests/golden/ref_throws.json, recorded from the reference)
      this._halt = true
      this._broken = true
      throw err
    }
    this.destroy(err)
    return false
  }
  if (batch.tooBig && batch.size <= lim) {
    this.destroy(new RangeError('Change frame of ' + batch.tooBig + ' bytes exceeds the maximum Buffer size'))
    return false
  }
  return true
}

// where a batch's protocol error is met: past its last delivered frame (the malformed Change
// itself when the error is in a Change payload)
Decoder.prototype._errPos = function (batch) {
  var res = batch.res
  var n = res.n
  var bad = res.errCode === 4 || res.errCode === 5
  if (bad) return res.off[n] + res.len[n] - 1
  return n ? res.off[n - 1] + Math.min(res.len[n - 1], batch.size - res.off[n - 1]) : 0
}

// One piece of blob frame i (or of the continuation of one opened in an earlier batch): the
// part of its payload inside the next written chunk, pushed as a slice of that chunk with one
// callback, as _onblobdata pushes each chunk's part (decode.js:179-202). 2: the frame's last
// piece is delivered (and the blob ended, unless it continues past the batch); 1: a piece was
// delivered; 0: the next piece lies in a later write.
Decoder.prototype._deliverBlob = function (batch, i, lim) {
  var res = batch.res
  var type = res.type[i]
  var off = res.off[i]
  var end = off + Math.min(res.len[i], batch.size - off)
  var pos = this._blobPos
  if (pos < 0) {
    pos = off
    if (!(type & CONT)) {
      this.blobs++
      this._blob = new BlobStream(this)
      this._onblob(this._blob, this._down) // (its cb balances the _pending++ at the blob's end)
    }
  }
  if (pos < end && pos >= lim) {
    this._blobPos = pos
    return 0
  }
  var chunks = batch.chunks
  var starts = batch.starts
  var k = this._ck
  while (k + 1 < chunks.length && starts[k + 1] <= pos) k++
  this._ck = k
  var stop = Math.min(end, starts[k] + chunks[k].length)
  var data = pos < stop ? chunks[k].slice(pos - starts[k], stop - starts[k]) : Buffer.alloc(0)
  var blob = this._blob
  var last = stop >= end
  this._blobPos = last ? -1 : stop
  blob._push(data, this._up())
  if (!last) return 1
  if (!(type & PARTIAL)) { // decode.js:171-177
    this._pending++ // released by the blob handler's cb
    this._blob = null
    blob._end()
  }
  return 2
}

module.exports = Decoder
