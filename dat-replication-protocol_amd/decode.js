// Decoder: the reference's streaming decode API (decode.js:63-142 of
// mafintosh/dat-replication-protocol v4.1.2) over the gfx950 batch codec.
//
// Writes are coalesced (everything written before the event loop comes round again, up to
// MAX_BATCH bytes) and decoded on the GPU in one call on a worker thread (frame split +
// Change decode, libdrp via lib/drp.node). The returned frame table is replayed here with the
// reference's callback discipline: a change/blob callback increments _pending, and replay stops
// while _pending > 0 and resumes from _down (decode.js:89-99, 144-169). The event sequence is
// the reference's; only the timing of write callbacks differs (a write below the batch
// threshold is acknowledged when queued; one that fills a batch when that batch has been
// delivered, which is the backpressure).
//
// Carry across batches (decode.js:75-81): an incomplete header (<= 10 bytes) is prepended to
// the next batch; an incomplete Change frame is collected once into a buffer of its declared
// size (as _onchangedata fills _buffer, decode.js:229-247) and decoded when complete; the
// bytes of an open blob continue through the next batch as pass-through (never sent to HBM).
'use strict'

var stream = require('stream')
var util = require('util')
var native = require('./native')

var FLUSH = Buffer.from([0]) // identity-compared end sentinel (decode.js:6, :125)
var MAX_BATCH = Number(process.env.DRP_MAX_BATCH) || 64 * 1024 * 1024
var PIECE = Number(process.env.DRP_PIECE) || 16 * 1024 * 1024 // bytes per GPU call
var MAX_FRAME = require('buffer').constants.MAX_LENGTH

// a batch whose frames average at most TEXT_PER_FRAME bytes is turned into one latin1 string
// for its ASCII keys (cheaper than a string per key); larger frames keep one string per key
var TEXT_PER_FRAME = 512
var TEXT_MAX = 256 * 1024 * 1024 // (below V8's string length limit)
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

// The chunks of a batch in one buffer: a page-locked staging block from the addon when one is
// free (the GPU copy then runs by DMA at the PCIe rate), else ordinary memory. The block is not
// reused while any slice of this batch is alive (native.js / drp_napi.c pinnedBuffer).
function coalesce (chunks) {
  var total = 0
  for (var i = 0; i < chunks.length; i++) total += chunks[i].length
  var out = native.pinnedBuffer ? native.pinnedBuffer(total) : null
  if (out === null) return Buffer.concat(chunks, total)
  for (var j = 0, at = 0; j < chunks.length; j++) at += chunks[j].copy(out, at)
  return out
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

// opts (not in the reference, whose constructor takes none):
//   keyHash: true  - every change object also carries keyHash, the XXH64 of its key bytes as
//                    a BigInt, computed on the GPU (drp_keys.hip)
//   device: k      - the GPU this stream decodes on (default: DRP_DEVICE or 0); independent
//                    streams are spread over a node's GPUs this way (index.js: shard)
function Decoder (opts) {
  if (!(this instanceof Decoder)) return new Decoder(opts)
  stream.Writable.call(this)
  this._keyPost = !!(opts && opts.keyHash)

  this.destroyed = false
  this.bytes = 0
  this.changes = 0
  this.blobs = 0

  this._pending = 0
  this._paused = false    // replay stopped at a callback that has not been acknowledged

  this._onchange = noopChange
  this._onblob = drainBlob
  this._onfinalize = noopFinalize

  this._ctx = native.context(opts && opts.device)
  this._queue = []        // written chunks not yet handed to the GPU
  this._queued = 0
  this._scheduled = false
  this._inflight = false  // a batch is on the GPU (worker thread)
  this._ready = null      // a decoded batch waiting for the one being replayed
  this._halt = false      // a batch ended in an error: nothing after it is decoded
  this._held = null       // write callback held back until its batch is on the GPU
  this._final = null      // end(): finalize once everything before it is delivered
  this._carry = null      // an incomplete frame header (<= 10 bytes)
  this._partial = null    // an incomplete Change frame of known size: {buf, filled}
  this._blobLeft = 0      // payload bytes of the open blob still to come
  this._blob = null       // the open BlobStream
  this._res = null        // decoded batch being replayed
  this._buf = null        // its bytes
  this._chunks = null     // the written chunks it was made of, and where each starts in it
  this._starts = null
  this._ck = 0            // the chunk holding the blob bytes delivered next
  this._blobPos = -1      // batch offset of the next piece of a blob row being delivered
  this._text = null       // its bytes as one latin1 string (ASCII keys are cut from it)
  this._tooBig = 0        // its carried Change frame was larger than a Buffer can hold
  this._next = 0          // next frame to deliver
  // ms, summed (and the bytes staged into HBM / blob payload bytes that stayed in host memory)
  this.timing = { batches: 0, h2d: 0, gpu: 0, d2h: 0, convert: 0, replay: 0, h2dBytes: 0, h2dSkipped: 0 }

  var self = this
  this._up = function () {
    self._pending++
    return self._down
  }
  this._down = function () {
    if (--self._pending > 0 || !self._paused) return
    self._paused = false
    self._replay()
  }
  this._kickFn = function () {
    self._scheduled = false
    self._kick()
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
  if (data === FLUSH) {
    this._final = cb
    return this._kick()
  }
  this.bytes += data.length
  this._queue.push(data)
  this._queued += data.length
  if (this._queued >= MAX_BATCH) {
    // backpressure: acknowledged once every queued byte has been handed to the GPU (_kick), so at
    // most one batch on the GPU, one decoded and waiting, one replaying and MAX_BATCH queued bytes
    // are held in memory at a time
    this._held = cb
    return this._kick()
  }
  cb()
  if (!this._scheduled) {
    this._scheduled = true
    setImmediate(this._kickFn)
  }
}

Decoder.prototype.end = function (data, enc, cb) {
  if (typeof data === 'function') return this.end(null, null, data)
  if (typeof enc === 'function') return this.end(data, null, enc)
  if (data) this.write(data)
  this.write(FLUSH)
  stream.Writable.prototype.end.call(this, cb)
}

// Hand the queued bytes to the GPU (one batch), or finish when nothing is left. At most one
// batch is on the GPU and one waits decoded while another is replayed: batch k + 1 is split and
// decoded on the worker thread while batch k's callbacks run here.
Decoder.prototype._kick = function () {
  if (this._inflight || this._ready || this._halt || this.destroyed) return
  if (!this._queued) {
    var held = this._held
    this._held = null
    if (held) held()
    if (this._final && !this._queued && !this._res && !this._inflight) {
      var fin = this._final
      this._final = null
      this._onfinalize(fin) // decode.js:125-128
    }
    return
  }
  // at most PIECE bytes go to the GPU at a time (a big write is cut into pieces, so the decode of
  // piece k + 1 overlaps the replay of piece k); the rest stays queued
  var chunks = this._queue
  if (this._queued <= PIECE) {
    this._queue = []
    this._queued = 0
  } else {
    var took = 0
    var k = 0
    while (took < PIECE) took += chunks[k++].length
    var last = chunks[k - 1]
    var over = took - PIECE
    this._queue = chunks.slice(k)
    if (over > 0) { // (slices share the write's memory: no copy)
      chunks[k - 1] = last.slice(0, last.length - over)
      this._queue.unshift(last.slice(last.length - over))
    }
    chunks = chunks.slice(0, k)
    this._queued -= PIECE
  }
  var p = this._partial
  if (p) {
    // collect the rest of a Change frame of known size: each byte is copied once
    var k = 0
    while (k < chunks.length && p.filled < p.buf.length) {
      var c = chunks[k]
      var take = Math.min(c.length, p.buf.length - p.filled)
      c.copy(p.buf, p.filled, 0, take)
      p.filled += take
      if (take < c.length) chunks[k] = c.slice(take)
      else k++
    }
    if (p.filled < p.buf.length) return this._kick() // nothing else to decode yet (or the rest of the queue)
    this._partial = null
    chunks = [p.buf].concat(chunks.slice(k))
  } else if (this._carry) {
    chunks.unshift(this._carry)
    this._carry = null
  }
  var batch = chunks.length === 1 ? chunks[0] : coalesce(chunks)
  // where each chunk starts in the batch: blob payloads are delivered as slices of the written
  // chunks themselves (decode.js:179-202 slices the chunk it was given), not of the batch copy
  var starts = new Array(chunks.length)
  for (var j = 0, at = 0; j < chunks.length; j++) {
    starts[j] = at
    at += chunks[j].length
  }
  this._inflight = true
  var held = this._queued ? null : this._held // all of its bytes are on their way to the GPU now
  if (held) this._held = null
  var self = this
  native.decode(this._ctx, batch, this._blobLeft, function (err, res) {
    self._ondecoded(err, res, batch, chunks, starts)
  }, this._keyPost)
  if (held) held()
}

Decoder.prototype._ondecoded = function (err, res, batch, chunks, starts) {
  this._inflight = false
  if (this.destroyed) return
  if (err) return this.destroy(err)
  // the carry into the next batch (decode.js:75-81) is known now, before the replay
  var tooBig = 0
  if (!res.errCode) {
    var rest = batch.length - res.consumed
    if (res.tailKind === TAIL_HEADER) {
      this._carry = Buffer.from(batch.slice(res.consumed)) // copied, as into _header
    } else if (res.tailKind === TAIL_CHANGE) {
      if (res.frameBytes > MAX_FRAME) {
        tooBig = res.frameBytes // reported after the frames before it (the reference throws)
      } else {
        var buf = Buffer.allocUnsafe(res.frameBytes) // decode.js:227 allocates _buffer the same way
        batch.copy(buf, 0, res.consumed)
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
    tm.convert += t.convert
    tm.h2dBytes += t.h2dBytes || 0
    tm.h2dSkipped += t.h2dSkipped || 0
  }
  var entry = { res: res, buf: batch, chunks: chunks, starts: starts, tooBig: tooBig }
  if (this._res) {
    this._ready = entry
    return
  }
  this._play(entry)
}

Decoder.prototype._play = function (e) {
  var res = e.res
  var batch = e.buf
  this._res = res
  this._buf = batch
  this._chunks = e.chunks
  this._starts = e.starts
  this._ck = 0
  this._blobPos = -1
  this._tooBig = e.tooBig
  this._text = res.asciiKeys && batch.length <= TEXT_MAX && batch.length <= TEXT_PER_FRAME * res.n
    ? batch.toString('latin1') : null
  this._next = 0
  this._kick() // the next batch goes to the GPU before this one's callbacks run
  this._replay()
}

// Deliver decoded frames in order while no callback is outstanding (decode.js:144-169).
// Change frames are built inline (the hot loop: one object, one key string, one value slice per
// frame); keys the GPU flagged ASCII are cut from one latin1 string of the batch (the same string
// buf.toString('utf8', ...) would give, without a UTF-8 decode per key).
Decoder.prototype._replay = function () {
  var res = this._res
  var buf = this._buf
  var n = res.n
  var type = res.type
  var off = res.off
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
  var text = this._text
  var down = this._down
  var i = this._next
  var t0 = process.hrtime()
  // (no callback can re-enter this loop: _down only resumes a paused replay)
  while (i < n && this._pending <= 0) {
    if ((type[i] & TYPE_MASK) !== 1) {
      if (this._deliverBlob(i)) i++ // (one push per written chunk the payload spans)
      if (this.destroyed) break
      continue
    }
    // messages.Change.decode result shape: {subset, key, change, from, to, value}
    var o = off[i]
    var f = flags[i]
    var k0 = o + ko[i]
    var k1 = k0 + kl[i]
    var vo = o + vcol[i]
    var change = {
      subset: (f & 1) ? buf.toString('utf8', o + so[i], o + so[i] + sl[i]) : '',
      key: (text !== null && (f & KEY_ASCII)) ? text.substring(k0, k1) : buf.toString('utf8', k0, k1),
      change: cc[i],
      from: cf[i],
      to: ct[i],
      value: (f & 2) ? buf.slice(vo, vo + vl[i]) : null
    }
    if (keyHash) change.keyHash = keyHash[i]
    this.changes++
    this._pending++ // released by the handler's cb (_up, decode.js:89-93)
    this._onchange(change, down)
    i++
    if (this.destroyed) break
  }
  this._next = i
  var dt = process.hrtime(t0)
  this.timing.replay += dt[0] * 1e3 + dt[1] * 1e-6
  if (this.destroyed) return
  if (this._pending > 0) {
    this._paused = true // resumed by _down
    return
  }
  if (res.errCode) return this.destroy(new Error(ERRORS[res.errCode](res.errDetail)))
  if (this._tooBig) {
    return this.destroy(new RangeError('Change frame of ' + this._tooBig + ' bytes exceeds the maximum Buffer size'))
  }
  this._res = null
  this._buf = null
  this._chunks = null
  this._starts = null
  this._text = null
  var next = this._ready
  this._ready = null
  if (next) this._play(next)
  else this._kick()
}

// One piece of blob frame i (or of the continuation of one opened in an earlier batch): the
// part of its payload inside the next written chunk, pushed as a slice of that chunk with one
// callback, as _onblobdata pushes each chunk's part (decode.js:179-202); true once the frame's
// last piece is delivered (and the blob ended, unless it continues past the batch).
Decoder.prototype._deliverBlob = function (i) {
  var res = this._res
  var type = res.type[i]
  var off = res.off[i]
  var end = off + Math.min(res.len[i], this._buf.length - off)
  var pos = this._blobPos
  if (pos < 0) {
    pos = off
    if (!(type & CONT)) {
      this.blobs++
      this._blob = new BlobStream(this)
      this._onblob(this._blob, this._down)
    }
  }
  var chunks = this._chunks
  var starts = this._starts
  var k = this._ck
  while (k + 1 < chunks.length && starts[k + 1] <= pos) k++
  this._ck = k
  var stop = Math.min(end, starts[k] + chunks[k].length)
  var data = pos < stop ? chunks[k].slice(pos - starts[k], stop - starts[k]) : this._buf.slice(pos, pos)
  var blob = this._blob
  var last = stop >= end
  this._blobPos = last ? -1 : stop
  blob._push(data, this._up())
  if (!last) return false
  if (!(type & PARTIAL)) { // decode.js:171-177
    this._pending++ // released by the blob handler's cb
    this._blob = null
    blob._end()
  }
  return true
}

module.exports = Decoder
