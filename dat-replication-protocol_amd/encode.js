// Encoder: the reference's streaming encode API (encode.js:46-151 of
// mafintosh/dat-replication-protocol v4.1.2) over the gfx950 batch codec.
//
// change() calls made in the same tick are encoded together on the GPU, on a worker thread
// (messages.Change.encode + varint(len+1) 0x01 framing, libdrp encode kernels), and pushed as
// one chunk; the byte stream is identical to the reference's. Everything the encoder outputs
// goes through one ordered queue, so a blob header or blob bytes issued after a batch of
// changes never overtake that batch's (asynchronous) encode. Blob ordering follows
// encode.js:77-117: blobs serialise in creation order (later blobs are corked) and changes
// issued while a blob is open wait until every open blob has finished.
'use strict'

var stream = require('stream')
var util = require('util')
var native = require('./native')

var MAX_BATCH = 1 << 16

function noop () {}

// blob header varint(len+1) 0x02 (encode.js:124-137); the blob payload itself is the
// caller's bytes, passed through untouched.
function blobHeader (len) {
  var out = []
  var n = len + 1
  while (n >= 0x80) {
    out.push((n % 0x80) | 0x80)
    n = Math.floor(n / 0x80)
  }
  out.push(n, 2)
  return Buffer.from(out)
}

// --- writable blob sub-stream (encode.js:11-44) -----------------------------------
function BlobStream (parent) {
  stream.Writable.call(this)
  this.destroyed = false
  this.corked = 0
  this._parent = parent
  this._pendingWrite = null
}
util.inherits(BlobStream, stream.Writable)

BlobStream.prototype.destroy = function (err) {
  if (this.destroyed) return
  this.destroyed = true
  if (err) this.emit('error', err)
  this.emit('close')
  if (this._parent) this._parent.destroy()
}

BlobStream.prototype.cork = function () { this.corked++ }

BlobStream.prototype.uncork = function () {
  if (!this.corked || --this.corked) return
  var args = this._pendingWrite
  this._pendingWrite = null
  if (args) this._write(args[0], args[1], args[2])
}

BlobStream.prototype._write = function (data, enc, cb) {
  if (this.corked) this._pendingWrite = [data, enc, cb]
  else this._parent._push(data, cb)
}

function required (obj, k) {
  var v = obj[k]
  if (v === undefined || v === null) throw new Error(k + ' is required')
  return v
}

function uint (obj, k) {
  var v = required(obj, k)
  if (typeof v !== 'number' || !Number.isInteger(v) || v < 0 || v > Number.MAX_SAFE_INTEGER) {
    throw new RangeError(k + ' must be an unsigned integer')
  }
  return v
}

// opts (not in the reference, whose constructor takes none): device: the GPU this stream
// encodes on (default: DRP_DEVICE or 0)
function Encoder (opts) {
  if (!(this instanceof Encoder)) return new Encoder(opts)
  stream.Readable.call(this)

  this.destroyed = false
  this.bytes = 0
  this.changes = 0
  this.blobs = 0

  this._blobs = []
  this._changes = []   // change() arguments queued behind open blobs
  this._batch = []     // [row, cb] awaiting the GPU encode
  this._scheduled = false
  this._ondrain = null
  this._out = []       // ordered output: {data, cb} (data null until its encode completes), or EOF
  this._ctx = native.context(opts && opts.device)
}
util.inherits(Encoder, stream.Readable)

Encoder.prototype.destroy = function (err) {
  if (this.destroyed) return
  this.destroyed = true
  while (this._blobs.length) this._blobs.shift().destroy()
  if (err) this.emit('error', err)
  this.emit('close')
}

Encoder.prototype.blob = function (len, cb) {
  if (this.destroyed) return null
  if (!len) throw new Error('Length is required')
  this._flush() // changes issued before this blob precede it on the wire

  this.blobs++
  var self = this
  var ws = new BlobStream(this)
  if (this._blobs.length) ws.cork()
  this._blobs.push(ws)
  ws.write(blobHeader(len))
  ws.on('finish', function () {
    if (self._blobs.shift() !== ws) throw new Error('Blob assertion failed')
    if (self._blobs.length) self._blobs[0].uncork()
    else while (!self._blobs.length && self._changes.length) self.change.apply(self, self._changes.shift())
    if (cb) cb()
  })
  return ws
}

Encoder.prototype.change = function (change, cb) {
  if (this.destroyed) return
  if (this._blobs.length) {
    this._changes.push([change, cb])
    return
  }
  // validate synchronously, as messages.Change.encode throws inside change()
  if (typeof required(change, 'key') !== 'string') throw new TypeError('key must be a string')
  var row = {
    key: Buffer.from(String(required(change, 'key')), 'utf8'),
    change: uint(change, 'change'),
    from: uint(change, 'from'),
    to: uint(change, 'to'),
    subset: (change.subset === undefined || change.subset === null) ? null : Buffer.from(String(change.subset), 'utf8'),
    value: (change.value === undefined || change.value === null) ? null
      : (Buffer.isBuffer(change.value) ? change.value : Buffer.from(String(change.value), 'utf8'))
  }
  this.changes++
  this._batch.push([row, cb || noop])
  if (this._batch.length >= MAX_BATCH) return this._flush()
  if (!this._scheduled) {
    this._scheduled = true
    var self = this
    process.nextTick(function () { self._flush() })
  }
}

// Encode the pending rows on the GPU and push them as one chunk.
Encoder.prototype._flush = function () {
  this._scheduled = false
  var batch = this._batch
  if (!batch.length || this.destroyed) return
  this._batch = []
  var n = batch.length
  var heapLen = 0
  for (var i = 0; i < n; i++) {
    var r = batch[i][0]
    heapLen += r.key.length + (r.subset ? r.subset.length : 0) + (r.value ? r.value.length : 0)
  }
  var heap = Buffer.allocUnsafe(heapLen)
  var ko = new Float64Array(n); var kl = new Uint32Array(n)
  var so = new Float64Array(n); var sl = new Uint32Array(n)
  var vo = new Float64Array(n); var vl = new Uint32Array(n)
  var ch = new Float64Array(n); var fr = new Float64Array(n); var to = new Float64Array(n)
  var fl = new Uint8Array(n)
  var p = 0
  for (i = 0; i < n; i++) {
    r = batch[i][0]
    ko[i] = p; kl[i] = r.key.length; p += r.key.copy(heap, p)
    if (r.subset) { so[i] = p; sl[i] = r.subset.length; p += r.subset.copy(heap, p); fl[i] |= 1 }
    if (r.value) { vo[i] = p; vl[i] = r.value.length; p += r.value.copy(heap, p); fl[i] |= 2 }
    ch[i] = r.change; fr[i] = r.from; to[i] = r.to
  }
  var cbs = batch.map(function (b) { return b[1] })
  var slot = { data: null, cb: function () { for (var k = 0; k < cbs.length; k++) cbs[k]() } }
  this._out.push(slot)
  var self = this
  native.encode(this._ctx, heap, n, ko, kl, so, sl, vo, vl, ch, fr, to, fl, function (err, wire) {
    if (self.destroyed) return
    if (err) return self.destroy(err)
    slot.data = wire
    self._drainOut()
  })
}

Encoder.prototype.finalize = function (cb) {
  this._flush()
  this._out.push({ eof: true, cb: cb || noop })
  this._drainOut()
}

// Queue output behind anything still being encoded (encode.js:139-145 pushes in call order).
Encoder.prototype._push = function (data, cb) {
  if (this.destroyed) return
  this._out.push({ data: data, cb: cb })
  this._drainOut()
}

Encoder.prototype._drainOut = function () {
  while (this._out.length && !this.destroyed) {
    var o = this._out[0]
    if (o.eof) {
      this._out.shift()
      if (!this._readableState.ended) this.push(null)
      o.cb()
      continue
    }
    if (!o.data) return // its encode is still running
    this._out.shift()
    this._emit(o.data, o.cb)
  }
}

Encoder.prototype._emit = function (data, cb) {
  this.bytes += data.length
  if (this.push(data)) return cb()
  var prev = this._ondrain
  this._ondrain = prev ? function () { prev(); cb() } : cb
}

Encoder.prototype._read = function () {
  var fn = this._ondrain
  this._ondrain = null
  if (fn) fn()
}

module.exports = Encoder
