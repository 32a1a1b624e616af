// Decoder: the reference's streaming decode API (decode.js:63-142 of
// mafintosh/dat-replication-protocol v4.1.2) over the gfx950 batch codec.
//
// Each chunk handed to _write is decoded on the GPU in one call (frame split + Change
// decode, libdrp via lib/drp.node); the returned frame table is then replayed here with
// the reference's callback discipline: a change/blob callback increments _pending, and
// replay stops while _pending > 0 and resumes from _down (decode.js:89-99, 144-169).
// Bytes of an incomplete trailing frame are carried into the next chunk
// (decode.js:75-81 state) and an open blob continues across chunks.
'use strict'

var stream = require('stream')
var util = require('util')
var native = require('./native')

var FLUSH = Buffer.from([0]) // identity-compared end sentinel (decode.js:6, :125)

var TYPE_MASK = 0x3f
var CONT = 0x40
var PARTIAL = 0x80

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

function Decoder () {
  if (!(this instanceof Decoder)) return new Decoder()
  stream.Writable.call(this)

  this.destroyed = false
  this.bytes = 0
  this.changes = 0
  this.blobs = 0

  this._pending = 0
  this._onflush = null

  this._onchange = noopChange
  this._onblob = drainBlob
  this._onfinalize = noopFinalize

  this._ctx = native.context()
  this._carry = null      // bytes of an incomplete frame (header and/or change payload)
  this._blobLeft = 0      // payload bytes of the open blob still to come
  this._blob = null       // the open BlobStream
  this._res = null        // decoded batch being replayed
  this._buf = null        // its bytes
  this._next = 0          // next frame to deliver

  var self = this
  this._up = function () {
    self._pending++
    return self._down
  }
  this._down = function () {
    if (--self._pending > 0) return
    var cb = self._onflush
    self._onflush = null
    if (cb) self._replay(cb)
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
  if (data === FLUSH) return this._onfinalize(cb)
  this.bytes += data.length

  var buf = this._carry ? Buffer.concat([this._carry, data]) : data
  this._carry = null
  var res = native.decode(this._ctx, buf, this._blobLeft)
  // tail kinds 1/2: an incomplete header / change payload is carried (copied, as the
  // reference copies it into _header / _buffer)
  if (!res.errCode && (res.tailKind === 1 || res.tailKind === 2)) this._carry = Buffer.from(buf.slice(res.consumed))
  this._blobLeft = res.blobRemaining
  this._res = res
  this._buf = buf
  this._next = 0
  this._replay(cb)
}

Decoder.prototype.end = function (data, enc, cb) {
  if (typeof data === 'function') return this.end(null, null, data)
  if (typeof enc === 'function') return this.end(data, null, enc)
  if (data) this.write(data)
  this.write(FLUSH)
  stream.Writable.prototype.end.call(this, cb)
}

// Deliver decoded frames in order while no callback is outstanding (decode.js:144-169).
Decoder.prototype._replay = function (cb) {
  var res = this._res
  while (this._next < res.n && this._pending <= 0 && !this.destroyed) {
    this._deliver(this._next++)
  }
  if (this.destroyed) return
  if (this._next >= res.n && res.errCode && this._pending <= 0) {
    this.destroy(new Error(ERRORS[res.errCode](res.errDetail)))
    return
  }
  if (this._pending <= 0) cb()
  else this._onflush = cb
}

Decoder.prototype._deliver = function (i) {
  var res = this._res
  var buf = this._buf
  var type = res.type[i]
  var off = res.off[i]
  if ((type & TYPE_MASK) === 1) {
    // messages.Change.decode result shape: {subset, key, change, from, to, value}
    var flags = res.flags[i]
    var change = {
      subset: (flags & 1) ? buf.toString('utf8', off + res.so[i], off + res.so[i] + res.sl[i]) : '',
      key: buf.toString('utf8', off + res.ko[i], off + res.ko[i] + res.kl[i]),
      change: res.change[i],
      from: res.from[i],
      to: res.to[i],
      value: (flags & 2) ? buf.slice(off + res.vo[i], off + res.vo[i] + res.vl[i]) : null
    }
    this.changes++
    this._onchange(change, this._up())
    return
  }
  // blob frame (or the continuation of one opened in an earlier chunk)
  if (!(type & CONT)) {
    this.blobs++
    this._blob = new BlobStream(this)
    this._onblob(this._blob, this._down)
  }
  var avail = Math.min(res.len[i], buf.length - off)
  this._blob._push(buf.slice(off, off + avail), this._up())
  if (!(type & PARTIAL)) {
    this._pending++ // released by the handler's cb (decode.js:171-177)
    this._blob._end()
    this._blob = null
  }
}

module.exports = Decoder
