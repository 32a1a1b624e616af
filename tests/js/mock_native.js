// TEST INFRASTRUCTURE ONLY: a CPU stand-in for the package's native module (native.js) so the
// JS host layer (decode.js: batching, carry, replay, backpressure) can be tested without a GPU.
// It is installed by the test harnesses through require.cache (never by the package itself,
// which has no CPU path) and answers decode(ctx, batch, blobRemaining, cb) with the result
// drp_decode_stage + drp_decode_fetch give for the same batch (include/drp.h), restated
// sequentially: a leading blob continuation as row 0, frames split by their varint headers
// (decode.js:251-262; the header policy of DESIGN.md), Change payloads decoded like the oracle's
// protocol-buffers@2 restatement (oracle/drp_oracle.c), and the carry (tail header / change /
// blob) for the next batch.
'use strict'

var TYPE_CHANGE = 1
var TYPE_BLOB = 2
var CONT = 0x40
var PARTIAL = 0x80
var JS_SAFE = Math.pow(2, 53)

// varint@3 decode with the policy: > 10 bytes or >= 2^64 is malformed (-1); 0 = ran out
function vdec (b, p, end) {
  var v = 0
  for (var i = 0; i < 10; i++) {
    if (p + i >= end) return [0, 0]
    var x = b[p + i]
    var bits = x & 0x7f
    if (i === 9 && bits > 1) return [0, -1]
    v += bits * Math.pow(2, 7 * i)
    if (!(x & 0x80)) return [v, i + 1]
  }
  return [0, -1]
}

// messages.Change.decode restated (oracle_change_decode): offsets relative to the payload
function changeDecode (b, o, len) {
  var c = { ko: 0, kl: 0, so: 0, sl: 0, vo: 0, vl: 0, change: 0, from: 0, to: 0, flags: 0, err: 0 }
  var found = 0
  var off = 0
  while (off < len) {
    var r = vdec(b, o + off, o + len)
    if (r[1] <= 0 || r[0] >= JS_SAFE) return bad(c)
    off += r[1]
    var prefix = r[0]
    var tag = (prefix % 4294967296 | 0) >> 3
    var wire = prefix % 8
    if (tag === 1 || tag === 2 || tag === 6) {
      r = vdec(b, o + off, o + len)
      if (r[1] <= 0 || r[0] >= JS_SAFE) return bad(c)
      off += r[1]
      var l = r[0]
      if (l > len - off) return bad(c)
      if (tag === 1) { c.so = off; c.sl = l; c.flags |= 1 } else if (tag === 2) { c.ko = off; c.kl = l; found |= 1 } else { c.vo = off; c.vl = l; c.flags |= 2 }
      off += l
    } else if (tag === 3 || tag === 4 || tag === 5) {
      r = vdec(b, o + off, o + len)
      if (r[1] <= 0) return bad(c)
      off += r[1]
      if (tag === 3) { c.change = r[0]; found |= 2 } else if (tag === 4) { c.from = r[0]; found |= 4 } else { c.to = r[0]; found |= 8 }
    } else if (wire === 0) {
      r = vdec(b, o + off, o + len)
      if (r[1] <= 0) return bad(c)
      off += r[1]
    } else if (wire === 1) {
      if (len - off < 8) return bad(c)
      off += 8
    } else if (wire === 2) {
      r = vdec(b, o + off, o + len)
      if (r[1] <= 0 || r[0] >= JS_SAFE) return bad(c)
      off += r[1]
      if (r[0] > len - off) return bad(c)
      off += r[0]
    } else if (wire === 5) {
      if (len - off < 4) return bad(c)
      off += 4
    } else {
      return bad(c)
    }
  }
  if (found !== 15) {
    c.err = 5
    c.flags |= 4 | 8
  }
  return c
}
function bad (c) {
  c.err = 4
  c.flags |= 4
  return c
}

function decodeBatch (b, brem) {
  var n = b.length
  var rows = []
  var out = { n: 0, errFrame: -1, errCode: 0, errDetail: 0, consumed: n, tailKind: 0, blobRemaining: 0, frameBytes: 0 }
  if (brem) {
    rows.push({ off: 0, len: Math.min(brem, 0xffffffff), type: TYPE_BLOB | CONT | (brem > n ? PARTIAL : 0) })
    if (brem >= n) {
      out.blobRemaining = brem - n
      out.tailKind = out.blobRemaining ? 3 : 0
      out.n = 1
      return finish(b, out, rows, 1)
    }
  }
  var p = brem
  var bad = 0
  while (p < n) {
    var r = vdec(b, p, n)
    var k = r[1]
    if (k === 0 || (k < 0 && n - p < 11) || (k > 0 && p + k >= n)) {
      out.tailKind = 1
      out.consumed = p
      break
    }
    if (k < 0) { out.errCode = 3; break }
    var L = r[0]
    var id = b[p + k]
    if (id >= 3) { out.errCode = 1; out.errDetail = id; break }
    if (id === 0) { p += k + 1; continue }
    if (L === 0) { out.errCode = 2; out.errDetail = id; break }
    var po = p + k + 1
    var pl = L - 1
    if (id === TYPE_CHANGE) {
      if (po + pl > n) {
        out.tailKind = 2
        out.consumed = p
        out.frameBytes = k + L
        break
      }
      var c = changeDecode(b, po, pl)
      c.off = po
      c.len = pl
      c.type = TYPE_CHANGE
      var ascii = true
      for (var q = po + c.ko; q < po + c.ko + c.kl; q++) if (b[q] >= 0x80) { ascii = false; break }
      if (!c.err && ascii) c.flags |= 0x10 | 0x20
      rows.push(c)
      if (c.err) {
        out.errCode = c.err
        bad = 1
        break
      }
    } else {
      if (po + pl > n) {
        rows.push({ off: po, len: Math.min(pl, 0xffffffff), type: TYPE_BLOB | PARTIAL })
        out.tailKind = 3
        out.blobRemaining = po + pl - n
        break
      }
      rows.push({ off: po, len: pl, type: TYPE_BLOB })
    }
    p = po + pl
  }
  out.n = rows.length - bad
  if (out.errCode) out.errFrame = out.n
  return finish(b, out, rows, rows.length)
}

function finish (b, out, rows, nrows) {
  var cols = { off: Float64Array, len: Uint32Array, type: Uint8Array, ko: Uint32Array, kl: Uint32Array, so: Uint32Array,
    sl: Uint32Array, vo: Uint32Array, vl: Uint32Array, change: Float64Array, from: Float64Array, to: Float64Array, flags: Uint8Array }
  Object.keys(cols).forEach(function (k) {
    var a = new cols[k](nrows)
    for (var i = 0; i < nrows; i++) a[i] = rows[i][k] || 0
    out[k] = a
  })
  // the key text (drp_napi.c key_text): the ASCII keys of the Change rows end to end
  var kp = new Uint32Array(nrows)
  var parts = []
  var tot = 0
  for (var r = 0; r < nrows; r++) {
    kp[r] = tot
    var x = rows[r]
    if ((x.type & 0x3f) === TYPE_CHANGE && (x.flags & 0x14) === 0x10) {
      parts.push(b.toString('latin1', x.off + x.ko, x.off + x.ko + x.kl))
      tot += x.kl
    }
  }
  out.kp = kp
  out.keyText = parts.join('')
  out.t = { h2d: 0, gpu: 0, d2h: 0, convert: 0 }
  return out
}

exports.install = function (pkgDir) {
  var path = require('path')
  var file = require.resolve(path.join(pkgDir, 'native.js'))
  require.cache[file] = {
    id: file,
    filename: file,
    loaded: true,
    exports: {
      context: function () { return {} },
      deviceContext: function () { return {} },
      deviceCount: function () { return 0 },
      nextDevice: function () { return 0 },
      decode: function (ctx, batch, brem, cb) { // (batch: a Buffer, or the written chunks end to end)
        var r = decodeBatch(Array.isArray(batch) ? Buffer.concat(batch) : batch, brem)
        setImmediate(function () { cb(null, r) })
      },
      decodeSync: function (ctx, batch, brem) { return decodeBatch(batch, brem) },
      abiVersion: 5
    }
  }
}
