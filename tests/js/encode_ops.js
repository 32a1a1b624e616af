// Run an encoder call sequence (tests/golden/ref_framing.json "ops" format) through the
// package's Encoder and print {wire sha256/hex, counters, pushFalse}. With "slow", the
// consumer reads one chunk per setImmediate through a 1-byte highWaterMark, so push() returns
// false and the drain path (encode.js:139-151) runs. finalize() is issued once every
// change/blob callback has fired, as in oracle/ref_js/ref_run.js.
// usage: node encode_ops.js <ops.json> [slow]
'use strict'
var fs = require('fs')
var path = require('path')
var crypto = require('crypto')
var protocol = require(path.join(__dirname, '..', '..', 'dat-replication-protocol_amd'))

var ops = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'))
var slow = process.argv[3] === 'slow'
var e = protocol.encode()
var parts = []
var pushFalse = 0
var origPush = e.push
e.push = function (x) {
  var r = origPush.call(this, x)
  if (x !== null && !r) pushFalse++
  return r
}
if (slow) {
  e._readableState.highWaterMark = 1
  var pump = function () {
    var x = e.read()
    if (x !== null) parts.push(x)
    if (!e._readableState.ended || e._readableState.length) setImmediate(pump)
    else done()
  }
  setImmediate(pump)
} else {
  e.on('data', function (x) { parts.push(x) })
  e.on('end', done)
}
var printed = false
function done () {
  if (printed) return
  printed = true
  var wire = Buffer.concat(parts)
  process.stdout.write(JSON.stringify({ sha256: crypto.createHash('sha256').update(wire).digest('hex'),
    hex: wire.length <= 4096 ? wire.toString('hex') : null, len: wire.length, changes: e.changes, blobs: e.blobs,
    bytes: e.bytes, pushFalse: pushFalse, acked: acked }) + '\n')
}
var outstanding = 0
var acked = 0
var wantFinal = false
function ack () {
  acked++
  if (--outstanding === 0 && wantFinal) e.finalize()
}
ops.forEach(function (o) {
  if (o.op === 'change') {
    var obj = { key: o.key, change: o.change, from: o.from, to: o.to }
    if (o.value !== undefined) obj.value = Buffer.from(o.value, 'hex')
    if (o.subset !== undefined) obj.subset = o.subset
    outstanding++
    e.change(obj, ack)
  } else if (o.op === 'blob') {
    outstanding++
    var b = e.blob(o.len, ack)
    o.writes.forEach(function (w) { b.write(Buffer.from(w, 'hex')) })
    b.end()
  } else if (o.op === 'finalize') {
    wantFinal = true
    if (outstanding === 0) e.finalize()
  }
})
setTimeout(function () { process.stderr.write('encode_ops: timeout\n'); process.exit(3) }, 60000).unref()
