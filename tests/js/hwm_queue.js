// The Decoder's write queue and highWaterMark (CPU, over the mock addon: tests/js/mock_native.js).
// usage: node hwm_queue.js <n writes> <bytes per write>
// Writes n distinct Buffers (each a C2-style Change frame run, fresh per write) one per
// event-loop turn after each callback, and prints JSON: the writable highWaterMark of a default
// decoder and of decode({highWaterMark: 16384}), write()'s return values for the latter while
// ~64 KiB is buffered, and the most written Buffers the decoder's queue still referenced after
// their write had been consumed (ADVICE r5: consumed writes must not be kept alive).
'use strict'
var path = require('path')
var pkg = path.join(__dirname, '..', '..', 'dat-replication-protocol_amd')
require('./mock_native').install(pkg)
var protocol = require(pkg)

var n = Number(process.argv[2] || 300)
var size = Number(process.argv[3] || 65536)

function frames (seed, bytes) { // Change frames: key k<seed>, one-byte numbers, value fill
  var parts = []
  var total = 0
  var i = 0
  while (total < bytes - 40) {
    var key = Buffer.from('k' + seed + '_' + i)
    var val = Buffer.alloc(16, i & 0xff)
    var p = Buffer.concat([Buffer.from([0x12, key.length]), key, Buffer.from([0x18, 1, 0x20, 2, 0x28, 3, 0x32, val.length]), val])
    var f = Buffer.concat([Buffer.from([p.length + 1, 1]), p])
    parts.push(f)
    total += f.length
    i++
  }
  return Buffer.concat(parts)
}

var out = {}
out.defaultHwm = protocol.decode().writableHighWaterMark
var small = protocol.decode({ highWaterMark: 16384 })
out.optionHwm = small.writableHighWaterMark
var rets = []
for (var k = 0; k < 4; k++) rets.push(small.write(frames(900 + k, 16384)))
out.writeReturns = rets // (the reference's 16 KiB: false once 16 KiB are buffered)
small.destroy()

var d = protocol.decode()
var written = []
var retained = 0
var changes = 0
d.change(function (c, cb) { changes++; cb() })
function liveConsumed () { // queue entries holding a write _write has already taken
  var q = d._q
  var live = 0
  for (var j = 0; j < d._qh; j++) if (q[j] !== undefined) live++
  return live
}
var w = 0
function next () {
  if (w === n) return d.end()
  var b = frames(w, size)
  written.push(b.length)
  w++
  d.write(b, function () {
    var r = liveConsumed()
    if (r > retained) retained = r
    setImmediate(next)
  })
}
d.on('finish', function () {
  out.changes = changes
  out.retained = retained
  out.queueLength = d._q.length
  out.writes = n
  console.log(JSON.stringify(out))
})
next()
