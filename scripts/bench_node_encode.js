// Node-path throughput of the package's Encoder (encode.js over the addon): `rows` change()
// calls issued back to back (the encoder batches each tick's calls, up to 65536, into one GPU
// encode on the worker thread), then finalize(); the Readable output is piped to a sink that
// discards it. Two shapes: "c1" rows (32-char [a-z0-9] key, change=i+1, from=i, to=i+1, 64 random
// value bytes: BASELINE C1 / the reference's "1M x 64 B values" encode row) and "c5" rows (key
// U[1,256] bytes of [a-z], change/from/to U[0,2^32), 4096 random value bytes). Rows are built
// before the clock starts. Prints one JSON line.
// usage: node bench_node_encode.js <c1|c5> <rows> <reps>
'use strict'
var path = require('path')
var stream = require('stream')
var protocol = require(path.join(__dirname, '..', 'dat-replication-protocol_amd'))

var shape = process.argv[2] || 'c1'
var rows = Number(process.argv[3] || 1000000)
var reps = Number(process.argv[4] || 3)

var seed = 12345
function rnd () { // xorshift32
  seed ^= seed << 13; seed >>>= 0
  seed ^= seed >>> 17
  seed ^= seed << 5; seed >>>= 0
  return seed
}
var ALPHA = 'abcdefghijklmnopqrstuvwxyz0123456789'
var vlen = shape === 'c5' ? 4096 : 64
var values = Buffer.allocUnsafe(vlen * Math.min(rows, 4096))
for (var b = 0; b < values.length; b++) values[b] = rnd() & 0xff
var changes = new Array(rows)
for (var i = 0; i < rows; i++) {
  var kl = shape === 'c5' ? 1 + rnd() % 256 : 32
  var key = ''
  for (var j = 0; j < kl; j++) key += ALPHA[rnd() % (shape === 'c5' ? 26 : 36)]
  var v = (i % 4096) * vlen
  changes[i] = shape === 'c5'
    ? { key: key, change: rnd(), from: rnd(), to: rnd(), value: values.slice(v, v + vlen) }
    : { key: key, change: i + 1, from: i, to: i + 1, value: values.slice(v, v + vlen) }
}

var times = []
var bytes = 0
function once (done) {
  var e = protocol.encode()
  var sink = new stream.Writable({ write: function (chunk, enc, cb) { bytes += chunk.length; cb() } })
  var t0 = process.hrtime.bigint()
  sink.on('finish', function () {
    times.push(Number(process.hrtime.bigint() - t0) / 1e9)
    done()
  })
  e.pipe(sink)
  for (var i = 0; i < rows; i++) e.change(changes[i])
  e.finalize()
}

;(function next (k) {
  if (k === reps + 1) {
    var t = times.slice(1) // the first pass warms up (device context, allocations)
    var mean = t.reduce(function (a, b) { return a + b }, 0) / t.length
    var wire = bytes / (reps + 1)
    process.stdout.write(JSON.stringify({ shape: shape, rows: rows, wire_bytes_per_pass: wire, seconds_mean: mean,
      seconds_best: Math.min.apply(null, t), frames_per_s: rows / mean, wire_GBps: wire / mean / 1e9,
      node: process.version }) + '\n')
    return
  }
  once(function () { next(k + 1) })
})(0)
