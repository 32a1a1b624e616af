// Node-path throughput of the package's Decoder (the product path north_star names): a wire
// file written in `write`-byte chunks with the decoder coalescing up to DRP_MAX_BATCH bytes per
// GPU call; no-op change callbacks (acknowledged synchronously). Prints one JSON line.
// usage: DRP_MAX_BATCH=<bytes> node bench_node.js <wire file> <write bytes> <reps>
'use strict'
var fs = require('fs')
var path = require('path')
var protocol = require(process.env.DRP_PKG || path.join(__dirname, '..', 'dat-replication-protocol_amd'))

var wire = fs.readFileSync(process.argv[2])
var write = Number(process.argv[3])
var reps = Number(process.argv[4] || 3)
var frames = 0
var times = []
var breakdown = []

function once (done) {
  var d = protocol.decode()
  d.change(function (c, cb) { frames++; cb() })
  var t0 = process.hrtime.bigint()
  d.on('finish', function () {
    times.push(Number(process.hrtime.bigint() - t0) / 1e9)
    breakdown.push(d.timing)
    done()
  })
  var pos = 0
  ;(function pump () {
    while (pos < wire.length) {
      var ok = d.write(wire.slice(pos, pos + write))
      pos += write
      if (!ok) return d.once('drain', pump)
    }
    d.end()
  })()
}

;(function next (i) {
  if (i === reps + 1) {
    var t = times.slice(1) // the first pass warms up (device context, allocations)
    var best = Math.min.apply(null, t)
    var mean = t.reduce(function (a, b) { return a + b }, 0) / t.length
    // per pass, ms, mean over the timed passes: H2D (staging into HBM), the decode kernels, the
    // D2H of the columns and their u64 -> Number conversion run on the addon's worker thread,
    // overlapped with the JS replay of the previous batch (building the change objects and
    // running the callbacks) on the main thread
    var b = breakdown.slice(1)
    var ms = {}
    ;['h2d', 'gpu', 'd2h', 'd2hMax', 'pinnedBatches', 'convert', 'replay', 'batches'].forEach(function (k) {
      ms[k] = b.reduce(function (a, x) { return a + x[k] }, 0) / b.length
    })
    process.stdout.write(JSON.stringify({ write_bytes: write, max_batch: Number(process.env.DRP_MAX_BATCH || 0) ||
      64 * 1024 * 1024, wire_bytes: wire.length, frames_per_pass: frames / (reps + 1), seconds_mean: mean,
      seconds_best: best, frames_per_s: frames / (reps + 1) / mean, wire_GBps: wire.length / mean / 1e9,
      breakdown_ms_per_pass: ms, wall_ms_per_pass: mean * 1e3, node: process.version }) + '\n')
    return
  }
  once(function () { next(i + 1) })
})(0)
