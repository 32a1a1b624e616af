// TEST INFRASTRUCTURE ONLY (this container; never shipped to the GPU box).
// Runs the UNMODIFIED reference (/root/reference/{decode,encode}.js, required in place) with
// the restated dependency shims under ./shims on NODE_PATH, to generate golden fixtures and
// the calibration timing. Driven by tests/golden/make_ref_fixtures.py.
//
//   node ref_run.js decode <wire file> <write sizes, comma separated, cycled>
//        -> JSON events [{t:'change', payload:hex} | {t:'blob', data:hex, ended} | {t:'error', message}
//                        | {t:'finish', changes, blobs, bytes}]
//   node ref_run.js decode-multi <wire file> <patterns.json>  -> [events per write pattern]
//   node ref_run.js encode <ops.json>   -> JSON {wire: hex, changes, blobs, bytes, drains}
//        ops: [{op:'change', key, change, from, to, value(hex)?, subset?} |
//              {op:'blob', len, writes:[hex,...]} | {op:'finalize'}]
//   node ref_run.js acks <wire file> <write sizes> <burst|paced>
//        -> the callback order of tests/js/ack_driver.js (write acknowledgements vs async handlers)
//   node ref_run.js throws <wire file> <write sizes> <burst|paced>   (DRP_REF_CODEC=strict)
//        -> how a rejected Change surfaces (tests/js/throw_driver.js)
//   node ref_run.js bench <wire file> <chunk> <seconds>   (DRP_REF_CODEC=full)
//        -> JSON {frames_per_s, bytes_per_s, frames, reps}
'use strict'
var fs = require('fs')
var path = require('path')
var REF = process.env.DRP_REFERENCE || '/root/reference'
var protocol = require(REF) // index.js:1-2 -> encode.js, decode.js

function decodeEvents (wire, sizes, done) {
  var out = []
  var d = protocol.decode()
  d.change(function (c, cb) {
    out.push({ t: 'change', payload: c.payload.toString('hex') })
    cb()
  })
  d.blob(function (b, cb) {
    var ev = { t: 'blob', data: [], ended: false }
    out.push(ev)
    b.on('data', function (x) { ev.data.push(x) })
    b.on('end', function () { ev.ended = true; cb() })
  })
  var finished = false
  function fin () {
    if (finished) return
    finished = true
    setImmediate(function () { // let pending blob 'data' events land
      out.forEach(function (e) { if (e.t === 'blob') e.data = Buffer.concat(e.data).toString('hex') })
      done(out)
    })
  }
  d.on('error', function (e) { out.push({ t: 'error', message: e.message }); fin() })
  d.on('finish', function () { out.push({ t: 'finish', changes: d.changes, blobs: d.blobs, bytes: d.bytes }); fin() })
  var pos = 0
  var k = 0
  while (pos < wire.length) {
    var n = sizes[k++ % sizes.length] || wire.length // 0 = the rest
    d.write(wire.slice(pos, pos + n))
    pos += n
  }
  d.end()
}

// every pattern in one process (write-size lists, cycled, 0 = the rest): [events per pattern]
function decodeMulti (wire, patterns, done) {
  var res = []
  ;(function next (i) {
    if (i === patterns.length) return done(res)
    decodeEvents(wire, patterns[i], function (ev) { res.push(ev); next(i + 1) })
  })(0)
}

function encodeOps (ops, done) {
  var e = protocol.encode()
  var parts = []
  var drains = 0
  var paused = false
  // a slow consumer: read in small pieces on a timer so push() returns false (encode.js:139-151)
  e.on('readable', function () {
    var x
    while ((x = e.read()) !== null) parts.push(x)
  })
  e.on('end', function () {
    done({ wire: Buffer.concat(parts).toString('hex'), changes: e.changes, blobs: e.blobs, bytes: e.bytes, drains: drains })
  })
  // finalize() pushes EOF at once (encode.js:119-122), so it is issued only after every
  // change/blob callback has fired (queued changes are pushed when the last blob finishes)
  var outstanding = 0
  var wantFinal = false
  function ack () { if (--outstanding === 0 && wantFinal) e.finalize() }
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
  void paused
}

function bench (wire, chunk, seconds) {
  var frames = 0
  var reps = 0
  var t0 = process.hrtime.bigint()
  var limit = BigInt(Math.round(seconds * 1e9))
  function once () {
    var d = protocol.decode()
    d.change(function (c, cb) { frames++; cb() })
    for (var pos = 0; pos < wire.length; pos += chunk) d.write(wire.slice(pos, pos + chunk))
    d.end()
    reps++
  }
  do { once() } while (process.hrtime.bigint() - t0 < limit)
  var dt = Number(process.hrtime.bigint() - t0) / 1e9
  process.stdout.write(JSON.stringify({ frames_per_s: frames / dt, bytes_per_s: reps * wire.length / dt,
    frames: frames, reps: reps, seconds: dt, node: process.version }) + '\n')
}

var cmd = process.argv[2]
if (cmd === 'decode') {
  var wire = fs.readFileSync(process.argv[3])
  var sizes = process.argv[4].split(',').map(Number)
  decodeEvents(wire, sizes, function (ev) { process.stdout.write(JSON.stringify(ev) + '\n') })
} else if (cmd === 'decode-multi') {
  decodeMulti(fs.readFileSync(process.argv[3]), JSON.parse(fs.readFileSync(process.argv[4], 'utf8')),
    function (r) { process.stdout.write(JSON.stringify(r) + '\n') })
} else if (cmd === 'encode') {
  var ops = JSON.parse(fs.readFileSync(process.argv[3], 'utf8'))
  encodeOps(ops, function (r) { process.stdout.write(JSON.stringify(r) + '\n') })
} else if (cmd === 'acks') { // node ref_run.js acks <wire file> <write sizes> <burst|paced>
  require(path.join(__dirname, '..', '..', 'tests', 'js', 'ack_driver.js'))(protocol, fs.readFileSync(process.argv[3]),
    process.argv[4].split(',').map(Number), process.argv[5], function (log) { process.stdout.write(JSON.stringify(log) + '\n') })
} else if (cmd === 'throws') { // node ref_run.js throws <wire file> <write sizes> <burst|paced> (DRP_REF_CODEC=strict)
  require(path.join(__dirname, '..', '..', 'tests', 'js', 'throw_driver.js'))(protocol, fs.readFileSync(process.argv[3]),
    process.argv[4].split(',').map(Number), process.argv[5], function (log) {
      process.stdout.write(JSON.stringify(log) + '\n')
      process.exit(0)
    })
} else if (cmd === 'bench') {
  bench(fs.readFileSync(process.argv[3]), Number(process.argv[4]), Number(process.argv[5]))
} else {
  process.stderr.write('usage: ref_run.js decode|encode|bench ...\n')
  process.exit(2)
}
void path
