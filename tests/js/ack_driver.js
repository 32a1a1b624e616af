// TEST INFRASTRUCTURE: the write-acknowledgement order of a decoder, shared by
// oracle/ref_js/ref_run.js (the reference, to record tests/golden/ref_acks.json) and
// tests/js/ack_order.js (this package, to compare). The log interleaves the decoder's
// callbacks: c<i> change i delivered, a<i> its handler acknowledged it (always on a later turn),
// b<j> blob j delivered, e<j> its stream ended (acknowledged on a later turn), w<k> write k's
// callback fired, f finalize, finish. Because every acknowledgement is asynchronous and every
// write completes a frame, the order is fixed by the decoder's rules alone (decode.js:89-99,
// 144-169: a write is acknowledged once its frames are delivered and acknowledged).
//   pattern 'burst': every write issued at once (the stream buffers them)
//   pattern 'paced': the next write issued from the previous write's callback
'use strict'

module.exports = function run (protocol, wire, sizes, pattern, done) {
  var log = []
  var d = protocol.decode()
  var nc = 0
  var nb = 0
  d.change(function (c, cb) {
    var i = nc++
    log.push('c' + i)
    setImmediate(function () { log.push('a' + i); cb() })
  })
  d.blob(function (b, cb) {
    var j = nb++
    log.push('b' + j)
    b.resume()
    b.on('end', function () { log.push('e' + j); setImmediate(cb) })
  })
  d.finalize(function (cb) { log.push('f'); cb() })
  d.on('error', function (e) { log.push('error:' + e.message); done(log) })
  d.on('finish', function () { log.push('finish'); done(log) })
  var pos = 0
  var k = 0
  function chunk () {
    var n = sizes[k++ % sizes.length]
    var c = wire.slice(pos, pos + n)
    pos += n
    return c
  }
  if (pattern === 'burst') {
    for (var w = 0; pos < wire.length; w++) {
      (function (id) { d.write(chunk(), function () { log.push('w' + id) }) })(w)
    }
    d.end()
  } else {
    (function next (id) {
      if (pos >= wire.length) return d.end()
      d.write(chunk(), function () { log.push('w' + id); next(id + 1) })
    })(0)
  }
}
