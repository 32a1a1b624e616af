// TEST INFRASTRUCTURE: how a decoder surfaces a Change its codec rejects, shared by
// oracle/ref_js/ref_run.js (the reference with the strict codec shim, to record
// tests/golden/ref_throws.json) and tests/js/throw_order.js (this package, to compare). The log
// holds, in order: c<i> change i delivered (its key), a<i> acknowledged (on a later turn), w<k>
// write k's callback, throw<k>:<message> an exception out of write k, error:<message> an 'error'
// event, uncaught:<message> an exception no caller caught (thrown from a callback the stream ran),
// close, finish. The run ends at the first of error / finish / uncaught / a quiet second.
//   pattern 'burst': every write issued at once (the stream buffers them)
//   pattern 'paced': the next write issued from the previous write's callback
'use strict'

module.exports = function run (protocol, wire, sizes, pattern, done) {
  var log = []
  var d = protocol.decode()
  var nc = 0
  var ended = false
  function end () {
    if (ended) return
    ended = true
    setTimeout(function () { done(log) }, 50)
  }
  process.on('uncaughtException', function (e) { log.push('uncaught:' + e.message); end() })
  d.change(function (c, cb) {
    var i = nc++
    // (the reference's pass-through codec shim hands the payload over: its key is the first field)
    log.push('c' + i + ':' + (c.key !== undefined ? c.key : c.payload.slice(2, 2 + c.payload[1]).toString()))
    setImmediate(function () { log.push('a' + i); cb() })
  })
  d.blob(function (b, cb) { b.resume(); b.on('end', function () { setImmediate(cb) }) })
  d.on('error', function (e) { log.push('error:' + e.message); end() })
  d.on('close', function () { log.push('close') })
  d.on('finish', function () { log.push('finish'); end() })
  setTimeout(end, 1000)
  var pos = 0
  var k = 0
  function chunk () {
    var n = sizes[k++ % sizes.length]
    var c = wire.slice(pos, pos + n)
    pos += n
    return c
  }
  function write (id, c, cb) {
    try {
      d.write(c, cb)
    } catch (e) {
      log.push('throw' + id + ':' + e.message)
    }
  }
  if (pattern === 'burst') {
    for (var w = 0; pos < wire.length; w++) {
      (function (id) { write(id, chunk(), function () { log.push('w' + id) }) })(w)
    }
    try { d.end() } catch (e) { log.push('throw-end:' + e.message) }
  } else {
    (function next (id) {
      if (pos >= wire.length) {
        try { d.end() } catch (e) { log.push('throw-end:' + e.message) }
        return
      }
      write(id, chunk(), function () { log.push('w' + id); next(id + 1) })
    })(0)
  }
}
