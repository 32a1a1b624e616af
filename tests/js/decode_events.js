// Feed a wire file through the package's Decoder in the given chunk sizes and print the
// delivered events as JSON lines (used by tests/test_js_api.py to compare with the oracle).
// usage: node decode_events.js <wire file> <chunk sizes comma separated, cycled> [asyncAck]
'use strict'
var fs = require('fs')
var path = require('path')
var protocol = require(path.join(__dirname, '..', '..', 'dat-replication-protocol_amd'))

var wire = fs.readFileSync(process.argv[2])
var sizes = (process.argv[3] || '65536').split(',').map(Number)
var asyncAck = process.argv[4] === 'async'
var out = []
var d = protocol.decode()
d.change(function (c, cb) {
  out.push({ t: 'change', subset: Buffer.from(c.subset, 'utf8').toString('hex'), key: Buffer.from(c.key, 'utf8').toString('hex'),
    change: c.change, from: c.from, to: c.to, value: c.value === null ? null : c.value.toString('hex') })
  if (asyncAck) setImmediate(cb); else cb()
})
d.blob(function (b, cb) {
  var parts = []
  b.on('data', function (x) { parts.push(x) })
  b.on('end', function () { out.push({ t: 'blob', data: Buffer.concat(parts).toString('hex') }); cb() })
})
d.on('error', function (e) { out.push({ t: 'error', message: e.message }); done() })
d.on('finish', function () { out.push({ t: 'finish', changes: d.changes, blobs: d.blobs, bytes: d.bytes }); done() })
var printed = false
function done () {
  if (printed) return
  printed = true
  process.stdout.write(JSON.stringify(out) + '\n')
}
var pos = 0
var k = 0
while (pos < wire.length) {
  var n = sizes[k++ % sizes.length]
  d.write(wire.slice(pos, pos + n))
  pos += n
}
d.end()
