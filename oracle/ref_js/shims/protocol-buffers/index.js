// TEST INFRASTRUCTURE ONLY. Stand-in for protocol-buffers@^2.1.4 (package.json:27 of the
// reference; not vendored, absent offline) for the one schema the reference compiles
// (messages/schema.proto:1-8, messages/index.js:5). Two codecs, chosen by DRP_REF_CODEC:
//   passthrough (default) - Change.decode returns {payload: <copy of the bytes>}: the
//                           fixtures then pin the reference's FRAMING only (decode.js/encode.js
//                           are the real code); codec parity is pinned separately
//                           (tests/golden/change_codec.json, google.protobuf vectors).
//   full                  - a restatement of the generated proto2 decoder (switch on tag,
//                           unknown fields skipped by wire type, last wins), used to time the
//                           reference path for the calibration ratio.
//   strict                - passthrough results, but it throws as the generated decoder does for
//                           a payload missing a required field (the codec-throw fixtures).
// Change.encode (both modes) writes present fields in field-number order, as the generated
// encoder does.
'use strict'
var varint = require('varint')

var FIELDS = [['subset', 1, 'string'], ['key', 2, 'string'], ['change', 3, 'uint32'],
  ['from', 4, 'uint32'], ['to', 5, 'uint32'], ['value', 6, 'bytes']]

function checkSchema (src) {
  var s = String(src)
  FIELDS.forEach(function (f) {
    var re = new RegExp('(optional|required)\\s+' + f[2] + '\\s+' + f[0] + '\\s*=\\s*' + f[1] + '\\s*;')
    if (!re.test(s)) throw new Error('schema shim: unexpected schema.proto (field ' + f[0] + ')')
  })
}

function encode (obj) {
  var parts = []
  function str (tag, v, isBuf) {
    var b = isBuf ? (Buffer.isBuffer(v) ? v : Buffer.from(v)) : Buffer.from(String(v), 'utf-8')
    parts.push(Buffer.from([tag]), Buffer.from(varint.encode(b.length)), b)
  }
  function num (tag, v) { parts.push(Buffer.from([tag]), Buffer.from(varint.encode(v))) }
  if (obj.subset !== undefined && obj.subset !== null) str(0x0a, obj.subset, false)
  if (obj.key === undefined || obj.key === null) throw new Error('key is required')
  str(0x12, obj.key, false)
  ;['change', 'from', 'to'].forEach(function (k, i) {
    if (obj[k] === undefined || obj[k] === null) throw new Error(k + ' is required')
    num(0x18 + 8 * i, obj[k])
  })
  if (obj.value !== undefined && obj.value !== null) str(0x32, obj.value, true)
  return Buffer.concat(parts)
}

function decodeFull (buf) {
  var o = { subset: '', key: '', change: 0, from: 0, to: 0, value: null }
  var off = 0
  while (off < buf.length) {
    var prefix = varint.decode(buf, off)
    off += varint.decode.bytes
    var tag = prefix >> 3
    var l
    switch (tag) {
      case 1: case 2: case 6:
        l = varint.decode(buf, off)
        off += varint.decode.bytes
        if (tag === 6) o.value = buf.slice(off, off + l)
        else o[tag === 1 ? 'subset' : 'key'] = buf.toString('utf-8', off, off + l)
        off += l
        break
      case 3: case 4: case 5:
        o[['change', 'from', 'to'][tag - 3]] = varint.decode(buf, off)
        off += varint.decode.bytes
        break
      default:
        var wire = prefix & 7
        if (wire === 0) { varint.decode(buf, off); off += varint.decode.bytes } else if (wire === 1) off += 8
        else if (wire === 2) { l = varint.decode(buf, off); off += varint.decode.bytes + l } else if (wire === 5) off += 4
        else throw new Error('Unknown wire type: ' + wire)
    }
  }
  return o
}

function decodePassthrough (buf) {
  return { payload: Buffer.from(buf) }
}

// strict: decodeFull, then the generated decoder's required-field check (protocol-buffers@2 throws
// Error('Decoded message is not valid') when a required field is missing): used to record how the
// reference's FRAMING surfaces a codec throw (tests/golden/make_throw_fixtures.py)
function decodeStrict (buf) {
  var seen = {}
  var off = 0
  while (off < buf.length) {
    var prefix = varint.decode(buf, off)
    if (varint.decode.bytes === 0) throw new Error('Decoded message is not valid')
    off += varint.decode.bytes
    var tag = prefix >> 3
    seen[tag] = true
    var l = (prefix & 7) === 2 ? varint.decode(buf, off) : 0
    if ((prefix & 7) === 2) off += varint.decode.bytes + l
    else { varint.decode(buf, off); off += varint.decode.bytes }
  }
  if (!seen[2] || !seen[3] || !seen[4] || !seen[5]) throw new Error('Decoded message is not valid')
  return decodePassthrough(buf)
}

module.exports = function (schema) {
  checkSchema(schema)
  var mode = process.env.DRP_REF_CODEC
  return { Change: { encode: encode, decode: mode === 'full' ? decodeFull : mode === 'strict' ? decodeStrict : decodePassthrough } }
}
