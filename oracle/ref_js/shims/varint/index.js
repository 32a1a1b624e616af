// TEST INFRASTRUCTURE ONLY. Restatement of varint@^3.0.0 (package.json:28 of the reference;
// not vendored, absent offline): LEB128 with the .bytes side channel that decode.js:255 and
// encode.js:132-133 read. Lets /root/reference/{decode,encode}.js be required in place to
// generate golden fixtures (tests/golden/make_ref_fixtures.py); never shipped or loaded on
// the GPU box.
'use strict'
var MSB = 0x80
var REST = 0x7F
var MSBALL = ~REST
var INT = Math.pow(2, 31)

function encode (num, out, offset) {
  out = out || []
  offset = offset || 0
  var old = offset
  while (num >= INT) {
    out[offset++] = (num & 0xFF) | MSB
    num /= 128
  }
  while (num & MSBALL) {
    out[offset++] = (num & 0xFF) | MSB
    num >>>= 7
  }
  out[offset] = num | 0
  encode.bytes = offset - old + 1
  return out
}

function decode (buf, offset) {
  var res = 0
  offset = offset || 0
  var shift = 0
  var counter = offset
  var b
  do {
    if (counter >= buf.length) {
      decode.bytes = 0
      return undefined
    }
    b = buf[counter++]
    res += shift < 28 ? (b & REST) << shift : (b & REST) * Math.pow(2, shift)
    shift += 7
  } while (b >= MSB)
  decode.bytes = counter - offset
  return res
}

function encodingLength (n) {
  var k = 1
  while (n >= 128) { n = Math.floor(n / 128); k++ }
  return k
}

module.exports = { encode: encode, decode: decode, encodingLength: encodingLength }
