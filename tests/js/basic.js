// The four round trips of the reference's test/basic.js (encode -> pipe -> decode), restated
// for this package with plain assertions. Prints "ok N" lines; exits non-zero on failure.
'use strict'
var assert = require('assert')
var path = require('path')
var protocol = require(path.join(__dirname, '..', '..', 'dat-replication-protocol_amd'))

var expectChange = { key: 'key', from: 0, to: 1, change: 1, value: Buffer.from('hello'), subset: '' }
var pending = 0
var passed = 0
function test (name, fn) {
  pending++
  fn(function () { passed++; console.log('ok ' + passed + ' ' + name); if (--pending === 0) process.exit(0) })
}
function collect (readable, cb) {
  var parts = []
  readable.on('data', function (x) { parts.push(x) })
  readable.on('end', function () { cb(Buffer.concat(parts)) })
}
setTimeout(function () { console.error('timeout: ' + pending + ' tests did not finish'); process.exit(1) }, 20000).unref()

test('encode + decode changes', function (end) {
  var e = protocol.encode()
  var d = protocol.decode()
  d.change(function (change) {
    assert.deepStrictEqual(change, expectChange)
    end()
  })
  e.change({ key: 'key', from: 0, to: 1, change: 1, value: Buffer.from('hello') })
  e.pipe(d)
})

test('encode + decode blob', function (end) {
  var e = protocol.encode()
  var d = protocol.decode()
  d.blob(function (blob) {
    collect(blob, function (data) {
      assert.strictEqual(data.length, 11)
      assert.deepStrictEqual(data, Buffer.from('hello world'))
      end()
    })
  })
  var blob = e.blob(11)
  blob.write('hello ')
  blob.write('world')
  blob.end()
  e.pipe(d)
})

test('encode + decode mixed blobs', function (end) {
  var expects = [Buffer.from('hello world'), Buffer.from('HELLO WORLD')]
  var seen = 0
  var e = protocol.encode()
  var d = protocol.decode()
  d.blob(function (blob, cb) {
    var exp = expects.shift()
    collect(blob, function (data) {
      assert.strictEqual(data.length, exp.length)
      assert.deepStrictEqual(data, exp)
      cb()
      if (++seen === 2) end()
    })
  })
  var b1 = e.blob(11)
  var b2 = e.blob(11)
  b1.write('hello ')
  b2.write('HELLO ')
  b1.write('world')
  b2.write('WORLD ')
  b1.end()
  b2.end()
  e.pipe(d)
})

test('encode + decode blob and changes', function (end) {
  var order = []
  var e = protocol.encode()
  var d = protocol.decode()
  d.blob(function (blob, cb) {
    collect(blob, function (data) {
      assert.deepStrictEqual(data, Buffer.from('hello world'))
      order.push('blob')
      cb()
    })
  })
  d.change(function (change, cb) {
    assert.deepStrictEqual(change, expectChange)
    order.push('change')
    cb()
    assert.deepStrictEqual(order, ['blob', 'change'])
    end()
  })
  var blob = e.blob(11)
  blob.write('hello ')
  blob.write('world')
  blob.end()
  e.change({ key: 'key', from: 0, to: 1, change: 1, value: Buffer.from('hello') })
  e.pipe(d)
})
