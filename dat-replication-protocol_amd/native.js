// Loads the N-API addon over libdrp (lib/drp.node). There is no JavaScript or CPU
// fallback: a missing addon or GPU is an error at require/first use.
//
// Device contexts (a HIP stream + scratch each, drp_open) are pooled per device: decoders and
// encoders take them round-robin, so several streams in one process run their GPU work side by
// side (a context's calls are serialised). DRP_CTX_POOL sets the pool size per device (default
// 4); DRP_DEVICE the default device; streams can also be placed with {device: k}.
'use strict'

var path = require('path')
var addon = require(path.join(__dirname, 'lib', 'drp.node'))

var POOL = Math.max(1, Number(process.env.DRP_CTX_POOL) || 4)
var pools = {}
var nextDev = 0

exports.deviceCount = function () { return addon.deviceCount() }

exports.context = function (device) {
  if (device === undefined || device === null) device = Number(process.env.DRP_DEVICE || 0)
  var p = pools[device] || (pools[device] = { ctx: [], next: 0 })
  if (p.ctx.length < POOL) {
    var c = addon.open(device)
    p.ctx.push(c)
    return c
  }
  return p.ctx[p.next++ % p.ctx.length]
}

// the contexts of a device in creation order (one is opened when there is none yet)
exports.deviceContext = function (device) {
  var p = pools[device]
  return p && p.ctx.length ? p.ctx[0] : exports.context(device)
}

// round-robin device for a new stream when the caller gives none
exports.nextDevice = function () {
  var n = addon.deviceCount()
  return n ? nextDev++ % n : 0
}

exports.decode = addon.decode
exports.decodeSync = addon.decodeSync
exports.encode = addon.encode
exports.indexAllgather = addon.indexAllgather
exports.abiVersion = addon.abiVersion
