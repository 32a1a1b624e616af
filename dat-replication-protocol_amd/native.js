// Loads the N-API addon over libdrp (lib/drp.node). There is no JavaScript or CPU
// fallback: a missing addon or GPU is an error at require/first use.
'use strict'

var path = require('path')
var addon = require(path.join(__dirname, 'lib', 'drp.node'))

var ctx = null

exports.context = function () {
  if (!ctx) ctx = addon.open(Number(process.env.DRP_DEVICE || 0))
  return ctx
}
exports.decode = addon.decode
exports.decodeSync = addon.decodeSync
exports.encode = addon.encode
exports.abiVersion = addon.abiVersion
