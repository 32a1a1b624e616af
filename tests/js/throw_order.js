// This package's side of tests/golden/ref_throws.json: tests/js/throw_driver.js over the package's
// Decoder (DRP_MOCK_NATIVE=1: the CPU stand-in addon). usage: node throw_order.js <wire> <sizes> <pattern>
'use strict'
var fs = require('fs')
var path = require('path')
var pkg = path.join(__dirname, '..', '..', 'dat-replication-protocol_amd')
if (process.env.DRP_MOCK_NATIVE === '1') require('./mock_native').install(pkg)
require('./throw_driver')(require(pkg), fs.readFileSync(process.argv[2]), process.argv[3].split(',').map(Number),
  process.argv[4], function (log) {
    process.stdout.write(JSON.stringify(log) + '\n')
    process.exit(0)
  })
