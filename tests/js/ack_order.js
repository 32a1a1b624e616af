// The package's Decoder through tests/js/ack_driver.js: prints the callback log as JSON.
// usage: node ack_order.js <wire file> <write sizes, comma separated, cycled> <burst|paced>
// DRP_MOCK_NATIVE=1: the CPU stand-in for the addon (tests/js/mock_native.js)
'use strict'
var fs = require('fs')
var path = require('path')
var pkg = path.join(__dirname, '..', '..', 'dat-replication-protocol_amd')
if (process.env.DRP_MOCK_NATIVE === '1') require('./mock_native').install(pkg)
var protocol = require(pkg)
require('./ack_driver')(protocol, fs.readFileSync(process.argv[2]), process.argv[3].split(',').map(Number),
  process.argv[4], function (log) { process.stdout.write(JSON.stringify(log) + '\n') })
