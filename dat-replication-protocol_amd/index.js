// Same entry points as the reference (index.js:1-2).
exports.encode = require('./encode')
exports.decode = require('./decode')
