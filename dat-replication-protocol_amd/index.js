// Same entry points as the reference (index.js:1-2).
exports.encode = require('./encode')
exports.decode = require('./decode')

// Multi-GPU (SURVEY §8e; no reference counterpart, the reference is one stream on one thread):
// independent replication streams are sharded over the node's GPUs in contiguous blocks, one
// device per stream (decode({device}) / encode({device})), and the per-stream counters are
// all-gathered over RCCL into the global index of every stream's first frame.
var native = require('./native')

exports.devices = function () { return native.deviceCount() }

// device of each of `nstreams` streams over `ndev` devices: contiguous blocks whose sizes differ
// by at most one (the same split as python/drp_dist.shard_range and bench.py's C4 shards)
exports.shard = function (nstreams, ndev) {
  if (!(ndev >= 1) || !(nstreams >= 0)) throw new RangeError('shard(nstreams, ndev): ndev >= 1')
  var base = Math.floor(nstreams / ndev)
  var extra = nstreams % ndev
  var out = new Array(nstreams)
  var s = 0
  for (var d = 0; d < ndev; d++) {
    var n = base + (d < extra ? 1 : 0)
    for (var k = 0; k < n; k++) out[s++] = d
  }
  return out
}

// Global frame index of finished streams: `decoders[i]` decoded stream i on device devs[i]
// (shard(decoders.length, ndev)). Each device contributes its block of (frames, changes, blobs,
// bytes) records; libdrp all-gathers them over RCCL (drp_index_allgather_host) and scans them.
// Returns {base: [global index of stream i's first frame], frames: [...]} in stream order.
exports.globalIndex = function (decoders, ndev) {
  ndev = ndev || Math.max(1, native.deviceCount())
  var devs = exports.shard(decoders.length, ndev)
  var per = Math.ceil(decoders.length / ndev)
  var stats = []
  var ctxs = []
  for (var d = 0; d < ndev; d++) {
    stats.push(new Float64Array(per * 4))
    ctxs.push(native.deviceContext(d))
  }
  var slot = new Array(decoders.length)
  var fill = new Array(ndev).fill(0)
  decoders.forEach(function (dec, i) {
    var d = devs[i]
    var k = fill[d]++
    slot[i] = d * per + k
    var st = stats[d]
    st[4 * k] = dec.changes + dec.blobs
    st[4 * k + 1] = dec.changes
    st[4 * k + 2] = dec.blobs
    st[4 * k + 3] = dec.bytes
  })
  var r = native.indexAllgather(ctxs, stats)
  return {
    base: slot.map(function (j) { return r.base[j] }),
    frames: slot.map(function (j) { return r.table[4 * j] })
  }
}
