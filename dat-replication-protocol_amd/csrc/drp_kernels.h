// drp_kernels.h — parameter blocks and launchers shared by the kernels and the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/drp.h"

namespace drp {

struct DecodeParams {
  const uint8_t *bytes;
  uint64_t nbytes;
  const uint64_t *stream_off;
  const uint64_t *entry;
  uint64_t nstreams;
  const uint64_t *tile_prefix;  // [nstreams+1]
  // outputs
  uint64_t *payload_off;
  uint32_t *payload_len;
  uint8_t *type;
  uint32_t *key_off, *key_len, *subset_off, *subset_len, *value_off, *value_len;
  uint64_t *change, *from, *to;
  uint8_t *flags;
  uint64_t cap;
  // per-tile scratch
  uint64_t *aggx, *inclx, *aggc, *inclc;  // look-back granules (value + 1; 0 = not yet)
  uint64_t *tile_x, *tile_exit, *tile_base, *tile_count;
  uint64_t *tile_nch, *tile_nbl, *tile_perr;  // per-tile change / blob counts, min bad frame
  const uint64_t *yover;  // per-tile corrected speculative exit (value + 1; 0 = none)
  // per-stream scratch
  uint64_t *payload_err;  // min absolute index of a malformed Change
  uint64_t *scount;       // [2*s] changes, [2*s+1] blobs
  // control
  uint32_t *counter;
  uint32_t *misspec;
  uint32_t *overflow;
  uint32_t strict;
  uint32_t *dbg;  // optional host-mapped progress markers (DRP_TRACE)
};

struct EncodeParams {
  drp_change_src src;
  const uint8_t *heap;
  uint64_t n;
  uint64_t *frame_off;  // [n+1] exclusive prefix of frame sizes (written)
  uint8_t *out;
  uint64_t cap;
  uint64_t *block_sum;  // per-block partial sums (scan scratch)
  uint32_t *overflow;
};

}  // namespace drp

extern "C" {
hipError_t drp_launch_tile_prefix(uint32_t B, const uint64_t *stream_off, uint64_t nstreams,
                                  uint64_t *tile_prefix, hipStream_t st);
hipError_t drp_launch_decode(uint32_t B, const drp::DecodeParams *P, uint32_t grid, hipStream_t st);
hipError_t drp_launch_finalize(const uint8_t *bytes, const uint64_t *stream_off, uint64_t nstreams,
                               const uint64_t *tile_prefix, const uint64_t *tile_exit,
                               const uint64_t *tile_base, const uint64_t *tile_count,
                               const uint64_t *payload_err, const uint64_t *scount,
                               const uint8_t *type, const uint8_t *flags, uint64_t cap,
                               drp_stream_result *res, hipStream_t st);
hipError_t drp_launch_peek(const uint32_t *dbg, uint32_t n, uint32_t *out, hipStream_t st);
hipError_t drp_launch_encode(const drp::EncodeParams *P, hipStream_t st);
hipError_t drp_launch_index_scan(const drp_stream_stats *stats, uint64_t count, uint64_t *base,
                                 hipStream_t st);
hipError_t drp_launch_stats_from_results(const drp_stream_result *res, const uint64_t *stream_off,
                                         uint64_t nstreams, drp_stream_stats *stats, hipStream_t st);
}
