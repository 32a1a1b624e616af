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
  // per-tile look-back words (value + 1, or READY-tagged; 0 = not yet published)
  uint64_t *ywd;    // Y_t: <= 3 distinct exits landing in tile t+1 (16-bit rel + 1) | READY
  uint64_t *aggv;   // agg_t: f_t on the slots of Y_{t-1} (16-bit codes) | READY
  uint64_t *aggn;   // frames delivered by tile t on each of those paths (16-bit) | READY
  uint64_t *inclx;  // exact exit of tile t + 1
  uint64_t *aggc;   // delivered frames of tile t + 1
  uint64_t *inclc;  // frames of tiles <= t + 1
  uint64_t *tile_exit, *tile_base, *tile_count;  // per-tile records for finalize
  // per super-group (64 tiles): completion counters, composed map, count sum (value + 1)
  uint32_t *sgc_agg, *sgc_cnt;
  uint64_t *sagg, *saggn, *scnt;  // saggn: 20-bit frame counts per key
  // per-stream scratch
  uint64_t *payload_err;  // min absolute index of a malformed Change
  uint64_t *scount;       // [2*s] changes, [2*s+1] blobs
  // control
  uint32_t *counter;
  uint32_t *overflow;  // bit 0 capacity, bit 1 bounded wait expired, bit 2 inconsistent walk
  uint32_t strict;     // look-back uses exact inclusive exits only (test hook)
  // speculate-and-verify kernel (drp_decode_spec.hip): per-tile words, value | READY or value + 1
  uint64_t *claim;     // predicted exit of tile t (or identity)
  uint64_t *incl_e;    // entry of tile t + 1
  uint64_t *agg_n;     // exact frames of tile t + 1
  uint64_t *incl_n;    // frames of tiles <= t + 1
  const uint32_t *tile_stream;  // tile -> stream (null: one stream)
  uint8_t *ent;                 // [tile][thread]: entry offset in the thread's 64 B, 0xFF none
  uint8_t *ent_n, *ent_c;       // [tile][thread]: frames / change frames from that entry
  uint32_t *work;               // tiles for the general claims kernel (edge / dense tiles)
  uint32_t *work_n;             //  and their count (the fast claims kernel appends)
  uint64_t *tile_nch;           // change frames of tile t (per-stream counts come from a scan:
  uint64_t *tile_nch_base;      //  same-address atomics per tile serialise across the XCDs)
  // verify_lite: tiles it leaves to verify_counts, and each tile's first entry thread (emit skips
  // the threads before it); null: verify_counts verifies every tile
  uint32_t *vlist, *vlist_n;
  uint8_t *tile_k;
  // per tile: 1 when the tile is sparse (every thread from tile_k on delivers at most one frame,
  // at its entry; a few frames in all): emit_sparse decodes its frames from HBM without staging
  // the tile, and emit_tiles skips it (emit_sparse clears the mark of a tile it cannot take)
  uint8_t *tile_sparse;
  uint64_t *first_miss;  // per stream: the first tile a verify pass repaired (~0: none)
  // verify_counts appends the tiles whose entry a repair changed (the next repair pass verifies
  // only those); a count past dlist_cap or a nonzero dlist_n[2] means the next pass must be a
  // full one
  uint32_t *dlist, *dlist_n;
  uint64_t dlist_cap;
  uint32_t *vlist_ovf;  // vlist is a dirty list: its overflow word (set: pass the overflow on, verify nothing)
  uint32_t *dstamp;     // per tile: the last pass id whose dirty list holds it (one entry per tile per list)
  uint32_t pass_id;     // this verify pass (1: the head's; zeroed stamps before it)
  uint32_t change_checks;  // 1: claims_fast checks long frames' Change structure (drp_api.hip picks)
  int kstrong_hbm;      // 0: DRP_KSTRONG_HBM; else frames a deferred candidate must survive (tests)
  uint32_t cascade_min;  // listed tiles that make the head's verify a cascade (drp_decode_spec.hip)
  uint32_t jump_min;     // claims tiles whose link rounds hit DRP_FL_CAP before the rest take the
                         // pointer-jumping form (counted in counter[12]; drp_decode_spec.hip)
  // region walkers (drp_walk.hip): per-stream region prefix [nstreams + 1], tiles per region
  uint64_t *walk_rp;
  uint64_t *walk_entry;  // region walkers: each region's entry (walk_sync)
  uint32_t walk_hop;      // 1: the hop walkers (claims_hop), 2: by walk_dense (hop walkers or claims_fast)
  unsigned long long *walk_dense;  // walk_density's sample: bytes, frames after stream entries
  uint32_t walk_tpr;
  // claims_fast's per-frame records (null: none): CR_TILE_WORDS words per tile; per tile REC_NONE
  // (no records: the tile takes the wire-reading emission) or 0, and verification's verdict for the
  // record emission (0: not, else 1 + the slot of the tile's first row)
  uint32_t *rec;
  uint32_t *tile_rec;
  uint8_t *tile_recok;
  uint32_t *chunk_tile;  // per 64 output rows: the tile holding the first (emit_recs' aligned row chunks)
  unsigned long long *stats;  // optional event counters (DRP_STATS=1), see drp_decode.hip
  unsigned long long *trace;  // optional per-tile timestamps (DRP_TRACE_FILE, with DRP_STATS)
};

struct EncodeParams {
  drp_change_src src;
  const uint8_t *heap;
  uint64_t heap_bytes;  // rows whose key/subset/value range leaves [0, heap_bytes) are rejected
  uint64_t n;
  uint64_t *frame_off;  // [n+1] exclusive prefix of frame sizes (written)
  uint8_t *out;
  uint64_t cap;
  uint64_t *block_sum;  // per-block partial sums (scan scratch)
  uint32_t *overflow;  // bit 0 output capacity, bit 1 a row's heap range is out of bounds
  // output-stationary write (enc_write_os): per output block of ENC_BS bytes the first frame whose
  // bytes it holds, the blocks left to the per-frame writer (more frames than fit its LDS), count
  uint64_t *oblk_first;
  uint32_t *dense;
  uint32_t *dense_n;
  uint64_t nob;  // output blocks the grid covers (from cap)
};

}  // namespace drp

extern "C" {
// regions a decode's prologue fills (drp_launch_prologue): byte value, 4-byte multiples
struct ClearSet {
  static constexpr uint32_t CAP = 12;  // (a decode fills up to 9: with records, the density sample and DRP_STATS)
  void *ptr[CAP];
  uint64_t bytes[CAP];
  uint32_t value[CAP];
  uint32_t n;
};
hipError_t drp_launch_prologue(uint32_t B, const uint64_t *stream_off, uint64_t nstreams, uint64_t *tile_prefix,
                               const ClearSet *cs, hipStream_t st);
hipError_t drp_launch_tile_prefix(uint32_t B, const uint64_t *stream_off, uint64_t nstreams,
                                  uint64_t *tile_prefix, hipStream_t st);
hipError_t drp_launch_decode(uint32_t B, const drp::DecodeParams *P, uint32_t grid, hipStream_t st);
uint32_t drp_decode_waves_per_group(void);  // tiles (waves) per workgroup; grid counts groups
uint32_t drp_spec_tile_bytes(void);
uint32_t drp_spec_rec_words(void);  // u32 record words per tile (claims_fast's per-frame records)
uint32_t drp_spec_retry_mask(void);
uint32_t drp_spec_miss_bit(void);
uint32_t drp_spec_cascade_bit(void);
hipError_t drp_launch_claims_walk(const drp::DecodeParams *P, uint64_t nt_max, hipStream_t st);
uint32_t drp_walk_tiles_per_region(uint64_t nt_max, int hop);
hipError_t drp_launch_walk_density(const drp::DecodeParams *P, hipStream_t st);
hipError_t drp_launch_spec_head(const drp::DecodeParams *P, uint64_t nt_max, uint64_t nstreams,
                                uint32_t *tile_stream, hipStream_t st);
// out[0] = payload bytes of the blob rows among rows [0, n) (out zeroed by the caller)
hipError_t drp_launch_blob_bytes(const uint8_t *type, const uint32_t *plen, uint64_t n, uint64_t *out, hipStream_t st);
// ctile: 64 u32 per tile of the range (seg_claims_par; null or too small: the serial seg_claims)
hipError_t drp_launch_seg_repair(const drp::DecodeParams *P, uint64_t s, uint64_t t0, uint64_t tl, uint64_t *scratch,
                                 uint32_t *ctile, uint64_t ctile_cap, hipStream_t st);
hipError_t drp_launch_spec_verify(const drp::DecodeParams *P, uint64_t nt_max, uint64_t nstreams,
                                  uint32_t *tile_stream, hipStream_t st);
hipError_t drp_launch_spec_verify_list(const drp::DecodeParams *P, uint64_t n, uint64_t nstreams,
                                       uint32_t *tile_stream, hipStream_t st);
hipError_t drp_launch_spec_tail(const drp::DecodeParams *P, uint64_t nt_max, uint64_t nstreams,
                                uint32_t *tile_stream, uint64_t *scan_tmp, hipStream_t st);
// exclusive scan of a per-tile u64 array over all tiles; flags capacity overflow of the total
hipError_t drp_launch_tile_scan(const uint64_t *in, const uint64_t *tile_prefix, uint64_t nstreams, uint64_t nt_max,
                                uint64_t *tmp, uint64_t *out, uint64_t cap, uint32_t *overflow, hipStream_t st);
// per-stream change / blob counts from the per-tile counts and their scans
hipError_t drp_launch_stream_counts(const uint64_t *tile_prefix, uint64_t nstreams, const uint64_t *count,
                                    const uint64_t *base, const uint64_t *nch, const uint64_t *nch_base,
                                    uint64_t *scount, hipStream_t st, uint32_t *total = nullptr);
hipError_t drp_launch_finalize(const uint8_t *bytes, const uint64_t *stream_off, uint64_t nstreams,
                               const uint64_t *tile_prefix, const uint64_t *tile_exit,
                               const uint64_t *tile_base, const uint64_t *tile_count,
                               const uint64_t *payload_err, const uint64_t *scount,
                               const uint8_t *type, const uint8_t *flags, uint64_t cap,
                               drp_stream_result *res, const uint32_t *abort_flag,
                               uint32_t abort_mask, hipStream_t st);
hipError_t drp_launch_encode(const drp::EncodeParams *P, hipStream_t st);
uint64_t drp_encode_out_blocks(uint64_t cap);
// key hash + key flags for every change frame written (no-op when co->key_hash is NULL)
hipError_t drp_launch_key_post(const uint8_t *bytes, const uint64_t *tile_prefix, uint64_t nstreams,
                               const uint64_t *tile_base, const uint64_t *tile_count, uint64_t cap,
                               const drp_frames *fr, const drp_changes *co, int flags_only, const uint32_t *abort_flag,
                               uint32_t abort_mask, hipStream_t st);
hipError_t drp_launch_index_scan(const drp_stream_stats *stats, uint64_t count, uint64_t *base,
                                 hipStream_t st);
hipError_t drp_launch_stats_from_results(const drp_stream_result *res, const uint64_t *stream_off,
                                         uint64_t nstreams, drp_stream_stats *stats, hipStream_t st);
}
