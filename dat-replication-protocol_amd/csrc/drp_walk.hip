// drp_walk.hip — gfx950 claims by region walkers: the claims kernel of large batches.
//
// Replaces the frame split of decode.js (Decoder._consume / _onheader, decode.js:144-169,
// 251-262) on the speculate-and-verify path, in place of claims_fast (drp_decode_spec.hip),
// with the same outputs: per 8 KiB tile its claim (the chain's first frame start past the tile,
// MARK_TERM | p for a tail, C_ID for none) and per 64-byte segment its record (entry offset |
// restart bit, frames, change frames). verify_lite / verify_counts prove them exactly as they
// prove claims_fast's, so every result still comes from the exact chain.
//
// claims_fast computes every tile from its own bytes: every live position of the tile is
// parsed and linked (~800 VALU instructions per 4 KiB wave, VALU-issue-bound). Here one LANE
// walks one REGION of consecutive interior tiles of a stream frame by frame, as decode.js does:
// the entry of a region's first tile is found once (a "sync": the first position whose Change
// payload parses exactly in the schema's shape, or whose chain survives WK_K frames), and every
// later frame start follows from its predecessor's header. The VALU work is per frame, not per
// byte (C2: ~1.5 frames per 128-byte window and lane).
//
// Data movement: the 64 regions of a wave advance together, 128 bytes (one "window") each per
// step. A step stages the windows of all 64 regions with LDS-DMA (8 global_load_lds_dwordx4 per
// step, each one 128-byte line of 8 regions: full lines, no VGPRs), three steps ahead into a ring
// of 4 slots (8 KiB each), so 16 KiB per wave are in flight while two windows are walked. One
// wave per workgroup (32 KiB of LDS: 5 per CU). The wire is read from HBM once; the kernel writes
// 3 bytes of records per 64 bytes and one claim per tile.
//
// Regions never cross a stream and hold only interior tiles (A >= stream start, A + IMG <= stream
// end); the edge tiles go to spec_claims' work list, as claims_fast sends them.
#include "drp_spec.h"

namespace drp {
namespace spec {

#ifndef DRP_WK_WB
#define DRP_WK_WB 128
#endif
constexpr uint32_t WK_WB = DRP_WK_WB;            // window bytes per region and step
constexpr uint32_t WK_WPT = TILE / WK_WB;        // windows per tile
constexpr uint32_t WK_GW = 512 / WK_WB;          // windows per group of 8 segment records
constexpr uint32_t WK_LPR = WK_WB / 16;          // lanes of one DMA instruction per region
constexpr uint32_t SY_NEAR = 256;                // a "near" sync chain's longest frame
constexpr uint64_t SY_TAIL = 16384;              // a sync chain's tail counts this close to the stream end
#ifndef DRP_SY_MERGE
#define DRP_SY_MERGE 1024
#endif
constexpr uint64_t SY_MERGE = DRP_SY_MERGE;              // a region's entry before its first shaped Change: this close
constexpr uint64_t SY_SHAPE = 8192;              // how far a region's first shaped Change is looked for
constexpr uint64_t SY_GENERAL = 2048;            // how far the general scan looks (else: no entry, the
                                                 // region's tiles claim identity and verification walks them)
#ifndef DRP_WK_SLOTS
#define DRP_WK_SLOTS 4
#define DRP_WK_AHEAD 3
#endif
#ifndef DRP_WK_REGIONS
#define DRP_WK_REGIONS 65536
#endif
constexpr uint32_t WK_SLOTS = DRP_WK_SLOTS;      // LDS ring slots
constexpr uint32_t WK_AHEAD = DRP_WK_AHEAD;      // windows staged ahead of the one walked
static_assert(WK_AHEAD == 2 || WK_AHEAD == 3, "the wait accounting below covers these");
constexpr uint32_t WK_SLOT = WAVE * WK_WB;       // bytes per slot (8 KiB)
constexpr uint32_t WK_NDMA = WK_SLOT / (WAVE * 16);  // DMA instructions per step (8)
constexpr uint32_t WK_K = 8;                     // frames a sync chain must survive (no Change shape)
constexpr uint32_t WK_REGIONS = DRP_WK_REGIONS;  // regions aimed at (one per resident lane)
#ifndef DRP_HOP_REGIONS
#define DRP_HOP_REGIONS 24576
#endif
constexpr uint32_t HOP_REGIONS = DRP_HOP_REGIONS;  // hop walkers: regions aimed at
static_assert(WK_WB == 64 || WK_WB == 128, "windows of one or two segments");
static_assert(WK_SLOTS >= WK_AHEAD + 1, "the ring holds the walked window, the next and the in-flight ones");

enum : uint32_t { WM_WALK = 1, WM_DONE = 2 };

// Interior tiles of stream s: i in [i_lo, i_lo + n) of its tiles (A_i = base + i * TILE).
struct Interior {
  uint64_t base, so, se;
  uint64_t i_lo, n;
};
__device__ __forceinline__ Interior interior(const DecodeParams &P, uint64_t s) {
  Interior I;
  I.so = P.stream_off[s];
  I.se = P.stream_off[s + 1];
  I.base = I.so & ~(uint64_t)(TILE - 1);
  const uint64_t nt = P.tile_prefix[s + 1] - P.tile_prefix[s];
  I.i_lo = I.base == I.so ? 0 : 1;
  I.n = 0;
  if (I.se >= I.base + IMG) {
    const uint64_t i_hi = umin64((I.se - IMG - I.base) / TILE, nt ? nt - 1 : 0);  // (inclusive)
    if (nt && i_hi >= I.i_lo) I.n = i_hi - I.i_lo + 1;
  }
  return I;
}

// One workgroup: every stream's region count (prefix into P.walk_rp[0..ns]) and its edge tiles
// appended to P.work (one atomic per wave).
__global__ __launch_bounds__(1024) void walk_regions(DecodeParams P) {
  __shared__ uint64_t part[1024];
  __shared__ uint64_t carry;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint64_t c0 = 0; c0 < P.nstreams; c0 += 1024) {
    const uint64_t s = c0 + tid;
    uint64_t nr = 0;
    uint32_t nedge = 0;
    uint64_t edge[3] = {0, 0, 0};
    if (s < P.nstreams) {
      const Interior I = interior(P, s);
      const uint64_t tf = P.tile_prefix[s], nt = P.tile_prefix[s + 1] - tf;
      nr = (I.n + P.walk_tpr - 1) / P.walk_tpr;
      // edge tiles: before i_lo (at most one) and after the last interior tile (at most two)
      // (a stream with no interior tile: all of its tiles; streams that short have few)
      const uint64_t lo = I.n ? I.i_lo : nt, hi = I.n ? I.i_lo + I.n : nt;
      for (uint64_t i = 0; i < nt; i++) {
        if (i >= lo && i < hi) {
          i = hi - 1;
          continue;
        }
        if (nedge < 3) edge[nedge++] = tf + i;
        else P.work[atomicAdd(P.work_n, 1u)] = (uint32_t)(tf + i);  // (only streams without interior tiles)
      }
    }
    // one atomic per wave for the edge tiles
    uint32_t inc = nedge;
#pragma unroll
    for (uint32_t d = 1; d < WAVE; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, d, WAVE);
      if (lane >= d) inc += y;
    }
    const uint32_t total = (uint32_t)__shfl((int)inc, 63, WAVE);
    uint32_t wb = 0;
    if (lane == 63 && total) wb = atomicAdd(P.work_n, total);
    wb = (uint32_t)__shfl((int)wb, 63, WAVE);
    for (uint32_t k = 0; k < nedge; k++) P.work[wb + inc - nedge + k] = (uint32_t)edge[k];
    part[tid] = nr;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
      const uint64_t v = tid >= d ? part[tid - d] : 0;
      __syncthreads();
      part[tid] += v;
      __syncthreads();
    }
    if (s < P.nstreams) P.walk_rp[s] = carry + part[tid] - nr;
    __syncthreads();
    if (tid == 1023) carry += part[1023];
    __syncthreads();
  }
  if (tid == 0) P.walk_rp[P.nstreams] = carry;
}

// ---- the walker -------------------------------------------------------------------------------
struct WalkLds {
  __attribute__((aligned(16))) uint32_t ring[WK_SLOTS * WK_SLOT / 4];
};

// dword of this lane's bytes at window-relative offset o (4-aligned, o < 2 * WK_WB: the window
// walked and the next one), from the ring
__device__ __forceinline__ uint32_t wk_rd(const WalkLds &S, uint32_t w, uint32_t o) {
  const uint32_t slot = (w + o / WK_WB) % WK_SLOTS;
  return S.ring[(slot * WK_SLOT + threadIdx.x * WK_WB + (o & (WK_WB - 1))) >> 2];
}

// the 8 bytes at window-relative offset o (o + 8 <= 2 * WK_WB + 4: the ring's two windows plus
// one dword), little endian
__device__ __forceinline__ uint64_t wk_rd8(const WalkLds &S, uint32_t w, uint32_t o) {
  const uint32_t d = o & ~3u, sh = (o & 3u) * 8u;
  const uint32_t a = wk_rd(S, w, d), b = wk_rd(S, w, d + 4), c = wk_rd(S, w, d + 8);
  const uint32_t lo = __builtin_amdgcn_alignbit(b, a, sh), hi = __builtin_amdgcn_alignbit(c, b, sh);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// 8 bytes at absolute position p from the batch (two aligned 8-byte loads; p + 16 <= nbytes).
// The value is waited for here, in the caller's branch: left to the compiler, the wait (a
// vmcnt(0), which also drains the ring's DMAs in flight) lands where the branch merges with the
// ring-read path, and every ring read pays for it.
__device__ __forceinline__ uint64_t g_rd8(const uint8_t *g, uint64_t p) {
  const uint64_t *q = reinterpret_cast<const uint64_t *>(g + (p & ~7ull));
  const uint32_t sh = (uint32_t)(p & 7u) * 8u;
  const uint64_t a = q[0], b = q[1];
  uint64_t x = sh ? (a >> sh) | (b << (64 - sh)) : a;
  asm volatile("" : "+v"(x));
  return x;
}

// 8 bytes at absolute position p from one 16-byte load at p's dword (the hop walkers: one memory
// request per frame; p + 16 <= nbytes + 3)
typedef uint32_t wk_u32x4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ uint64_t g_rd8x(const uint8_t *g, uint64_t p) {
  const wk_u32x4 v = *reinterpret_cast<const wk_u32x4 *>(g + (p & ~3ull));
  const uint32_t sh = (uint32_t)(p & 3u) * 8u;
  return (uint64_t)__builtin_amdgcn_alignbit(v.y, v.x, sh) | ((uint64_t)__builtin_amdgcn_alignbit(v.z, v.y, sh) << 32);
}

// A frame header from its first 8 bytes x: the length varint of 1..5 bytes, then the id.
// k = 0: a longer varint (L >= 2^35: the slow path decides).
struct WHdr {
  uint64_t L;
  uint32_t k, id;
};
__device__ __forceinline__ WHdr wk_hdr(uint64_t x) {  // (branch-free)
  WHdr h;
  const uint64_t tm = ~x & 0x8080808080ull;
  const uint32_t k = ((uint32_t)__builtin_ctzll(tm | (1ull << 63)) >> 3) + 1u;  // (8: none)
  const uint64_t v = (x & 0x7Full) | ((x >> 1) & 0x3F80ull) | ((x >> 2) & 0x1FC000ull) | ((x >> 3) & 0xFE00000ull) |
                     ((x >> 4) & 0x7F0000000ull);
  const bool ok = k <= 5u;
  h.k = ok ? k : 0u;
  h.L = ok ? v & ((1ull << (7u * k)) - 1ull) : 0ull;
  h.id = ok ? (uint32_t)(x >> (8u * k)) & 0xFFu : 0xFFu;
  return h;
}

// Byte reader for the sync checks: this lane's windows w, w + 1 from the ring, anything else
// from the batch (rare: Change fields past the next window).
struct WkReader {
  const WalkLds &S;
  const uint8_t *g;
  uint64_t W0, nbytes;
  uint32_t w;
  __device__ __forceinline__ uint64_t rd8(uint64_t p) const {
    const uint64_t o = p - W0;
    if (o + 12 <= 2 * WK_WB) return wk_rd8(S, w, (uint32_t)o);
    if (p + 16 > nbytes) return 0;  // (past the batch: parses as nothing valid)
    return g_rd8(g, p);
  }
};

// Byte reader for the region syncs (walk_sync): the batch, read through the caches.
struct GReader {
  const uint8_t *g;
  uint64_t nbytes;
  __device__ __forceinline__ uint64_t rd8(uint64_t p) const {
    if (p + 16 > nbytes) return 0;  // (past the batch: parses as nothing valid)
    return g_rd8(g, p);
  }
};

// Sync check of a Change candidate: its payload [po, po + pl) parses in the schema's own shape
// (one-byte tags with their wire types, in protocol-buffers' field order: [subset] key change
// from to [value], varint numbers of <= 10 bytes, lengths inside the payload) and its last field
// ends exactly at the payload end. 1: strong; 0: not a Change of that shape. Prediction only.
template <class Rd>
__device__ __forceinline__ uint32_t wk_change_shape(const Rd &R, uint64_t po, uint64_t pl) {
  uint64_t off = 0;
  uint32_t last = 0;  // the field number of the previous field (schema order)
#pragma unroll 1
  for (uint32_t f = 0; f < 6u; f++) {
    if (off >= pl) break;
    const uint64_t x = R.rd8(po + off);
    const uint32_t b0 = (uint32_t)x & 0xFFu, fn = b0 >> 3, wt = b0 & 7u;
    if (b0 >= 0x80u || fn < 1u || fn > 6u || fn <= last) return 0;
    const bool num = fn >= 3u && fn <= 5u;
    if (wt != (num ? 0u : 2u)) return 0;
    if ((fn == 3u && last < 2u) || (fn > 3u && last != fn - 1u)) return 0;  // key, change, from, to: required, in order
    const uint64_t y = x >> 8;  // the varint (<= 5 bytes read here; longer numbers: a second read)
    const uint64_t tm = ~y & 0x8080808080ull;
    uint32_t kb;
    uint64_t v;
    if (tm) {
      kb = ((uint32_t)__builtin_ctzll(tm) >> 3) + 1u;
      v = ((y & 0x7Full) | ((y >> 1) & 0x3F80ull) | ((y >> 2) & 0x1FC000ull) | ((y >> 3) & 0xFE00000ull) |
           ((y >> 4) & 0x7F0000000ull)) & ((1ull << (7u * kb)) - 1ull);
    } else {
      if (!num) return 0;  // a length of >= 2^35
      const uint64_t z = R.rd8(po + off + 6);  // varint bytes 5..12
      const uint64_t tz = ~z & 0x8080808080ull;
      if (!tz) return 0;
      kb = 5u + ((uint32_t)__builtin_ctzll(tz) >> 3) + 1u;
      if (kb > 10u) return 0;
      v = 0;
    }
    if (1u + kb > pl - off) return 0;
    off += 1u + kb;
    if (!num) {
      if (v > pl - off) return 0;
      off += v;
    }
    last = fn;
  }
  return (off == pl && last >= 5u) ? 1u : 0u;
}

// A complete Change frame at c whose payload has the schema's shape (wk_change_shape) and whose
// next header is valid: strong by itself.
template <class Rd>
__device__ __forceinline__ bool wk_shaped(const Rd &R, uint64_t c, uint64_t se) {
  if (c >= se) return false;
  const WHdr h = wk_hdr(R.rd8(c));
  if (h.k == 0 || h.id != 1u || h.L <= 1 || h.L - 1 > se - c - h.k - 1) return false;
  if (!wk_change_shape(R, c + h.k + 1u, h.L - 1u)) return false;
  const uint64_t n = c + h.k + h.L;
  if (n >= se) return true;
  const WHdr g = wk_hdr(R.rd8(n));
  return g.k != 0 && g.id <= 2u && (g.id == 0 || g.L != 0);
}

// Does the chain from candidate c survive? A header is valid when its id is <= 2 (and a Change or
// blob declares a length); a Change frame must start with a Change tag. Steps past the two ring
// windows read the batch. 1: survives WK_K frames, or ends at the stream end (exactly, or in a
// tail starting within SY_TAIL of it) after at least two complete frames (a shadow header whose
// varint swallows a real one's length bytes declares a frame of ~1 MB+, which the batch cuts: no
// evidence alone).
// near: no frame of the chain is longer than the two ring windows.
template <class Rd>
__device__ __forceinline__ bool wk_survives(const Rd &R, uint64_t c, uint64_t se, bool &near) {
  uint64_t p = c;
  near = true;
#pragma unroll 1
  for (uint32_t f = 0; f < WK_K; f++) {
    if (p >= se) return p == se && f >= 2u;
    const uint64_t x = R.rd8(p);
    const WHdr h = wk_hdr(x);
    if (h.k == 0 || h.id > 2u || (h.id != 0 && h.L == 0)) return false;
    if (h.id == 0) {
      p += h.k + 1u;
      continue;
    }
    // a tail (the chain ends in a frame the stream end cuts): evidence only close to that end; a
    // header whose varint swallows a real header's declares a frame of ~64 MB+ (C5: 4 KB frames
    // with 2-byte lengths), a "tail" wherever it lies
    if (h.L > se - p - h.k) return f >= 2u && se - p <= SY_TAIL;
    near = near && h.k + h.L <= SY_NEAR;
    if (h.id == 1) {
      const uint32_t t = (h.k < 7u) ? (uint32_t)(x >> (8u * (h.k + 1u))) & 0xFFu : (uint32_t)R.rd8(p + h.k + 1) & 0xFFu;
      constexpr uint64_t TAGS = (1ull << 0x0a) | (1ull << 0x12) | (1ull << 0x18) | (1ull << 0x20) | (1ull << 0x28) |
                                (1ull << 0x32);
      if (h.L > 1 && !(t < 64u && ((TAGS >> t) & 1ull))) return false;
    }
    p += h.k + h.L;
  }
  return true;
}

// Byte masks of 16 positions from 20 bytes (a, b, c, d, e: dwords): bit i of the result is set
// when position i can start a header: a length varint of 1..3 bytes followed by a byte <= 2.
__device__ __forceinline__ uint32_t wk_live16(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e) {
  constexpr uint32_t H = 0x80808080u;
  auto le2 = [](uint32_t x) { return ~(((x | 0x80808080u) - 0x03030303u) | x) & 0x80808080u; };
  auto g4 = [](uint32_t x) {  // MSBs of the 4 bytes -> bits 0..3
    return ((x >> 7) & 1u) | ((x >> 14) & 2u) | ((x >> 21) & 4u) | ((x >> 28) & 8u);
  };
  const uint32_t M = g4(a & H) | (g4(b & H) << 4) | (g4(c & H) << 8) | (g4(d & H) << 12) | (g4(e & H) << 16);
  const uint32_t S = g4(le2(a)) | (g4(le2(b)) << 4) | (g4(le2(c)) << 8) | (g4(le2(d)) << 12) | (g4(le2(e)) << 16);
  const uint32_t X = ~M & (S >> 1);                                  // varint terminator then id <= 2
  return (X | (M & ((X >> 1) | ((M >> 1) & (X >> 2))))) & 0xFFFFu;  // through 0, 1 or 2 MSB bytes
}

// ---- per-frame records for the record emission (emit_rec) ------------------------------------
// One delivered frame as 32 bytes: what decode_change and the frame table write for it, so that
// the emission expands records into columns without reading the wire again.
//   x: payload offset from the tile's first byte (14 bits) | id << 14 | partial << 16 |
//      DRP_F_SUBSET << 17 | DRP_F_VALUE << 18        y: payload length (clamped as the column)
//   z: key_off | subset_off << 8 | key_len << 16     w: value_off | subset_len << 16
//   then change, from, to (low 32 bits) and their bits 32..41 (10 bits each)
// Only Change payloads in protocol-buffers' own shape are recorded ([subset] key change from to
// [value], one-byte tags, lengths of < 2^28 in <= 4 bytes, numbers of < 2^42, the last field
// ending the payload, every offset and length inside its field); any other frame makes its tile
// take the wire-reading emission (emit_lean / emit_tiles), as does a region whose records
// overflow its share of the record buffer.
constexpr uint32_t WK_REC_BYTES = 64;  // the record buffer holds one record per this many wire bytes

// a varint of <= n bytes from y (little endian): bytes used (0: none ends within n)
__device__ __forceinline__ uint32_t wk_varint(uint64_t y, uint32_t n, uint64_t &v) {
  const uint64_t tm = ~y & 0x808080808080ull & ((1ull << (8u * n)) - 1ull);
  if (!tm) return 0;
  const uint32_t kb = ((uint32_t)__builtin_ctzll(tm) >> 3) + 1u;
  v = ((y & 0x7Full) | ((y >> 1) & 0x3F80ull) | ((y >> 2) & 0x1FC000ull) | ((y >> 3) & 0xFE00000ull) |
       ((y >> 4) & 0x7F0000000ull) | ((y >> 5) & 0x3F800000000ull)) &
      ((1ull << (7u * kb)) - 1ull);
  return kb;
}

// One field at q: its tag byte must be `tag`, then a varint of <= n bytes (into v: 0 when there is
// none) inside [q, end); returns the field's header bytes (tag + varint), and clears ok when the
// field is not there. Computed without early exits: the record's checks below run as one
// straight-line sequence (divergent early returns out of this parse were miscompiled into
// records with zeroed numbers: change / to columns of 0 on every frame).
__device__ __forceinline__ uint32_t wk_field(const WkReader &R, uint64_t q, uint64_t end, uint32_t tag, uint32_t n,
                                             uint64_t &v, bool &ok) {
  const uint64_t x = R.rd8(q);
  v = 0;
  const uint32_t kb = wk_varint(x >> 8, n, v);
  ok = ok && q < end && (x & 0xFFu) == tag && kb != 0 && 1u + kb <= end - q;
  return 1u + kb;
}

__device__ __forceinline__ bool wk_record(const WkReader &R, uint64_t po, uint64_t pl, uint4 &a, uint4 &b) {
  const uint64_t end = po + pl;
  uint64_t q = po, slen = 0, klen = 0, nc = 0, nf = 0, nt = 0, vlen = 0;
  bool ok = true, sub = (R.rd8(q) & 0xFFu) == 0x0Au, sok = true;
  const uint32_t sh = wk_field(R, q, end, 0x0Au, 4, slen, sok);  // subset (when its tag is there)
  ok = !sub || (sok && slen <= end - q - sh && slen < 0x10000u);
  const uint32_t soff = sub ? sh : 0u;
  slen = sub ? slen : 0u;
  q = sub && ok ? q + sh + slen : q;
  const uint32_t kh = wk_field(R, q, end, 0x12u, 4, klen, ok);  // key
  ok = ok && klen <= end - q - kh && klen < 0x10000u && q - po + kh < 0x100u;
  const uint32_t koff = (uint32_t)(q - po) + kh;
  q = ok ? q + kh + klen : end;
  q += wk_field(R, q, end, 0x18u, 6, nc, ok);  // change
  q += wk_field(R, q, end, 0x20u, 6, nf, ok);  // from
  q += wk_field(R, q, end, 0x28u, 6, nt, ok);  // to
  const bool val = ok && q != end;  // value: the last field
  bool vok = true;
  const uint32_t vh = wk_field(R, q, end, 0x32u, 4, vlen, vok);
  ok = ok && (!val || (vok && vlen == end - q - vh && q - po + vh < 0x10000u));
  const uint32_t fl = (sub ? DRP_F_SUBSET : 0u) | (val ? DRP_F_VALUE : 0u);
  a.x |= fl << 17;
  a.z = koff | (soff << 8) | ((uint32_t)klen << 16);
  a.w = (val ? (uint32_t)(q - po) + vh : 0u) | ((uint32_t)slen << 16);
  b.x = (uint32_t)nc;
  b.y = (uint32_t)nf;
  b.z = (uint32_t)nt;
  b.w = (uint32_t)(nc >> 32) | ((uint32_t)(nf >> 32) << 10) | ((uint32_t)(nt >> 32) << 20);
  return ok;
}

// s_waitcnt vmcnt(n) for a count known only at run time (wave-uniform): the largest immediate
// <= n of a small set (waiting for more operations than needed is always safe)
__device__ __forceinline__ void wk_wait_vm(uint32_t n) {
  n = __builtin_amdgcn_readfirstlane(n);  // (scalar branches)
  if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if (n >= 28) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
  else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (n >= 22) asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
  else if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else if (n >= 19) asm volatile("s_waitcnt vmcnt(19)" ::: "memory");
  else if (n >= 18) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
  else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Region r of the batch: its first tile (t0, at A0), its stream end, its windows, and for a
// stream's first tile the exact entry.
struct Region {
  uint64_t t0, A0, se, entry;
  uint32_t nw;
  bool exact;
};
__device__ __forceinline__ Region region_of(const DecodeParams &P, uint64_t r) {
  uint64_t s = 0;
  if (P.nstreams > 1) {  // walk_rp[s] <= r < walk_rp[s + 1]
    uint64_t lo = 0, hi = P.nstreams;
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (P.walk_rp[mid] <= r) lo = mid;
      else hi = mid;
    }
    s = lo;
  }
  const Interior I = interior(P, s);
  const uint64_t i0 = I.i_lo + (r - P.walk_rp[s]) * P.walk_tpr;
  Region G;
  G.t0 = P.tile_prefix[s] + i0;
  G.A0 = I.base + i0 * TILE;
  G.se = I.se;
  G.nw = (uint32_t)umin64(P.walk_tpr, I.i_lo + I.n - i0) * WK_WPT;
  G.exact = G.A0 == I.so;
  G.entry = I.so + (P.entry ? P.entry[s] : 0ull);
  return G;
}

// ---- region syncs ----------------------------------------------------------------------------
// One lane per region: the entry its walker starts from (P.walk_entry[r]; NONE: no chain found in
// the region, whose tiles then claim identity). A stream's first tile has its exact entry. Else,
// first, the region's first "shaped" candidate: a complete Change whose payload parses in the
// schema's own shape and whose next header is valid (random bytes essentially never pass; the
// checks read only the candidate's own bytes). Before it, a candidate whose chain survives WK_K
// short frames ("near": <= 256 bytes each, so the checks stay in the cached bytes around it) is
// taken instead (the region starts in blobs or other frames); a chain that survives by landing on
// a shaped Change right after its first frame is taken at that Change (the candidate itself is
// most likely a shadow merging into the real chain). Only a region with no shaped candidate at all
// (blobs, non-Change data) runs the general scan, which also weighs "far" chains (see
// sync_general). Prediction only: verification proves the claims.
template <class Rd>
__device__ __forceinline__ uint32_t sync_live16(const Rd &R, uint64_t p) {
  const uint64_t x0 = R.rd8(p), x1 = R.rd8(p + 8);
  return wk_live16((uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32), (uint32_t)R.rd8(p + 16));
}

// live positions of the 64 bytes x[0..7] (x: 72 bytes; 4 masks of 16)
__device__ __forceinline__ uint64_t sync_live64w(const uint64_t *x) {
  uint64_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; i++)
    m |= (uint64_t)wk_live16((uint32_t)x[2 * i], (uint32_t)(x[2 * i] >> 32), (uint32_t)x[2 * i + 1],
                             (uint32_t)(x[2 * i + 1] >> 32), (uint32_t)x[2 * i + 2]) << (16 * i);
  return m;
}

// live positions of 64 bytes [p, p + 64) (the loads issued together)
__device__ __forceinline__ uint64_t sync_live64(const GReader &R, uint64_t p) {
  uint64_t x[9];
#pragma unroll
  for (int i = 0; i < 9; i++) x[i] = R.rd8(p + 8u * i);
  uint64_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; i++)
    m |= (uint64_t)wk_live16((uint32_t)x[2 * i], (uint32_t)(x[2 * i] >> 32), (uint32_t)x[2 * i + 1],
                             (uint32_t)(x[2 * i + 1] >> 32), (uint32_t)x[2 * i + 2]) << (16 * i);
  return m;
}

// The general scan (a region without a shaped candidate near its start): candidates in order. A
// candidate must survive WK_K frames; it is taken at once when near, else ("far") the first one
// is held back while the scan goes on, up to its successor or its tile's end, and dropped for a
// near candidate: a header whose length varint swallows a real header's first bytes declares a
// frame of ~1 MB that lands on the real chain with odds of one in the real frame size, and then
// "survives". At the held-back chain's successor the scan stops: when the held-back frame is
// short and its successor is a shaped Change, the chain is taken there, else at the held-back
// candidate.
__device__ __forceinline__ uint64_t sync_general(const GReader &R, uint64_t A0, uint64_t end, uint64_t se) {
  uint64_t far_c = 0, far_n = 0, far_t = 0;
#pragma unroll 1
  for (uint64_t c64 = A0; c64 < end; c64 += 64u) {
    uint64_t live = sync_live64(R, c64);
#pragma unroll 1
    while (live) {
      const uint64_t c = c64 + (uint32_t)__builtin_ctzll(live);
      live &= live - 1u;
      if (far_c && (c >= far_n || c >= far_t)) {
        if (c >= far_n && far_n - far_c <= SY_NEAR && wk_shaped(R, far_n, se)) return far_n;
        return far_c;
      }
      const WHdr h = wk_hdr(R.rd8(c));
      if (h.k == 0 || h.id > 2u || (h.id != 0 && h.L == 0)) continue;
      bool near = false;
      if (!wk_survives(R, c, se, near)) continue;
      if (near) {
        const uint64_t n1 = c + h.k + (h.id ? h.L : 1u);
        return n1 - c <= SY_NEAR && wk_shaped(R, n1, se) ? n1 : c;
      }
      if (!far_c) {
        far_c = c;
        far_n = c + h.k + h.L;
        far_t = ((c - A0) / TILE + 1) * TILE + A0;  // (its tile's end)
      }
    }
  }
  return far_c ? far_c : ~0ull;
}

// Positions of 16 bytes (from 20: dwords a..e) that can start a Change header followed by the
// schema's first tag: a length varint of 1..3 bytes, the id 1, then 0x0a (subset) or 0x12 (key).
// Every shaped candidate is one; random bytes give one in ~2^15 positions, so the shape check's
// reads are only made for these.
__device__ __forceinline__ uint32_t wk_shape16(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e) {
  auto zero8 = [](uint32_t y) { return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u; };  // (exact)
  auto g4 = [](uint32_t x) { return ((x >> 7) & 1u) | ((x >> 14) & 2u) | ((x >> 21) & 4u) | ((x >> 28) & 8u); };
  const uint32_t w[5] = {a, b, c, d, e};
  uint32_t HI = 0, E1 = 0, T = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    HI |= g4(w[i] & 0x80808080u) << (4 * i);
    E1 |= g4(zero8(w[i] ^ 0x01010101u)) << (4 * i);
    T |= g4(zero8(w[i] ^ 0x0a0a0a0au) | zero8(w[i] ^ 0x12121212u)) << (4 * i);
  }
  const uint32_t LO = ~HI;
  const uint32_t m1 = LO & (E1 >> 1) & (T >> 2);
  const uint32_t m2 = HI & (LO >> 1) & (E1 >> 2) & (T >> 3);
  const uint32_t m3 = HI & (HI >> 1) & (LO >> 2) & (E1 >> 3) & (T >> 4);
  return (m1 | m2 | m3) & 0xFFFFu;
}

// Is there a byte pair 0x01, then 0x0a or 0x12, at positions q, q + 1 with q in [0, 132) of the
// 136 bytes in x? Every shape candidate in the first 128 of them has one (its id byte, then the
// first tag), so the exact masks are only computed for a block that passes (~1 in 240 of random
// 128-byte blocks; once per real Change header). ~5 VALU per byte instead of ~13.
__device__ __forceinline__ bool sync_pairs136(const uint64_t *x) {
  auto zero8 = [](uint32_t y) { return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u; };  // (exact)
  auto tag = [&](uint32_t w) { return zero8(w ^ 0x0a0a0a0au) | zero8(w ^ 0x12121212u); };
  uint32_t any = 0;
  uint32_t t = tag((uint32_t)x[0]);
#pragma unroll
  for (int j = 0; j < 33; j++) {
    const uint32_t w = j & 1 ? (uint32_t)(x[j >> 1] >> 32) : (uint32_t)x[j >> 1];
    const uint32_t wn = (j + 1) & 1 ? (uint32_t)(x[(j + 1) >> 1] >> 32) : (uint32_t)x[(j + 1) >> 1];
    const uint32_t tn = tag(wn);
    any |= zero8(w ^ 0x01010101u) & __builtin_amdgcn_alignbit(tn, t, 8);  // (tag of the byte after)
    t = tn;
  }
  return any != 0;
}

// shape-candidate positions of the 128 bytes x[0..15] (x: 136 bytes)
__device__ __forceinline__ uint64_t sync_shape128(const uint64_t *x, uint64_t &hi) {
  uint64_t lo = 0;
  hi = 0;
  if (!sync_pairs136(x)) return 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t m = wk_shape16((uint32_t)x[2 * i], (uint32_t)(x[2 * i] >> 32), (uint32_t)x[2 * i + 1],
                                  (uint32_t)(x[2 * i + 1] >> 32), (uint32_t)x[2 * i + 2]);
    if (i < 4) lo |= m << (16 * i);
    else hi |= m << (16 * (i - 4));
  }
  return lo;
}

// Does the chain from c reach exactly `to` (every frame complete before it, <= 16 frames)?
__device__ __forceinline__ bool sync_merges(const GReader &R, uint64_t c, uint64_t to) {
  uint64_t p = c;
#pragma unroll 1
  for (uint32_t f = 0; f < 16u && p < to; f++) {
    const WHdr h = wk_hdr(R.rd8(p));
    if (h.k == 0 || h.id > 2u || (h.id != 0 && h.L == 0)) return false;
    p += h.k + (h.id ? h.L : 1u);
  }
  return p == to;
}

// A region's sync runs on SY_LANES consecutive lanes (a group): each step of the scans gives every
// lane of the group its own block, in address order, and the group takes the first lane that found
// (a ballot), so the result is the one-lane scan's. More lanes per region puts more waves on the
// SIMDs: the scans are chains of dependent loads, and one lane per region left one wave per SIMD
// with nothing to overlap its waits.
#ifndef DRP_SY_LANES
#define DRP_SY_LANES 8
#endif
constexpr uint32_t SY_LANES = DRP_SY_LANES;
static_assert(SY_LANES == 1 || SY_LANES == 2 || SY_LANES == 4 || SY_LANES == 8, "lanes per region");

// the group's lanes holding b (bit j: the group's lane j)
__device__ __forceinline__ uint32_t grp_ballot(bool b, uint32_t lane) {
  return (uint32_t)((__ballot(b) >> (lane & ~(SY_LANES - 1u))) & ((1u << SY_LANES) - 1u));
}
// v of the group's lane j
__device__ __forceinline__ uint64_t grp_take(uint64_t v, uint32_t lane, uint32_t j) {
  const int src = (int)((lane & ~(SY_LANES - 1u)) + j);
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// The entry of region G (see above), on the group's lane `sub` (every lane of the group returns it;
// the general scan's only on sub 0).
__device__ __forceinline__ uint64_t sync_entry(const DecodeParams &P, const Region &G, uint32_t lane, uint32_t sub,
                                               uint64_t &t_shape) {
  if (G.exact) return G.entry;
  const GReader R{P.bytes, P.nbytes};
  const uint64_t se = G.se, end = G.A0 + (uint64_t)(G.nw / WK_WPT) * TILE;
  // the first shaped candidate (within SY_SHAPE bytes: a stream without Changes goes on to the
  // general scan soon), 128 bytes per lane and step
  uint64_t shaped = ~0ull;
  const uint64_t aend = umin64(end, G.A0 + SY_SHAPE);
#pragma unroll 1
  for (uint64_t cs = G.A0; cs < aend; cs += 128u * SY_LANES) {
    const uint64_t c128 = cs + 128u * sub;
    uint64_t found = ~0ull;
    if (c128 < aend) {
      if (P.stats) atomicAdd(&P.stats[40], 1ull);
      uint64_t x[17];
#pragma unroll
      for (uint32_t i = 0; i < 17; i++) x[i] = R.rd8(c128 + 8u * i);
      uint64_t hi;
      uint64_t m = sync_shape128(x, hi);
#pragma unroll 1
      for (uint32_t half = 0; half < 2u && found == ~0ull; half++, m = hi) {
#pragma unroll 1
        while (m) {
          const uint64_t c = c128 + 64u * half + (uint32_t)__builtin_ctzll(m);
          m &= m - 1u;
          if (P.stats) atomicAdd(&P.stats[41], 1ull);
          if (wk_shaped(R, c, se)) {
            found = c;
            break;
          }
        }
      }
    }
    const uint32_t fm = grp_ballot(found != ~0ull, lane);
    if (fm) {
      shaped = grp_take(found, lane, (uint32_t)__builtin_ctz(fm));
      break;
    }
  }
  t_shape = P.stats ? __builtin_amdgcn_s_memtime() : 0;
  if (shaped == ~0ull) {
    if (sub) return ~0ull;
    if (P.stats) atomicAdd(&P.stats[44], 1ull);
    return sync_general(R, G.A0, umin64(end, G.A0 + SY_GENERAL), se);
  }
  // an earlier candidate (up to SY_MERGE bytes before it) whose chain lands exactly on it: the
  // region starts in other frames (blobs, short frames); 64 bytes per lane and step
  const uint64_t from = shaped - G.A0 > SY_MERGE ? (shaped - SY_MERGE) & ~63ull : G.A0;
#pragma unroll 1
  for (uint64_t cs = from; cs < shaped; cs += 64u * SY_LANES) {
    const uint64_t c64 = cs + 64u * sub;
    uint64_t found = ~0ull;
    if (c64 < shaped) {
      uint64_t x[9];
#pragma unroll
      for (uint32_t i = 0; i < 9; i++) x[i] = R.rd8(c64 + 8u * i);
      uint64_t live = sync_live64w(x);
#pragma unroll 1
      while (live) {
        const uint64_t c = c64 + (uint32_t)__builtin_ctzll(live);
        live &= live - 1u;
        if (c >= shaped) break;
        const WHdr h = wk_hdr(R.rd8(c));
        if (P.stats) atomicAdd(&P.stats[42], 1ull);
        if (h.k == 0 || h.id > 2u || (h.id != 0 && h.L == 0) || c + h.k + (h.id ? h.L : 1u) > shaped) continue;
        if (P.stats) atomicAdd(&P.stats[43], 1ull);
        if (sync_merges(R, c, shaped)) {
          found = c;
          break;
        }
      }
    }
    const uint32_t fm = grp_ballot(found != ~0ull, lane);
    if (fm) return grp_take(found, lane, (uint32_t)__builtin_ctz(fm));
  }
  return shaped;
}

__global__ __launch_bounds__(256) void walk_sync(DecodeParams P) {
  const uint32_t lane = threadIdx.x & (WAVE - 1u), sub = threadIdx.x & (SY_LANES - 1u);
  const uint64_t r = ((uint64_t)blockIdx.x * 256u + threadIdx.x) / SY_LANES;
  if (r >= P.walk_rp[P.nstreams]) return;  // (whole groups)
  const Region G = region_of(P, r);
  const uint64_t t0 = P.stats ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t t_shape = 0;
  const uint64_t found = sync_entry(P, G, lane, sub, t_shape);
  if (sub) return;
  P.walk_entry[r] = found;
  if (P.stats) {  // (DRP_STATS: cycle sums over the regions of the shaped scan, the rest, the whole sync)
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (found != ~0ull) atomicAdd(&P.stats[31], 1ull);
    if (t_shape) {
      atomicAdd(&P.stats[33], (unsigned long long)(t_shape - t0));
      atomicAdd(&P.stats[34], (unsigned long long)(t1 - t_shape));
    }
    atomicAdd(&P.stats[35], (unsigned long long)(t1 - t0));
  }
}

// The batch's frame density, sampled before the claims form is chosen (drp_launch_spec_head):
// four frames from the exact entries of up to 256 streams spread over the batch
// (P.walk_dense: bytes, frames).
__global__ __launch_bounds__(256) void walk_density(DecodeParams P) {
  const uint64_t ns = P.nstreams, k = threadIdx.x;
  if (k >= ns || k >= 256u) return;
  const uint64_t s = k * ns / umin64(ns, 256u);
  const uint64_t e = P.stream_off[s] + (P.entry ? P.entry[s] : 0ull), se = P.stream_off[s + 1];
  const GReader R{P.bytes, P.nbytes};
  uint64_t p = e;
  uint32_t nf = 0;
#pragma unroll 1
  for (; nf < 4u && p < se; nf++) {
    const WHdr h = wk_hdr(R.rd8(p));
    if (h.k == 0 || h.id > 2u || (h.id != 0 && h.L == 0) || p + h.k + h.L > se) break;
    p += h.k + (h.id ? h.L : 1u);
  }
  if (nf) {
    atomicAdd(&P.walk_dense[0], (unsigned long long)(p - e));
    atomicAdd(&P.walk_dense[1], (unsigned long long)nf);
  }
}

// ---- the walkers -----------------------------------------------------------------------------
// One lane per region, from its entry (walk_sync), frame by frame through the ring. A frame that
// breaks the grammar ends the region's walk ("death": a mispredicted entry, or a protocol error):
// its tile and the rest of the region claim identity, and verification walks them exactly.
template <bool REC>
__global__ __launch_bounds__(WAVE) void claims_walk(DecodeParams P) {
  __shared__ WalkLds S;
  const uint32_t lane = threadIdx.x;
  const uint64_t nreg = P.walk_rp[P.nstreams];
  const uint64_t r = (uint64_t)blockIdx.x * WAVE + lane;
  if ((uint64_t)blockIdx.x * WAVE >= nreg || walk_hops(P)) return;  // (whole wave)
  // ---- this lane's region ---------------------------------------------------------------------
  uint64_t t0 = 0, A0 = 0, se = 0, pos = ~0ull;
  uint64_t rbase = 0;  // this region's first record slot (P.rec_cap slots per region)
  uint32_t nw = 0;
  if (r < nreg) {
    const Region G = region_of(P, r);
    t0 = G.t0;
    A0 = G.A0;
    se = G.se;
    nw = G.nw;
    rbase = r * P.rec_cap;
    pos = P.walk_entry[r];
  }
  uint32_t mode = pos != ~0ull ? WM_WALK : WM_DONE;
  bool rs = true;  // the next frame noted restarts the records' chain
  // ---- DMA addressing: instruction i stages regions 8 i .. 8 i + 7 (16 bytes per lane) ---------
  uint64_t dA[WK_NDMA];
#pragma unroll
  for (uint32_t i = 0; i < WK_NDMA; i++) {
    const int src = (int)(i * (WAVE / WK_LPR) + lane / WK_LPR);
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)A0, src, WAVE), hi = (uint32_t)__shfl((int)(uint32_t)(A0 >> 32), src, WAVE);
    dA[i] = (((uint64_t)hi << 32) | lo) + (lane % WK_LPR) * 16u;
  }
  uint32_t nwmax = nw;
#pragma unroll
  for (uint32_t d = 1; d < WAVE; d <<= 1) nwmax = max(nwmax, (uint32_t)__shfl_xor((int)nwmax, d, WAVE));
  nwmax = __builtin_amdgcn_readfirstlane(nwmax);
  // (the LDS-DMA is issued from inline asm: the compiler would otherwise put a vmcnt(0) wait in
  // front of every LDS read, since it cannot tell which slot a pending DMA writes; the one wait
  // the ring needs is the counted one below)
  const uint32_t ring0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)S.ring;
  // The regions' windows w into the ring slot w % WK_SLOTS; returns the DMA instructions issued.
  // Only the windows a walk may read are staged: from the one holding the region's next frame
  // start on (a region whose frames are long skips the windows inside them; a finished one all).
  // When every region needs it (dense streams: nearly every step), one unmasked form.
  const uint64_t act = __ballot(nw != 0);
  auto issue = [&](uint32_t w) -> uint32_t {
    const uint32_t slot = w % WK_SLOTS;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the slot's last reads, a step ago, are done)
    const uint64_t need = __ballot(w <= nw && mode == WM_WALK && pos < A0 + (uint64_t)(w + 1u) * WK_WB);
    if (need == act) {  // (inactive lanes load bytes of the batch's first lines, unread)
#pragma unroll
      for (uint32_t i = 0; i < WK_NDMA; i++) {
        const uint8_t *g = P.bytes + dA[i] + (uint64_t)w * WK_WB;
        const uint32_t l = __builtin_amdgcn_readfirstlane(ring0 + slot * WK_SLOT + i * 1024u);
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
      }
      return WK_NDMA;
    }
    uint32_t n = 0;
#pragma unroll
    for (uint32_t i = 0; i < WK_NDMA; i++) {
      constexpr uint32_t RPI = WAVE / WK_LPR;  // regions per DMA instruction
      const uint32_t sub = (uint32_t)(need >> (i * RPI)) & (uint32_t)((1ull << RPI) - 1u);
      if (sub) {
        n++;
        if ((sub >> (lane / WK_LPR)) & 1u) {
          const uint8_t *g = P.bytes + dA[i] + (uint64_t)w * WK_WB;
          const uint32_t l = __builtin_amdgcn_readfirstlane(ring0 + slot * WK_SLOT + i * 1024u);
          asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
        }
      }
    }
    return n;
  };
  uint32_t d_pre = 0;
#pragma unroll
  for (uint32_t w = 0; w < WK_AHEAD; w++) d_pre = issue(w);
  // segment records of the current 4-window group (8 segments: byte j = segment j)
  uint64_t ent = ~0ull, fn = 0, fc = 0;
  bool had = false;   // a chain frame started in the current tile
  bool dead = false;  // the chain died in the current tile
  uint64_t term = 0;  // MARK_TERM | p: the tail that ended the chain in the current tile
  // records (P.rec): the next slot of the region, the current tile's first one, and whether every
  // frame of the tile so far has one
  uint32_t rnext = 0, rtile = 0;
  bool rok = REC && mode == WM_WALK;
  // vector-memory operations issued after the DMA of window w + 1 (loads, stores and DMAs count
  // together, in issue order): the stores of the steps since and the DMAs issued since (lower
  // bounds, so the wait below is never short)
  uint32_t st2 = 0, st1 = 0, d1 = d_pre;
#pragma unroll 1
  for (uint32_t w = 0; w < nwmax; w++) {
    const uint32_t d0 = issue(w + WK_AHEAD);
    wk_wait_vm(WK_AHEAD == 3 ? st2 + d1 + st1 + d0 : st1 + d0);  // windows w and w + 1 have landed
    const uint32_t q = w % WK_WPT;  // window of the tile (the same for every lane)
    uint32_t nrec = 0;              // records this lane stored in this step
    if (w < nw) {
      const uint64_t W0 = A0 + (uint64_t)w * WK_WB, W1 = W0 + WK_WB;
      const uint64_t T0 = A0 + (uint64_t)(w - q) * WK_WB;  // the tile's first byte
      const WkReader R{S, P.bytes, W0, P.nbytes, w};
      // a frame start p (in window w, so in the current group) into the segment records
      auto note = [&](uint64_t p, uint32_t id, bool deliver) {
        const uint32_t rp = (uint32_t)(p - T0), sh = 8u * ((rp >> 6) & 7u);
        const uint64_t e = (uint64_t)((rp & 63u) | (rs ? 0x40u : 0u)) << sh;
        const uint64_t m = ((ent >> sh) & 0xFFull) == 0xFFull ? 0xFFull << sh : 0ull;  // (the segment's first)
        ent = (ent & ~m) | (e & m);
        rs = false;
        had = true;
        fn += (uint64_t)(deliver ? 1u : 0u) << sh;
        fc += (uint64_t)(deliver && id == 1u ? 1u : 0u) << sh;
      };
      // this frame's record
      auto record = [&](uint32_t k, uint64_t L, uint32_t id, bool tail) {
        uint4 a = make_uint4((uint32_t)(pos + k + 1u - T0) | (id << 14) | ((tail ? 1u : 0u) << 16),
                             (uint32_t)umin64(L - 1u, 0xFFFFFFFFull), 0u, 0u),
              b = make_uint4(0u, 0u, 0u, 0u);
        rok = rnext < P.rec_cap && (id != 1u || wk_record(R, pos + k + 1u, L - 1u, a, b));
        if (rok) {
          uint4 *d = reinterpret_cast<uint4 *>(P.rec + (rbase + rnext) * 8u);
          d[0] = a;
          d[1] = b;
          rnext++;
          nrec++;
        }
      };
      // The straight path: complete Change and blob frames (nearly every frame). A lane stops it
      // at any other frame (a long varint, a header-only frame, a tail, a death), which the
      // general step below takes, one frame, before the straight path resumes.
#pragma unroll 1
      while (__ballot(mode == WM_WALK && pos < W1)) {
        bool go = mode == WM_WALK && pos < W1;
#pragma unroll 1
        while (go) {
          const WHdr h = wk_hdr(wk_rd8(S, w, (uint32_t)(pos - W0)));
          const bool plain = (h.k != 0u) & (h.id - 1u < 2u) & (h.L != 0u) & (h.L <= se - pos - h.k);
          if (plain) {
            note(pos, h.id, true);
            if (REC && rok) record(h.k, h.L, h.id, false);
            pos += h.k + h.L;
          }
          go = plain & (pos < W1);
        }
        if (mode != WM_WALK || pos >= W1) continue;
        // the general step: one frame
        const uint32_t o = (uint32_t)(pos - W0);
        const WHdr h = wk_hdr(wk_rd8(S, w, o));
        uint64_t L = h.L;
        uint32_t k = h.k, id = h.id;
        if (k == 0) {  // a length varint of 6..10 bytes: the exact grammar
          const Hdr e = hdr_global(P.bytes, pos, se);
          if (e.kind == H_VALID || e.kind == H_TAIL_CHANGE || e.kind == H_TAIL_BLOB) {
            k = e.vlen;
            L = e.L;
            id = e.id;
          } else {
            id = 0xFF;  // (an error or a cut header: the chain ends)
          }
        }
        if (id > 2u || (id != 0u && L == 0)) {  // the chain dies
          dead = true;
          mode = WM_DONE;
          if (P.stats) {  // (DRP_STATS: deaths; the first one's bytes from LDS and from HBM)
            if (atomicAdd(&P.stats[32], 1ull) == 0) {
              P.stats[36] = pos;
              P.stats[37] = wk_rd8(S, w, o);
              P.stats[38] = g_rd8(P.bytes, pos);
              P.stats[39] = ((uint64_t)w << 32) | (lane << 16) | o;
            }
          }
        } else if (id == 0u) {
          note(pos, 0u, false);
          pos += k + 1u;
        } else {
          const bool tail = L > se - pos - k;  // the stream ends inside this frame
          note(pos, id, !tail || id == 2u);    // (a cut Change is carried, a cut blob delivered)
          if (REC && rok && (!tail || id == 2u)) record(k, L, id, tail);
          if (tail) {
            term = MARK_TERM | pos;
            mode = WM_DONE;
          } else {
            pos += k + L;
          }
        }
      }
      if (q % WK_GW == WK_GW - 1) {  // flush the group's 8 segment records
        const uint64_t ix = (t0 + w / WK_WPT) * NT + (q / WK_GW) * 8u;
        *reinterpret_cast<uint64_t *>(P.ent + ix) = ent;
        *reinterpret_cast<uint64_t *>(P.ent_n + ix) = fn;
        *reinterpret_cast<uint64_t *>(P.ent_c + ix) = fc;
        ent = ~0ull;
        fn = 0;
        fc = 0;
      }
      if (q == WK_WPT - 1) {  // the tile's claim
        // (a dead tile's records mix two chains, which no record marks: identity, so verification
        // re-walks it from its exact entry; the rest of the region is not walked)
        uint64_t cl = C_ID;
        if (term) cl = term;
        else if (mode == WM_WALK && had) cl = pos;
        if (dead) cl = C_ID;
        P.claim[t0 + w / WK_WPT] = cl;
        if (REC) {  // its first record (or none: the tile takes the wire-reading emission)
          P.tile_rec[t0 + w / WK_WPT] = rok && !dead ? (uint32_t)(rbase + rtile) : REC_NONE;
          rtile = rnext;
          rok = rnext < P.rec_cap && !dead && mode == WM_WALK;
        }
        had = false;
        term = 0;
        dead = false;
      }
    }
    // this step's stores (at least one lane is active: the one with nwmax windows)
    uint32_t st = (q % WK_GW == WK_GW - 1 ? 3u : 0u) + (q == WK_WPT - 1 ? (REC ? 2u : 1u) : 0u);
    if (REC) {
#pragma unroll
      for (uint32_t d = 1; d < WAVE; d <<= 1) nrec = max(nrec, (uint32_t)__shfl_xor((int)nrec, d, WAVE));
      st += 2u * __builtin_amdgcn_readfirstlane(nrec);
    }
    st2 = st1;
    st1 = st;
    d1 = d0;
  }
}

// ---- the hop walkers --------------------------------------------------------------------------
// One lane per region, from its entry (walk_sync), frame to frame with a direct read of each
// header (two 8-byte loads through the caches; nothing staged): a frame costs one dependent load
// and ~60 instructions, and a frame of any length costs the same (C5's 4 KB values are never
// read). Enough regions (lanes) keep enough loads in flight for the stream to be read at the HBM
// rate (a 128-byte line holds ~1.5 C2 headers: the wire is read about once). Outputs as
// claims_walk: per tile its claim, per 64-byte segment its record (flushed 8 segments at a
// time), the same death and tail rules.
__global__ __launch_bounds__(256) void claims_hop(DecodeParams P) {
  const uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (r >= P.walk_rp[P.nstreams] || !walk_hops(P)) return;
  const Region G = region_of(P, r);
  const uint64_t A0 = G.A0, se = G.se;
  const uint32_t ntr = G.nw / WK_WPT;       // tiles
  const uint64_t end = A0 + (uint64_t)ntr * TILE;
  uint64_t pos = P.walk_entry[r];
  uint32_t mode = pos != ~0ull ? WM_WALK : WM_DONE;
  bool rs = true;     // the next frame noted restarts the records' chain
  bool had = false;   // a chain frame started in the current tile
  bool dead = false;  // the chain died in the current tile
  uint64_t term = 0;  // MARK_TERM | p: the tail that ended the chain in the current tile
  uint64_t ent = ~0ull, fn = 0, fc = 0;  // records of the current group of 8 segments (512 bytes)
  uint32_t gcur = 0, tcur = 0;           // current group and tile of the region
  // groups [gcur, gto) to memory (the registers, then empty groups)
  // (the records were preset to "no frame starts here" (drp_launch_claims_walk): only groups
  // where a frame starts are written, one or two per frame however long it is)
  auto flush_to = [&](uint32_t gto) {
    if (gcur < gto && (ent != ~0ull || fn || fc)) {
      const uint64_t ix = (G.t0 + gcur / 16u) * NT + (gcur % 16u) * 8u;
      *reinterpret_cast<uint64_t *>(P.ent + ix) = ent;
      *reinterpret_cast<uint64_t *>(P.ent_n + ix) = fn;
      *reinterpret_cast<uint64_t *>(P.ent_c + ix) = fc;
      ent = ~0ull;
      fn = 0;
      fc = 0;
    }
    if (gcur < gto) gcur = gto;
  };
  // tiles [tcur, tto) end before pos: their claims (a dead tile's records mix two chains: identity,
  // so verification re-walks it from its exact entry; the region is not walked further)
  auto close_to = [&](uint32_t tto) {
#pragma unroll 1
    for (; tcur < tto; tcur++) {
      uint64_t cl = C_ID;
      if (term) cl = term;
      else if (mode == WM_WALK && had) cl = pos;
      if (dead) cl = C_ID;
      P.claim[G.t0 + tcur] = cl;
      had = false;
      term = 0;
      dead = false;
    }
  };
  auto note = [&](uint32_t rel, uint32_t id, bool deliver) {
    const uint32_t sh = 8u * ((rel >> 6) & 7u);
    const uint64_t e = (uint64_t)((rel & 63u) | (rs ? 0x40u : 0u)) << sh;
    const uint64_t m = ((ent >> sh) & 0xFFull) == 0xFFull ? 0xFFull << sh : 0ull;  // (the segment's first)
    ent = (ent & ~m) | (e & m);
    rs = false;
    had = true;
    fn += (uint64_t)(deliver ? 1u : 0u) << sh;
    fc += (uint64_t)(deliver && id == 1u ? 1u : 0u) << sh;
  };
#pragma unroll 1
  while (mode == WM_WALK && pos < end) {
    const uint64_t x = g_rd8x(P.bytes, pos);
    const uint32_t rel = (uint32_t)(pos - A0);
    if (rel / TILE > tcur) close_to(rel / TILE);
    if (rel / 512u > gcur) flush_to(rel / 512u);
    const WHdr h = wk_hdr(x);
    if ((h.k != 0u) & (h.id - 1u < 2u) & (h.L != 0u) & (h.L <= se - pos - h.k)) {  // (nearly every frame)
      note(rel % TILE, h.id, true);
      pos += h.k + h.L;
      continue;
    }
    uint64_t L = h.L;
    uint32_t k = h.k, id = h.id;
    if (k == 0) {  // a length varint of 6..10 bytes: the exact grammar
      const Hdr e = hdr_global(P.bytes, pos, se);
      if (e.kind == H_VALID || e.kind == H_TAIL_CHANGE || e.kind == H_TAIL_BLOB) {
        k = e.vlen;
        L = e.L;
        id = e.id;
      } else {
        id = 0xFF;  // (an error or a cut header: the chain ends)
      }
    }
    if (id > 2u || (id != 0u && L == 0)) {  // the chain dies
      dead = true;
      mode = WM_DONE;
      if (P.stats) atomicAdd(&P.stats[32], 1ull);
    } else if (id == 0u) {
      note(rel % TILE, 0u, false);
      pos += k + 1u;
    } else {
      const bool tail = L > se - pos - k;  // the stream ends inside this frame
      note(rel % TILE, id, !tail || id == 2u);  // (a cut Change is carried, a cut blob delivered)
      if (tail) {
        term = MARK_TERM | pos;
        mode = WM_DONE;
      } else {
        pos += k + L;
      }
    }
  }
  flush_to(ntr * 16u);
  close_to(ntr);
}

// ---- record emission ---------------------------------------------------------------------------
// The tiles verification lets it take (tile_recok: every frame of the tile has a record and its
// first record is the frame at e_t): rows [tile_base, + tile_count) from the tile's records, a wave
// per tile, in XCD-contiguous order (neighbouring tiles' column lines meet in one L2). Reads
// 32 bytes per row and writes the columns; the wire is not read again.
constexpr uint32_t ER_WAVES = 4;
__global__ __launch_bounds__(ER_WAVES * WAVE) void emit_rec(DecodeParams P) {
  if (*P.overflow & (F_MISS | F_WAIT)) return;  // (a failed prediction: emitted after its repair)
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  uint64_t g;
  {
    const uint32_t n = gridDim.x, q = n / 8u, r = n % 8u, x = blockIdx.x % 8u;
    g = (uint64_t)x * q + min(x, r) + blockIdx.x / 8u;
  }
  const uint64_t t = g * ER_WAVES + wid;
  if (t >= P.tile_prefix[P.nstreams] || !P.tile_recok[t]) return;  // (whole wave)
  const uint64_t base = P.tile_base[t], n = P.tile_count[t];
  const uint64_t r0 = P.tile_rec[t];
  const uint64_t A = tile_geo(P, t).A;
#pragma unroll 1
  for (uint64_t i = lane; i < n; i += WAVE) {
    const uint64_t f = base + i;
    if (f >= P.cap) break;
    const uint4 *src = reinterpret_cast<const uint4 *>(P.rec + (r0 + i) * 8u);
    const uint4 a = src[0], b = src[1];
    const uint32_t id = (a.x >> 14) & 3u, fl = (a.x >> 17) & 3u;
    P.payload_off[f] = A + (a.x & 0x3FFFu);
    P.payload_len[f] = a.y;
    P.type[f] = (uint8_t)(id | (((a.x >> 16) & 1u) ? DRP_FRAME_PARTIAL : 0u));
    if (id != 1u) continue;
    P.key_off[f] = a.z & 0xFFu;
    P.subset_off[f] = (a.z >> 8) & 0xFFu;
    P.key_len[f] = a.z >> 16;
    P.value_off[f] = a.w & 0xFFFFu;
    P.subset_len[f] = a.w >> 16;
    P.value_len[f] = (fl & DRP_F_VALUE) ? a.y - (a.w & 0xFFFFu) : 0u;
    P.change[f] = b.x | ((uint64_t)(b.w & 0x3FFu) << 32);
    P.from[f] = b.y | ((uint64_t)((b.w >> 10) & 0x3FFu) << 32);
    P.to[f] = b.z | ((uint64_t)((b.w >> 20) & 0x3FFu) << 32);
    P.flags[f] = (uint8_t)fl;
  }
}

}  // namespace spec
}  // namespace drp

using namespace drp;

extern "C" hipError_t drp_launch_emit_rec(const DecodeParams *P, uint64_t nt_max, hipStream_t st) {
  if (nt_max == 0 || !P->rec) return hipSuccess;
  hipLaunchKernelGGL(spec::emit_rec, dim3((uint32_t)((nt_max + spec::ER_WAVES - 1) / spec::ER_WAVES)),
                     dim3(spec::ER_WAVES * WAVE), 0, st, *P);
  return hipGetLastError();
}

// record slots per region (P->rec_cap) for tpr tiles per region
extern "C" uint64_t drp_walk_rec_cap(uint32_t tpr) { return (uint64_t)tpr * spec::TILE / spec::WK_REC_BYTES; }

// Region walkers in place of claims_fast: the region list (and the edge tiles onto P->work), then
// the walkers. P->walk_rp: nstreams + 1 words; P->walk_tpr: tiles per region.
extern "C" hipError_t drp_launch_claims_walk(const DecodeParams *P, uint64_t nt_max, hipStream_t st) {
  if (nt_max == 0) return hipSuccess;
  hipLaunchKernelGGL(spec::walk_regions, dim3(1), dim3(1024), 0, st, *P);
  const uint64_t maxr = nt_max / P->walk_tpr + P->nstreams + 1;
  hipLaunchKernelGGL(spec::walk_sync, dim3((uint32_t)((maxr * spec::SY_LANES + 255) / 256)), dim3(256), 0, st, *P);
  if (P->walk_hop) {
    const size_t nrec = (size_t)nt_max * spec::NT;  // (one record byte per 64-byte segment)
    hipError_t e = hipMemsetAsync(P->ent, 0xFF, nrec, st);
    if (e == hipSuccess) e = hipMemsetAsync(P->ent_n, 0, nrec, st);
    if (e == hipSuccess) e = hipMemsetAsync(P->ent_c, 0, nrec, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(spec::claims_hop, dim3((uint32_t)((maxr + 255) / 256)), dim3(256), 0, st, *P);
  }
  if (P->walk_hop) return hipGetLastError();  // (2: dense batches take claims_fast, launched by the caller)
  hipLaunchKernelGGL(spec::claims_walk<false>, dim3((uint32_t)((maxr + WAVE - 1) / WAVE)), dim3(WAVE), 0, st, *P);
  return hipGetLastError();
}

extern "C" hipError_t drp_launch_walk_density(const DecodeParams *P, hipStream_t st) {
  hipLaunchKernelGGL(spec::walk_density, dim3(1), dim3(256), 0, st, *P);
  return hipGetLastError();
}

extern "C" uint32_t drp_walk_tiles_per_region(uint64_t nt_max, int hop) {
  const uint64_t nr = hop == 1 ? spec::HOP_REGIONS : spec::WK_REGIONS;  // (2: either form, by density)
  const uint64_t t = (nt_max + nr - 1) / nr;
  return (uint32_t)(t ? t : 1);
}
