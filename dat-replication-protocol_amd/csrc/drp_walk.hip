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
// parsed and linked (~800 VALU instructions per 4 KiB wave, VALU-issue-bound). For sparse streams
// (frames of more than HOP_FRAME bytes on average, decided per launch from walk_density's sample)
// one LANE instead walks one REGION of consecutive interior tiles of a stream frame by frame, as
// decode.js does: the entry of a region's first tile is found once (walk_sync: the first position
// whose Change payload parses exactly in the schema's shape, or whose chain survives WK_K
// frames), and every later frame start follows from its predecessor's header, one 16-byte load
// per frame (claims_hop): a 4 KB value is never read by the claims. The kernel writes the records
// of the 64-byte segments where a frame starts and one claim per tile.
//
// Regions never cross a stream and hold only interior tiles (A >= stream start, A + IMG <= stream
// end); the edge tiles go to spec_claims' work list, as claims_fast sends them.
#include "drp_spec.h"

namespace drp {
namespace spec {

constexpr uint32_t SY_NEAR = 256;                // a "near" sync chain's longest frame
constexpr uint64_t SY_TAIL = 16384;              // a sync chain's tail counts this close to the stream end
#ifndef DRP_SY_MERGE
#define DRP_SY_MERGE 1024
#endif
constexpr uint64_t SY_MERGE = DRP_SY_MERGE;              // a region's entry before its first shaped Change: this close
constexpr uint64_t SY_SHAPE = 8192;              // how far a region's first shaped Change is looked for
constexpr uint64_t SY_GENERAL = 2048;            // how far the general scan looks (else: no entry, the
                                                 // region's tiles claim identity and verification walks them)
#ifndef DRP_WK_REGIONS
#define DRP_WK_REGIONS 65536
#endif
constexpr uint32_t WK_K = 8;                     // frames a sync chain must survive (no Change shape)
constexpr uint32_t WK_REGIONS = DRP_WK_REGIONS;  // regions aimed at (one per resident lane)
#ifndef DRP_HOP_REGIONS
#define DRP_HOP_REGIONS 24576
#endif
constexpr uint32_t HOP_REGIONS = DRP_HOP_REGIONS;  // hop walkers: regions aimed at

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

// Region r of the batch: its first tile (t0, at A0), its stream end, its windows, and for a
// stream's first tile the exact entry.
struct Region {
  uint64_t t0, A0, se, entry;
  uint32_t nt;  // interior tiles of the region
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
  G.nt = (uint32_t)umin64(P.walk_tpr, I.i_lo + I.n - i0);
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
  const uint64_t se = G.se, end = G.A0 + (uint64_t)G.nt * TILE;
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
  const uint32_t ntr = G.nt;       // tiles
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

}  // namespace spec
}  // namespace drp

using namespace drp;

// Hop walkers in place of claims_fast: the region list (and the edge tiles onto P->work), the region
// syncs, then the walkers. P->walk_rp: nstreams + 1 words; P->walk_tpr: tiles per region.
extern "C" hipError_t drp_launch_claims_walk(const DecodeParams *P, uint64_t nt_max, hipStream_t st) {
  if (nt_max == 0) return hipSuccess;
  hipLaunchKernelGGL(spec::walk_regions, dim3(1), dim3(1024), 0, st, *P);
  const uint64_t maxr = nt_max / P->walk_tpr + P->nstreams + 1;
  hipLaunchKernelGGL(spec::walk_sync, dim3((uint32_t)((maxr * spec::SY_LANES + 255) / 256)), dim3(256), 0, st, *P);
  const size_t nrec = (size_t)nt_max * spec::NT;  // (one record byte per 64-byte segment)
  hipError_t e = hipMemsetAsync(P->ent, 0xFF, nrec, st);
  if (e == hipSuccess) {  // (ent_c follows ent_n in the scratch: one fill for both)
    if (P->ent_c == P->ent_n + nrec) {
      e = hipMemsetAsync(P->ent_n, 0, 2 * nrec, st);
    } else {
      e = hipMemsetAsync(P->ent_n, 0, nrec, st);
      if (e == hipSuccess) e = hipMemsetAsync(P->ent_c, 0, nrec, st);
    }
  }
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(spec::claims_hop, dim3((uint32_t)((maxr + 255) / 256)), dim3(256), 0, st, *P);
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
