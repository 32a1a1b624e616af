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

constexpr uint32_t WK_WB = 128;                  // window bytes per region and step
constexpr uint32_t WK_WPT = TILE / WK_WB;        // windows per tile (64)
constexpr uint32_t WK_SLOTS = 4;                 // LDS ring slots
constexpr uint32_t WK_AHEAD = 3;                 // windows staged ahead of the one walked
constexpr uint32_t WK_SLOT = WAVE * WK_WB;       // bytes per slot (8 KiB)
constexpr uint32_t WK_NDMA = WK_SLOT / (WAVE * 16);  // DMA instructions per step (8)
constexpr uint32_t WK_K = 8;                     // frames a sync chain must survive (no Change shape)
constexpr uint32_t WK_REGIONS = 65536;           // regions aimed at (one per resident lane)
static_assert(WK_WPT % 4 == 0, "records are flushed every 4 windows (8 segments)");
static_assert(WK_SLOTS >= WK_AHEAD + 1, "the ring holds the walked window, the next and the in-flight ones");

enum : uint32_t { WM_SYNC = 0, WM_WALK = 1, WM_DONE = 2 };

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
  const uint32_t slot = (w + (o >> 7)) % WK_SLOTS;
  return S.ring[(slot * WK_SLOT + threadIdx.x * WK_WB + (o & (WK_WB - 1))) >> 2];
}

// the 8 bytes at window-relative offset o (o + 8 <= 2 * WK_WB + 4: the ring's two windows plus
// one dword), little endian
__device__ __forceinline__ uint64_t wk_rd8(const WalkLds &S, uint32_t w, uint32_t o) {
  const uint32_t d = o & ~3u, sh = (o & 3u) * 8u;
  const uint32_t a = wk_rd(S, w, d), b = wk_rd(S, w, d + 4), c = (o & 3u) ? wk_rd(S, w, d + 8) : 0u;
  const uint32_t lo = __builtin_amdgcn_alignbit(b, a, sh), hi = __builtin_amdgcn_alignbit(c, b, sh);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// 8 bytes at absolute position p from the batch (two aligned 8-byte loads; p + 16 <= nbytes)
__device__ __forceinline__ uint64_t g_rd8(const uint8_t *g, uint64_t p) {
  const uint64_t *q = reinterpret_cast<const uint64_t *>(g + (p & ~7ull));
  const uint32_t sh = (uint32_t)(p & 7u) * 8u;
  const uint64_t a = q[0];
  if (!sh) return a;
  return (a >> sh) | (q[1] << (64 - sh));
}

// A frame header from its first 8 bytes x: the length varint of 1..5 bytes, then the id.
// k = 0: a longer varint (L >= 2^35: the slow path decides).
struct WHdr {
  uint64_t L;
  uint32_t k, id;
};
__device__ __forceinline__ WHdr wk_hdr(uint64_t x) {
  WHdr h;
  const uint64_t tm = ~x & 0x8080808080ull;
  if (!tm) {
    h.k = 0;
    h.L = 0;
    h.id = 0xFF;
    return h;
  }
  h.k = ((uint32_t)__builtin_ctzll(tm) >> 3) + 1u;
  const uint64_t v = (x & 0x7Full) | ((x >> 1) & 0x3F80ull) | ((x >> 2) & 0x1FC000ull) | ((x >> 3) & 0xFE00000ull) |
                     ((x >> 4) & 0x7F0000000ull);
  h.L = v & ((1ull << (7u * h.k)) - 1ull);
  h.id = (uint32_t)(x >> (8u * h.k)) & 0xFFu;
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

// Sync check of a Change candidate: its payload [po, po + pl) parses in the schema's own shape
// (one-byte tags with their wire types, in protocol-buffers' field order: [subset] key change
// from to [value], varint numbers of <= 10 bytes, lengths inside the payload) and its last field
// ends exactly at the payload end. 1: strong; 0: not a Change of that shape. Prediction only.
__device__ __forceinline__ uint32_t wk_change_shape(const WkReader &R, uint64_t po, uint64_t pl) {
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

// Does the chain from candidate c survive? A header is valid when its id is <= 2 (and a Change or
// blob declares a length); a Change frame must start with a Change tag. Steps past the two ring
// windows read the batch. 1: survives WK_K frames, or ends at the stream end (exactly, or in a
// tail) after at least two complete frames (a shadow header whose varint swallows a real one's
// length byte declares a frame of ~1 MB+, which a short batch cuts: no evidence alone).
__device__ __forceinline__ bool wk_survives(const WkReader &R, uint64_t c, uint64_t se) {
  uint64_t p = c;
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
    if (h.L > se - p - h.k) return f >= 2u;  // a tail: the chain ends at the stream end
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

__global__ __launch_bounds__(WAVE) void claims_walk(DecodeParams P) {
  __shared__ WalkLds S;
  const uint32_t lane = threadIdx.x;
  const uint64_t nreg = P.walk_rp[P.nstreams];
  const uint64_t r = (uint64_t)blockIdx.x * WAVE + lane;
  if ((uint64_t)blockIdx.x * WAVE >= nreg) return;  // (whole wave)
  // ---- this lane's region ---------------------------------------------------------------------
  uint64_t t0 = 0, A0 = 0, se = 0, pos = 0;
  uint32_t nw = 0, mode = WM_DONE;
  bool rs = false;
  if (r < nreg) {
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
    const uint64_t j = r - P.walk_rp[s];
    const uint64_t i0 = I.i_lo + j * P.walk_tpr;
    const uint64_t ntr = umin64(P.walk_tpr, I.i_lo + I.n - i0);
    t0 = P.tile_prefix[s] + i0;
    A0 = I.base + i0 * TILE;
    se = I.se;
    nw = (uint32_t)ntr * WK_WPT;
    mode = WM_SYNC;
    if (A0 == I.so) {  // the stream's first tile: its entry is exact
      mode = WM_WALK;
      pos = I.so + (P.entry ? P.entry[s] : 0ull);
      rs = true;
    }
  }
  // ---- DMA addressing: instruction i stages regions 8 i .. 8 i + 7 (16 bytes per lane) ---------
  uint64_t dA[WK_NDMA];
  uint32_t dN[WK_NDMA];
#pragma unroll
  for (uint32_t i = 0; i < WK_NDMA; i++) {
    const int src = (int)(i * 8u + (lane >> 3));
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)A0, src, WAVE), hi = (uint32_t)__shfl((int)(uint32_t)(A0 >> 32), src, WAVE);
    dA[i] = (((uint64_t)hi << 32) | lo) + (lane & 7u) * 16u;
    dN[i] = (uint32_t)__shfl((int)nw, src, WAVE);  // windows 0 .. nw (the last: the halo's first bytes)
  }
  uint32_t nwmax = nw;
#pragma unroll
  for (uint32_t d = 1; d < WAVE; d <<= 1) nwmax = max(nwmax, (uint32_t)__shfl_xor((int)nwmax, d, WAVE));
  // (the LDS-DMA is issued from inline asm: the compiler would otherwise put a vmcnt(0) wait in
  // front of every LDS read, since it cannot tell which slot a pending DMA writes; the one wait
  // the ring needs is the counted one below)
  const uint32_t ring0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)S.ring;
  auto issue = [&](uint32_t w) {
    const uint32_t slot = w % WK_SLOTS;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the slot's last reads, a step ago, are done)
#pragma unroll
    for (uint32_t i = 0; i < WK_NDMA; i++)
      if (dN[i] && w <= dN[i]) {
        const uint8_t *g = P.bytes + dA[i] + (uint64_t)w * WK_WB;
        const uint32_t l = __builtin_amdgcn_readfirstlane(ring0 + slot * WK_SLOT + i * 1024u);
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
      }
  };
#pragma unroll
  for (uint32_t w = 0; w < WK_AHEAD; w++) issue(w);
  // records of the current 4-window group (8 segments: byte j = segment j)
  uint64_t ent = ~0ull, fn = 0, fc = 0;
  bool had = false;        // a chain frame started in the current tile
  uint64_t term = 0;       // MARK_TERM | p: the tail that ended the chain in the current tile
  uint32_t from = 0;       // SYNC: the first window-relative offset to scan
  // SYNC: a strong "far" candidate of this tile (its first frame leaves the ring) held back while
  // the scan looks for a strong near one: position, successor, id (0: none)
  uint64_t far_c = 0, far_n = 0;
  uint32_t far_id = 0;
#pragma unroll 1
  for (uint32_t w = 0; w < nwmax; w++) {
    issue(w + WK_AHEAD);
    // windows w and w + 1 have landed (only the two youngest steps' DMAs may be in flight)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((WK_AHEAD - 1) * WK_NDMA) : "memory");
    if (w >= nw) continue;
    const uint32_t q = w % WK_WPT;  // window of the tile
    const uint64_t W0 = A0 + (uint64_t)w * WK_WB, W1 = W0 + WK_WB;
    const uint64_t T0 = A0 + (uint64_t)(w - q) * WK_WB;  // the tile's first byte
    const uint64_t tcur = t0 + w / WK_WPT;
    const WkReader R{S, P.bytes, W0, P.nbytes, w};
    // a frame start p of the current tile (id, delivered) into the segment records: the current
    // 4-window group's registers, or memory for a group already flushed (a far candidate taken late)
    auto note = [&](uint64_t p, uint32_t id, bool deliver) {
      const uint32_t seg = (uint32_t)(p - T0) >> 6, e = ((uint32_t)(p - T0) & 63u) | (rs ? 0x40u : 0u);
      rs = false;
      had = true;
      if ((seg >> 3) != (q >> 2)) {
        const uint64_t ix = tcur * NT + seg;
        P.ent[ix] = (uint8_t)e;
        P.ent_n[ix] = deliver ? 1u : 0u;
        P.ent_c[ix] = deliver && id == 1u ? 1u : 0u;
        return;
      }
      const uint32_t sh = 8u * (seg & 7u);
      if (((ent >> sh) & 0xFFull) == 0xFFull) ent = (ent & ~(0xFFull << sh)) | ((uint64_t)e << sh);
      fn += (uint64_t)(deliver ? 1u : 0u) << sh;
      fc += (uint64_t)(deliver && id == 1u ? 1u : 0u) << sh;
    };
    // the held-back far candidate becomes the chain (its frame noted where it starts)
    auto take_far = [&]() {
      rs = true;
      note(far_c, far_id, far_id != 0u);
      pos = far_n;
      mode = WM_WALK;
      far_c = 0;
      if (P.stats) atomicAdd(&P.stats[31], 1ull);
    };
#pragma unroll 1
    for (uint32_t guard = 0; guard < 2 * WK_WB; guard++) {  // (a death re-enters the scan)
      if (mode == WM_SYNC && far_c && far_n < W1) take_far();  // (no near candidate up to its successor)
      if (mode == WM_SYNC) {
        // Candidates from `from` on, through this window and the next one's first 112 bytes (both
        // are in the ring), in order. A complete Change whose payload has the schema's shape and
        // whose next header is valid is taken at once (random bytes essentially never pass). Any
        // other candidate must survive WK_K frames; it is taken at once when its first frame stays
        // in the ring ("near"), else ("far") held back while the scan goes on, up to its successor
        // or the tile's end, and dropped for any candidate taken at once: a header whose length
        // varint swallows a real header's first bytes declares a frame of ~1 MB that lands on the
        // real chain with odds of one in the real frame size (C2: 1/86), and then "survives".
#pragma unroll 1
        for (uint32_t c16 = from & ~15u; c16 < WK_WB + 112u; c16 += 16u) {
          uint32_t live = wk_live16(wk_rd(S, w, c16), wk_rd(S, w, c16 + 4), wk_rd(S, w, c16 + 8), wk_rd(S, w, c16 + 12),
                                    wk_rd(S, w, c16 + 16));
          if (c16 < from) live &= ~0u << (from - c16);
#pragma unroll 1
          while (live) {
            const uint32_t o = c16 + (uint32_t)__builtin_ctz(live);
            live &= live - 1u;
            const uint64_t c = W0 + o;
            if (far_c && c >= far_n) break;  // (the held-back chain's successor: it wins from there)
            const WHdr h = wk_hdr(wk_rd8(S, w, o));
            if (h.k == 0 || h.id > 2u || (h.id != 0 && h.L == 0)) continue;
            bool shape = false;
            if (h.id == 1u && h.L > 1 && h.L - 1 <= se - c - h.k - 1) {  // a complete Change: its shape
              shape = wk_change_shape(R, c + h.k + 1u, h.L - 1u) != 0;
              const uint64_t n = c + h.k + h.L;
              if (shape && n < se) {
                const WHdr g = wk_hdr(R.rd8(n));
                shape = g.k != 0 && g.id <= 2u && (g.id == 0 || g.L != 0);
              }
            }
            if (!shape && !wk_survives(R, c, se)) continue;
            if (shape || h.id == 0 || h.k + h.L <= 2 * WK_WB) {
              pos = c;
              mode = WM_WALK;
              rs = true;
              far_c = 0;
              if (P.stats) atomicAdd(&P.stats[31], 1ull);
              break;
            }
            if (!far_c && o < WK_WB) {
              far_c = c;
              far_n = c + h.k + h.L;
              far_id = h.id;
            }
          }
          if (mode == WM_WALK) break;
        }
        if (mode == WM_SYNC) from = WK_WB;
      }
      if (mode == WM_WALK) {
#pragma unroll 1
        while (pos < W1) {
          const uint32_t o = (uint32_t)(pos - W0);
          WHdr h = wk_hdr(wk_rd8(S, w, o));
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
          if (id > 2u || (id != 0u && L == 0)) {  // the chain dies: scan for a new one after it
            if (P.stats) {  // (DRP_STATS: deaths; the first one's bytes from LDS and from HBM)
              if (atomicAdd(&P.stats[32], 1ull) == 0) {
                P.stats[36] = pos;
                P.stats[37] = wk_rd8(S, w, o);
                P.stats[38] = g_rd8(P.bytes, pos);
                P.stats[39] = ((uint64_t)w << 32) | (lane << 16) | o;
              }
            }
            mode = WM_SYNC;
            from = o + 1u;
            break;
          }
          if (id == 0u) {
            note(pos, 0u, false);
            pos += k + 1u;
            continue;
          }
          if (L > se - pos - k) {  // a tail: the stream ends inside this frame
            note(pos, id, id == 2u);  // (a cut Change is carried, a cut blob delivered)
            term = MARK_TERM | pos;
            mode = WM_DONE;
            break;
          }
          note(pos, id, true);
          pos += k + L;
        }
        if (mode == WM_SYNC && from < WK_WB) continue;
      }
      break;
    }
    if (q == WK_WPT - 1 && mode == WM_SYNC && far_c) take_far();  // (its frame leaves the tile)
    if ((q & 3u) == 3u) {  // flush the group's 8 segment records
      const uint64_t ix = tcur * NT + (q >> 2) * 8u;
      *reinterpret_cast<uint64_t *>(P.ent + ix) = ent;
      *reinterpret_cast<uint64_t *>(P.ent_n + ix) = fn;
      *reinterpret_cast<uint64_t *>(P.ent_c + ix) = fc;
      ent = ~0ull;
      fn = 0;
      fc = 0;
    }
    if (q == WK_WPT - 1) {  // the tile's claim
      uint64_t cl = C_ID;
      if (term) cl = term;
      else if (mode == WM_WALK && had) cl = pos;
      P.claim[tcur] = cl;
      had = false;
      term = 0;
    }
    if (mode == WM_SYNC) from = 0;
  }
}

}  // namespace spec
}  // namespace drp

using namespace drp;

// Region walkers in place of claims_fast: the region list (and the edge tiles onto P->work), then
// the walkers. P->walk_rp: nstreams + 1 words; P->walk_tpr: tiles per region.
extern "C" hipError_t drp_launch_claims_walk(const DecodeParams *P, uint64_t nt_max, hipStream_t st) {
  if (nt_max == 0) return hipSuccess;
  hipLaunchKernelGGL(spec::walk_regions, dim3(1), dim3(1024), 0, st, *P);
  const uint64_t maxr = nt_max / P->walk_tpr + P->nstreams + 1;
  hipLaunchKernelGGL(spec::claims_walk, dim3((uint32_t)((maxr + WAVE - 1) / WAVE)), dim3(WAVE), 0, st, *P);
  return hipGetLastError();
}

extern "C" uint32_t drp_walk_tiles_per_region(uint64_t nt_max) {
  const uint64_t t = (nt_max + spec::WK_REGIONS - 1) / spec::WK_REGIONS;
  return (uint32_t)(t ? t : 1);
}
