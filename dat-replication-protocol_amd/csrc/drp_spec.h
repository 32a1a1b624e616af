// drp_spec.h — tile geometry, claim encodings and header parsing shared by the speculative
// decode kernels (drp_decode_spec.hip) and the region walker (drp_walk.hip).
#pragma once
#include "drp_device.h"
#include "drp_kernels.h"

namespace drp {
namespace spec {

#ifndef DRP_SPEC_NT
#define DRP_SPEC_NT 128
#endif
constexpr int NT = DRP_SPEC_NT;               // threads per workgroup (64: one wave, no s_barrier)
constexpr uint32_t SEGB = 64;                 // bytes per thread
constexpr uint32_t TILE = NT * SEGB;          // 8 KiB (4 KiB at NT 64): the B = NT tile geometry of tile_prefix
static_assert(NT == 64 || NT == 128, "one or two waves per tile");

// Workgroup barrier. A one-wave workgroup needs none: its LDS accesses complete in issue order,
// so only the compiler must not move LDS accesses across this point (and earlier ones retire).
__device__ __forceinline__ void bsync() {
  if constexpr (NT == 64) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else __syncthreads();
}
constexpr uint32_t HALO = 512;
constexpr uint32_t IMG = TILE + HALO;         // LDS image bytes (+32 slack)

constexpr uint64_t RDY = 1ull << 63;          // published word: value | RDY
constexpr uint64_t C_ID = 1ull << 62;         // claim: identity (no chain survives the tile)
constexpr uint64_t M_ERR = 1ull << 60;        // with MARK_TERM: the chain ended at an error header
constexpr uint64_t NONE = ~0ull;              // internal: no chain
constexpr uint32_t REC_NONE = 0xFFFFFFFFu;    // tile_rec: the tile has no records (fast_records)

constexpr uint32_t F_MISS = 1u << 12;         // overflow bit: prediction failed -> exact re-run
constexpr uint32_t F_WAIT = 1u << 13;
constexpr uint32_t F_CASCADE = 1u << 14;      // with F_MISS: go straight to the segmented repair
         // overflow bit: bounded wait expired -> exact re-run

// header parse on a 16-byte window (same grammar as parse_hdr_lds)
__device__ __forceinline__ Hdr parse_win(uint64_t w0, uint64_t w1, uint64_t p, uint64_t se) {
  Hdr h;
  h.succ = 0;
  h.id = 0;
  const uint64_t avail = se - p;
  const uint32_t b0 = (uint32_t)(w0 & 0xFF);
  if (b0 < 0x80u && avail >= 2) {  // one-byte length varint (the common case)
    const uint32_t id = (uint32_t)((w0 >> 8) & 0xFF);
    h.L = b0;
    h.vlen = 1;
    h.id = id;
    if (id >= 3) { h.kind = H_ERR_TYPE; return h; }
    if (id == 0) { h.kind = H_VALID; h.succ = p + 2; return h; }
    if (b0 == 0) { h.kind = H_ERR_LEN; return h; }
    if ((uint64_t)b0 > avail - 1) { h.kind = (id == 1) ? H_TAIL_CHANGE : H_TAIL_BLOB; return h; }
    h.kind = H_VALID;
    h.succ = p + 1 + b0;
    return h;
  }
  uint64_t L;
  const int k = win_varint(w0, w1, 0, avail, L);
  h.L = L;
  h.vlen = (uint32_t)(k > 0 ? k : 0);
  if (k == 0) { h.kind = H_TAIL_HDR; return h; }
  if (k < 0) { h.kind = (avail < 11) ? H_TAIL_HDR : H_ERR_VARINT; return h; }
  if ((uint64_t)k >= avail) { h.kind = H_TAIL_HDR; return h; }
  const uint32_t id = win_byte(w0, w1, (uint32_t)k);
  h.id = id;
  if (id >= 3) { h.kind = H_ERR_TYPE; return h; }
  if (id == 0) { h.kind = H_VALID; h.succ = p + (uint64_t)k + 1; return h; }
  if (L == 0) { h.kind = H_ERR_LEN; return h; }
  if (L > avail - (uint64_t)k) { h.kind = (id == 1) ? H_TAIL_CHANGE : H_TAIL_BLOB; return h; }
  h.kind = H_VALID;
  h.succ = p + (uint64_t)k + L;
  return h;
}

__device__ __forceinline__ uint64_t funnel(uint64_t lo, uint64_t hi, uint32_t sh) {
  return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}
__device__ __forceinline__ uint4 ld16(const uint8_t *g, uint64_t p, uint64_t se) {
  if (p + 16 <= se) return *reinterpret_cast<const uint4 *>(g + p);
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t k = 0; k < 16; k++)
    if (p + k < se) w[k >> 2] |= (uint32_t)g[p + k] << (8 * (k & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}


__device__ __forceinline__ bool is_pos(uint64_t v) { return v < (1ull << 60); }

// Tile geometry shared by both kernels.
// A load through the constant address space: a scalar load (s_load, no vmcnt) for a uniform
// address. Only for arrays no kernel that uses it writes (the stream and tile geometry, and the
// output bases in emit_tiles).
template <class T>
__device__ __forceinline__ T ldc(const T *p) {
  return *reinterpret_cast<const __attribute__((address_space(4))) T *>(reinterpret_cast<uintptr_t>(p));
}

struct TileGeo {
  uint64_t s, tf, so, se, A, e0;
};
__device__ __forceinline__ TileGeo tile_geo(const DecodeParams &P, uint64_t t) {
  TileGeo G;
  G.s = P.tile_stream ? ldc(P.tile_stream + t) : 0;
  if (G.s >= P.nstreams) G.s = P.nstreams - 1;  // (t past the last tile: read before the exit check)
  G.tf = ldc(P.tile_prefix + G.s);
  G.so = ldc(P.stream_off + G.s);
  G.se = ldc(P.stream_off + G.s + 1);
  G.A = (G.so & ~(uint64_t)(TILE - 1)) + (t - G.tf) * TILE;
  G.e0 = G.so + (P.entry ? ldc(P.entry + G.s) : 0ull);
  return G;
}

__device__ __forceinline__ void push_work(const DecodeParams &P, uint64_t t) {
  if (threadIdx.x == 0) P.work[atomicAdd(P.work_n, 1u)] = (uint32_t)t;
}

__device__ __forceinline__ Hdr hdr_global(const uint8_t *g, uint64_t p, uint64_t se) {  // (as Img::at from HBM)
  uint64_t w0, w1;
  const uint64_t a = p & ~15ull;
  const uint4 u = ld16(g, a, se), v = ld16(g, a + 16, se);
  const uint64_t q0 = ((uint64_t)u.y << 32) | u.x, q1 = ((uint64_t)u.w << 32) | u.z;
  const uint64_t q2 = ((uint64_t)v.y << 32) | v.x, q3 = ((uint64_t)v.w << 32) | v.z;
  const uint32_t o = (uint32_t)(p & 15);
  if (o < 8) {
    w0 = funnel(q0, q1, 8 * o);
    w1 = funnel(q1, q2, 8 * o);
  } else {
    w0 = funnel(q1, q2, 8 * (o - 8));
    w1 = funnel(q2, q3, 8 * (o - 8));
  }
  return parse_win(w0, w1, p, se);
}


// The claims form of a large batch (drp_launch_spec_head chooses it per launch from a density
// sample, walk_density): streams averaging <= HOP_FRAME bytes per frame take claims_fast, sparser
// ones the hop walkers (claims_hop: one header read per frame, so long frames cost nothing
// extra). P.walk_hop: 1 the hop walkers (forced: DRP_CLAIMS=hop), 2 by the density sample.
constexpr uint32_t HOP_FRAME = 512;
__device__ __forceinline__ bool walk_hops(const DecodeParams &P) { return P.walk_hop == 1u; }

}  // namespace spec
}  // namespace drp
