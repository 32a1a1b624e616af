// drp_decode_spec.hip — gfx950 decode, speculate-and-verify form (the default path).
//
// Replaces the per-frame loop of decode.js (Decoder._consume / _onheader / _onchangedata /
// _onchangeend / _onblobdata, decode.js:144-262) and messages.Change.decode
// (messages/index.js:5), like decode_tiles (drp_decode.hip), but with far less work per byte.
//
// Frames carry no sync marker, so a tile's first frame start e_t depends on every byte before
// it. decode_tiles resolves that exactly for every possible entry (lane DP + pointer doubling);
// this kernel instead *predicts* each tile's exit and proves the prediction afterwards:
//
//   1. stage     One workgroup = one 8 KiB tile (128 threads x 64 B) + a 512 B halo, read
//                from HBM once (dwordx4, coalesced) into LDS.
//   2. spec      Every thread takes the first live position of its 64 B whose header chain
//                survives KSTRONG frames ("strong" candidate). False chains in byte-random data
//                die with ~98% probability per frame; the stream's own chain never dies. The
//                threads' chains are linked (a thread continues the chain that enters it) by a
//                few Jacobi rounds; the chain's exit past the tile is the tile's *claim*
//                (or "identity" when no chain survives: the tile sits inside a long payload).
//                The claim is published at once — it does not depend on the tile's entry.
//   3. entry     Decoupled look-back over claims: e_t = the nearest predecessor claim that is
//                not identity (or the stream entry). Helping publishes inclusive values.
//   4. verify    The exact chain from e_t is walked (Jacobi again, seeded with the spec
//                chain, so usually one round). Its exit must equal claim_t (or e_t for an
//                identity claim); by induction from the stream entry every e_t is then exact.
//                Any mismatch raises SPEC_MISS; the missed tile's claim becomes its
//                verified exit and the host re-runs verification (repair passes) before
//                anything is emitted, falling back to the exact kernel (decode_tiles) only
//                when that does not settle, so results never depend on the prediction.
//   5. count     Exact frame count of the tile -> decoupled look-back (with helping) for the
//                output base; frames are decoded from LDS into the SoA columns.
//
// Workgroups take tiles in stream order from an atomic ticket, so a tile only ever waits on
// tiles already taken: no deadlock for any grid size. Cross-workgroup words are agent-scope
// relaxed atomics whose values are self-validating (READY bit / value + 1).
#include "drp_spec.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace drp {
namespace spec {

#ifndef DRP_K1_WAVES
#define DRP_K1_WAVES 8  // min waves per SIMD for claims_fast (its occupancy without an LDS image, see DRP_K1_GIMG)
#endif
#ifndef DRP_EMIT_WAVES
#define DRP_EMIT_WAVES 5  // min waves per SIMD for the emit kernel (0.88 -> 0.79 ms at 20M frames)
#endif
#ifndef DRP_KSTRONG
#define DRP_KSTRONG 4
#endif
constexpr int KSTRONG = DRP_KSTRONG;                    // frames a candidate chain must survive
struct Img {
  const uint8_t *lds;  // LDS image: byte 0 = absolute position A
  const uint8_t *g;    // the batch in HBM (16-byte aligned)
  uint64_t A, se;
  bool local = true;   // false: no LDS image (every header from HBM / L2)
  // header at absolute p < se: from LDS when its 16-byte window is inside the image,
  // else from HBM (two aligned 16-byte loads; only chains probed past the halo get here)
  __device__ __forceinline__ Hdr at(uint64_t p) const {
    uint64_t w0, w1;
    if (local && p + 16 <= A + IMG) {
      lds_win16(lds, (uint32_t)(p - A), w0, w1);
    } else {
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
    }
    return parse_win(w0, w1, p, se);
  }
};

__device__ __forceinline__ uint64_t term_of(const Hdr &h, uint64_t p) {
  return MARK_TERM | (h.kind >= H_ERR_VARINT ? M_ERR : 0ull) | p;
}

// The chain from entry E through this thread's bytes [.., s1): returns the first chain position
// >= s1 (or E itself when E >= s1 / is not a position), or MARK_TERM|q when the chain ends at
// q (tail or error); n = frames delivered on the way (decode.js delivers id 1/2 and partial blobs)
// in the low 16 bits, change frames among them in the high 16 bits (<= 32 each per thread).
// Prediction-side plausibility of a valid frame at p (never used on the exact path): a change
// frame behind a multi-byte length varint must hold a well-formed Change when it ends inside
// the LDS image. Shadow headers whose varint swallows a real header's first bytes declare
// ~10 KB+ "frames" whose payload runs on into the next frames' headers; real long frames
// (4 KB values) cost one field walk.
__device__ __forceinline__
bool change_ok(const uint8_t *lds, uint64_t A, uint64_t se, uint64_t po, uint64_t pl) {
  const LdsReader rd{lds, A, umin64(A + IMG, se)};
  const ChangeCols cc = decode_change(rd, po, pl);
  return !cc.err || cc.err == ERR_UNREACHABLE;
}
__device__ __forceinline__ bool plausible(const Img &m, uint64_t p, const Hdr &h, bool any_len) {
  if (!m.local || h.id != 1 || (!any_len && h.vlen < 2) || h.succ > m.A + IMG) return true;
  return change_ok(m.lds, m.A, m.se, p + h.vlen + 1, h.L - 1);
}

template <bool SPEC = false>
__device__ __forceinline__ uint64_t walk(const Img &m, uint64_t E, uint64_t s1, uint32_t &n) {
  n = 0;
  if (!is_pos(E)) return E;
  uint64_t p = E;
  while (p < s1 && p < m.se) {
    const Hdr h = m.at(p);
    if (SPEC && h.kind == H_VALID && !plausible(m, p, h, false)) return MARK_TERM | M_ERR | p;
    if (h.kind == H_VALID) {
      n += (h.id != 0) + ((h.id == 1) << 16);
      p = h.succ;
      continue;
    }
    n += h.kind == H_TAIL_BLOB;
    return term_of(h, p);
  }
  return p;
}

// Candidate c is strong if its chain survives KSTRONG frames (or reaches the stream end / a
// tail there after at least three frames) and its frames pass plausible(). far = its first
// frame ends past the tile. LOCAL: steps stay inside the LDS image; a chain that leaves it
// returns S_HBM (undecided) instead of reading HBM. On success also returns walk(c) for this
// thread (exit past s1 and the frames delivered in the thread's bytes).
enum : uint32_t { S_DEAD = 0, S_OK = 1, S_HBM = 2 };
#ifndef DRP_KSTRONG_HBM
#define DRP_KSTRONG_HBM 4
#endif
template <bool LOCAL>
__device__ __forceinline__ uint32_t strong(const Img &m, uint64_t c, uint64_t s1, uint64_t &R, uint32_t &n,
                                           bool &far, int khbm = 0) {
  uint64_t p = c;
  n = 0;
  R = NONE;
  far = false;
  // frames a deferred candidate survives in HBM (khbm: a weaker test prediction, DecodeParams)
  const int K = LOCAL ? KSTRONG : (khbm ? khbm : DRP_KSTRONG_HBM);
#pragma unroll 1
  for (int k = 0; k < K; k++) {
    if (p >= m.se) break;  // reached the stream end: survived
    if (LOCAL && p + 16 > m.A + IMG) return S_HBM;
    const Hdr h = m.at(p);
    if (h.kind == H_VALID) {
      if (k == 0) far = h.succ >= m.A + TILE;
      if (!plausible(m, p, h, false)) return S_DEAD;
      if (p < s1) n += (h.id != 0) + ((h.id == 1) << 16);
      p = h.succ;
      if (R == NONE && p >= s1) R = p;
      continue;
    }
    // errors kill the candidate; so does a tail soon after it: shadow headers with long
    // varints declare lengths past the stream end, real tails only end a long chain
    if (h.kind >= H_ERR_VARINT || k < 3) return S_DEAD;
    if (R == NONE) {  // the tail is inside this thread's bytes
      n += h.kind == H_TAIL_BLOB;
      R = term_of(h, p);
    }
    return S_OK;
  }
  if (R == NONE) {  // many tiny frames: finish this thread's bytes
    uint32_t n2;
    R = walk<true>(m, p, s1, n2);
    n += n2;
  }
  return S_OK;
}

// Link the threads' chains: thread l's entry is the exit of the latest thread before it whose
// entry lies inside its own bytes (a "carrier"; threads in between are jumped over). Spec mode:
// no carrier, or a carrier whose chain died at an error, restarts at the thread's own strong
// candidate g. Verify mode: a virtual carrier before thread 0 exits at e_first, errors pass on.
// One block-wide "latest carrier" scan per round; rounds repeat until no entry changes.
template <bool VERIFY>
__device__ __forceinline__
void link(const Img &m, uint64_t s1, uint64_t g, uint64_t e_first, uint64_t &E,
                                     uint64_t &R, uint32_t &n, uint64_t *wl, uint32_t *fl, uint32_t *overflow,
                                     bool *restart = nullptr) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  constexpr uint32_t NWV = NT / WAVE;
  for (uint32_t round = 0;; round++) {
    const bool carrier = is_pos(E) && E < s1;
    uint64_t x = carrier ? R : NONE;  // inclusive "latest carrier exit" over the wave
#pragma unroll
    for (uint32_t d = 1; d < WAVE; d <<= 1) {
      const uint64_t y = shfl_up64(x, d);
      if (lane >= d && x == NONE) x = y;
    }
    if (lane == 63) wl[wid] = x;
    bsync();  // (A) wl of this round visible; fl reads of the last round are done
    uint64_t prev = VERIFY ? e_first : NONE;  // latest carrier exit before this wave
#pragma unroll
    for (uint32_t w = 0; w < NWV; w++)
      if (w < wid && wl[w] != NONE) prev = wl[w];
    uint64_t ex = shfl_up64(x, 1);
    if (lane == 0 || ex == NONE) ex = prev;
    const bool rs = !VERIFY && (ex == NONE || ((ex & MARK_TERM) && (ex & M_ERR)));
    const uint64_t En = VERIFY ? ex : (rs ? g : ex);
    if (restart) *restart = rs;
    const bool ch = En != E;
    // only carriers feed the scan: a thread that neither is nor becomes one (its bytes lie
    // inside a frame that jumps over it) takes the passing exit without another round
    const bool relevant = ch && (carrier || (is_pos(En) && En < s1));
    const uint64_t any = __ballot(relevant);
    if (lane == 0) fl[wid] = any != 0;
    bsync();  // (B) fl visible; wl reads of this round are done
    uint32_t more = 0;
#pragma unroll
    for (uint32_t w = 0; w < NWV; w++) more |= fl[w];
    if (!more) {
      if (ch) {  // a non-carrier passes the exit on (walk returns it unchanged, no frames)
        E = En;
        R = En;
        n = 0;
      }
      break;
    }
    if (round > NT + 2) {  // cannot happen: entries settle thread by thread
      if (tid == 0) atomicOr(overflow, F_WAIT);
      break;
    }
    if (ch) {
      E = En;
      R = walk<!VERIFY>(m, E, s1, n);
    }
  }
}

// Wave scans and reductions on DPP (row shifts, then row broadcasts): __shfl_xor reductions cost
// ~5 VALU and a ds_bpermute per step. The compiler leaves update_dpp + op uncombined in the claims
// kernels (three VALU per step), so the prefix sum is one DPP op per step in inline asm (C2 claims
// ~30 VALU per wave fewer; 5.35 -> 5.32 ms per decode). Every use of it runs with all 64 lanes
// active (block-level code). s_nop 4 first: the five wait states between an SALU write of EXEC
// (the end of the branch before) and a DPP op; s_nop 1: the two between a VALU write and a DPP read.
#define DRP_DPP_STEPS(op)                                                                    \
  "s_nop 4\n\t" op " %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"     \
  "s_nop 1\n\t" op " %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"     \
  "s_nop 1\n\t" op " %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"     \
  "s_nop 1\n\t" op " %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"     \
  "s_nop 1\n\t" op " %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"              \
  "s_nop 1\n\t" op " %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
// inclusive prefix sum over the wave
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v) {
  asm volatile(DRP_DPP_STEPS("v_add_u32_dpp") : "+v"(v));
  return v;
}
// wave-uniform sum / maximum (lane 63 of the inclusive scan)
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp(v), 63);
}
__device__ __forceinline__ uint32_t wave_max_dpp(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ uint32_t wave_min_dpp(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, 0x111, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, 0x112, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, 0x114, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, 0x118, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, 0x142, 0xA, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, 0x143, 0xC, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// block-wide reductions over the NT threads (two barriers; scratch: NT / WAVE words). The scratch
// must not be one whose last reads were not followed by a barrier (link()'s fl: the first wave
// to finish would overwrite it under the other's last read, which then runs another link round
// against the wrong barrier; the shuffle reductions of earlier rounds only hid this by taking
// longer than that read).
__device__ __forceinline__ uint32_t block_max_u32(uint32_t v, uint32_t *xf) {
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  v = wave_max_dpp(v);
  if constexpr (NT == WAVE) return v;
  if (lane == 0) xf[wid] = v;
  bsync();
  uint32_t r = 0;
#pragma unroll
  for (uint32_t w = 0; w < NT / WAVE; w++) r = max(r, xf[w]);
  bsync();
  return r;
}
// two maxima with one exchange (scratch: 2 * NT / WAVE words)
__device__ __forceinline__ void block_max2_u32(uint32_t &a, uint32_t &b, uint32_t *xf) {
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  a = wave_max_dpp(a);
  b = wave_max_dpp(b);
  if constexpr (NT == WAVE) return;
  if (lane == 0) {
    xf[wid] = a;
    xf[NT / WAVE + wid] = b;
  }
  bsync();
#pragma unroll
  for (uint32_t w = 0; w < NT / WAVE; w++) {
    a = max(a, xf[w]);
    b = max(b, xf[NT / WAVE + w]);
  }
  bsync();
}
// need = any thread's pn; js = (the last thread with pj) + 1, or 0: ballots and one exchange
// (block_max2_u32 over 0/1 and tid + 1 values, without the wave reductions)
__device__ __forceinline__ void block_any_last(bool pn, bool pj, uint32_t &need, uint32_t &js, uint32_t *xf) {
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  const uint64_t bn = __ballot(pn), bj = __ballot(pj);
  const uint32_t n_w = bn != 0, j_w = bj ? wid * WAVE + 64u - (uint32_t)__builtin_clzll(bj) : 0u;
  if constexpr (NT == WAVE) {
    need = n_w;
    js = j_w;
    return;
  }
  if (lane == 0) {
    xf[wid] = n_w;
    xf[NT / WAVE + wid] = j_w;
  }
  bsync();
  need = 0;
  js = 0;
#pragma unroll
  for (uint32_t w = 0; w < NT / WAVE; w++) {
    need |= xf[w];
    js = max(js, xf[NT / WAVE + w]);
  }
  bsync();
}
// bits strictly above bit j of the 128-bit mask (m0 low, m1 high) exist
__device__ __forceinline__ bool any_above(uint64_t m0, uint64_t m1, uint32_t j) {
  if (j >= 64) return j < 127 && (m1 >> (j - 63)) != 0;
  return m1 != 0 || (j < 63 && (m0 >> (j + 1)) != 0);
}
// bits at or above bit j exist
__device__ __forceinline__ bool any_from(uint64_t m0, uint64_t m1, uint32_t j) {
  if (j >= 128) return false;
  if (j >= 64) return (m1 >> (j - 64)) != 0;
  return m1 != 0 || (m0 >> j) != 0;
}

__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v, uint32_t *xf) {
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  v = wave_sum_dpp(v);
  if constexpr (NT == WAVE) return v;
  if (lane == 0) xf[wid] = v;
  bsync();
  uint32_t r = 0;
#pragma unroll
  for (uint32_t w = 0; w < NT / WAVE; w++) r += xf[w];
  bsync();
  return r;
}

__device__ __forceinline__ uint64_t lane_min64(uint64_t v) {
#pragma unroll
  for (uint32_t k = 1; k < WAVE; k <<= 1) {
    const uint64_t o = ((uint64_t)shfl_xor32((uint32_t)(v >> 32), k) << 32) | shfl_xor32((uint32_t)v, k);
    v = o < v ? o : v;
  }
  return v;
}

// DRP_STATS=1: per-phase cycle sums of thread 0 in P.stats[40 + k] (profiling aid)
#define PHASE(k)                                                          \
  do {                                                                    \
    if (P.stats && threadIdx.x == 0) {                                    \
      const uint64_t now_ = __builtin_amdgcn_s_memtime();                 \
      atomicAdd(&P.stats[40 + (k)], (unsigned long long)(now_ - tl_));    \
      tl_ = now_;                                                         \
    }                                                                     \
  } while (0)


// The tile's bytes (64 per thread) and halo, loaded with no per-load branch when the whole
// image lies inside the batch buffer (bytes past the stream end are then the next stream's or
// padding: every parser bounds-checks against the stream end, and the live mask drops them);
// near the buffer end, guarded loads zero-fill. One uniform branch, so all loads are in flight
// together instead of one bounds-checked load at a time.
__device__ __forceinline__ void load_image(const DecodeParams &P, const TileGeo &G, uint4 (&v)[SEGB / 16], uint4 &h) {
  const uint32_t tid = threadIdx.x;
  const uint64_t lb = G.A + (uint64_t)tid * SEGB;
  if (G.A + IMG <= P.nbytes) {
    const uint4 *q = reinterpret_cast<const uint4 *>(P.bytes + lb);
#pragma unroll
    for (int k = 0; k < (int)(SEGB / 16); k++) v[k] = q[k];
    h = tid < HALO / 16 ? *reinterpret_cast<const uint4 *>(P.bytes + G.A + TILE + tid * 16) : make_uint4(0, 0, 0, 0);
  } else {
#pragma unroll
    for (int k = 0; k < (int)(SEGB / 16); k++) v[k] = ld16(P.bytes, lb + 16 * k, G.se);
    h = tid < HALO / 16 ? ld16(P.bytes, G.A + TILE + tid * 16, G.se) : make_uint4(0, 0, 0, 0);
  }
}

__device__ __forceinline__ void stage(const DecodeParams &P, const TileGeo &G, uint8_t *buf) {
  const uint32_t tid = threadIdx.x;
  uint4 v[SEGB / 16], h;
  load_image(P, G, v, h);
#pragma unroll
  for (int k = 0; k < (int)(SEGB / 16); k++) *reinterpret_cast<uint4 *>(buf + tid * SEGB + 16 * k) = v[k];
  if (tid < HALO / 16) *reinterpret_cast<uint4 *>(buf + TILE + tid * 16) = h;
  if (tid < 2) *reinterpret_cast<uint4 *>(buf + IMG + tid * 16) = make_uint4(0, 0, 0, 0);
  bsync();
}

// The image load_image() fetched into registers (a prefetch), written to LDS as stage() does.
__device__ __forceinline__ void put_image(uint8_t *buf, const uint4 (&v)[SEGB / 16], const uint4 &h) {
  const uint32_t tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < (int)(SEGB / 16); k++) *reinterpret_cast<uint4 *>(buf + tid * SEGB + 16 * k) = v[k];
  if (tid < HALO / 16) *reinterpret_cast<uint4 *>(buf + TILE + tid * 16) = h;
  if (tid < 2) *reinterpret_cast<uint4 *>(buf + IMG + tid * 16) = make_uint4(0, 0, 0, 0);
  bsync();
}

// Stage the tile and its halo with LDS-DMA (global_load_lds_dwordx4: no VGPRs hold the image;
// wave w's k-th load fills LDS bytes [4096 w + 1024 k, +1024) from the same offsets of the tile),
// except near the end of the batch buffer (guarded register loads there).
__device__ __forceinline__ void stage_glds(const DecodeParams &P, const TileGeo &G, uint8_t *buf) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  if (G.A + IMG > P.nbytes) {
    stage(P, G, buf);
    return;
  }
  const uint8_t *g = P.bytes + G.A;
#pragma unroll
  for (uint32_t k = 0; k < TILE / (NT / WAVE) / 1024; k++) {
    const uint32_t o = wid * (TILE / (NT / WAVE)) + k * 1024u;
    __builtin_amdgcn_global_load_lds((const void *)(g + o + lane * 16u),
                                     (__attribute__((address_space(3))) void *)(buf + o), 16, 0, 0);
  }
  if (wid == 0 && lane < HALO / 16)
    __builtin_amdgcn_global_load_lds((const void *)(g + TILE + lane * 16u),
                                     (__attribute__((address_space(3))) void *)(buf + TILE), 16, 0, 0);
  if (tid < 2) *reinterpret_cast<uint4 *>(buf + IMG + tid * 16) = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bsync();
}

// Stage the tile (64 B per thread, coalesced dwordx4) and its halo into LDS; returns the
// thread's live mask: positions in [max(so, A), se) whose bytes can start a header with
// id <= 2 (a varint terminator followed by a byte <= 2, reached through a run of MSB bytes).
__device__ __forceinline__ uint64_t stage_live(const DecodeParams &P, const TileGeo &G, uint8_t *buf) {
  const uint32_t tid = threadIdx.x;
  const uint64_t lb = G.A + (uint64_t)tid * SEGB;
  uint4 v[SEGB / 16], hv;
  load_image(P, G, v, hv);
#pragma unroll
  for (int k = 0; k < (int)(SEGB / 16); k++) *reinterpret_cast<uint4 *>(buf + tid * SEGB + 16 * k) = v[k];
  if (tid < HALO / 16) *reinterpret_cast<uint4 *>(buf + TILE + tid * 16) = hv;
  if (tid < 2) *reinterpret_cast<uint4 *>(buf + IMG + tid * 16) = make_uint4(0, 0, 0, 0);
  bsync();
  uint32_t m16[5], s16[5];
#pragma unroll
  for (int k = 0; k < 4; k++) gather16(v[k], m16[k], s16[k]);
  gather16(*reinterpret_cast<const uint4 *>(buf + tid * SEGB + SEGB), m16[4], s16[4]);
  const uint64_t M0 = (uint64_t)m16[0] | ((uint64_t)m16[1] << 16) | ((uint64_t)m16[2] << 32) | ((uint64_t)m16[3] << 48);
  const uint64_t S0 = (uint64_t)s16[0] | ((uint64_t)s16[1] << 16) | ((uint64_t)s16[2] << 32) | ((uint64_t)s16[3] << 48);
  const uint64_t M1 = m16[4], S1 = s16[4];
  uint64_t X[2], Mk[2];
  X[0] = ~M0 & ((S0 >> 1) | (S1 << 63));
  X[1] = ~M1 & (S1 >> 1);
  Mk[0] = M0;
  Mk[1] = M1;
#pragma unroll
  for (uint32_t d = 1; d <= 8; d <<= 1) {
    const uint64_t x0 = (X[0] >> d) | (X[1] << (64 - d)), x1 = X[1] >> d;
    X[0] |= Mk[0] & x0;
    X[1] |= Mk[1] & x1;
    if (d < 8) {
      const uint64_t m0 = (Mk[0] >> d) | (Mk[1] << (64 - d)), m1 = Mk[1] >> d;
      Mk[0] &= m0;
      Mk[1] &= m1;
    }
  }
  uint64_t live = X[0];
  const uint64_t lo = G.so > lb ? G.so - lb : 0, hi = G.se > lb ? G.se - lb : 0;
  if (lo >= 64 || hi == 0) live = 0;
  else {
    if (lo) live &= ~0ull << lo;
    if (hi < 64) live &= (1ull << hi) - 1;
  }
  return live;
}

// stage_live's live mask of this thread's bytes, from an image already staged in LDS
__device__ __forceinline__ uint64_t live_lds(const TileGeo &G, const uint8_t *buf) {
  const uint32_t tid = threadIdx.x;
  const uint64_t lb = G.A + (uint64_t)tid * SEGB;
  uint32_t m16[5], s16[5];
#pragma unroll
  for (int k = 0; k < 5; k++) gather16(*reinterpret_cast<const uint4 *>(buf + tid * SEGB + 16 * k), m16[k], s16[k]);
  const uint64_t M0 = (uint64_t)m16[0] | ((uint64_t)m16[1] << 16) | ((uint64_t)m16[2] << 32) | ((uint64_t)m16[3] << 48);
  const uint64_t S0 = (uint64_t)s16[0] | ((uint64_t)s16[1] << 16) | ((uint64_t)s16[2] << 32) | ((uint64_t)s16[3] << 48);
  const uint64_t M1 = m16[4], S1 = s16[4];
  uint64_t X[2], Mk[2];
  X[0] = ~M0 & ((S0 >> 1) | (S1 << 63));
  X[1] = ~M1 & (S1 >> 1);
  Mk[0] = M0;
  Mk[1] = M1;
#pragma unroll
  for (uint32_t d = 1; d <= 8; d <<= 1) {
    const uint64_t x0 = (X[0] >> d) | (X[1] << (64 - d)), x1 = X[1] >> d;
    X[0] |= Mk[0] & x0;
    X[1] |= Mk[1] & x1;
    if (d < 8) {
      const uint64_t m0 = (Mk[0] >> d) | (Mk[1] << (64 - d)), m1 = Mk[1] >> d;
      Mk[0] &= m0;
      Mk[1] &= m1;
    }
  }
  uint64_t live = X[0];
  const uint64_t lo = G.so > lb ? G.so - lb : 0, hi = G.se > lb ? G.se - lb : 0;
  if (lo >= 64 || hi == 0) live = 0;
  else {
    if (lo) live &= ~0ull << lo;
    if (hi < 64) live &= (1ull << hi) - 1;
  }
  return live;
}

// ==== kernel 1: every tile's claim (entry-independent, no waiting) ===========================
#ifndef DRP_LLCAP
#define DRP_LLCAP (8 * DRP_SPEC_NT)  // 1024 live positions per 8 KiB tile (C2 has ~220)
#endif
constexpr uint32_t LLCAP = DRP_LLCAP;  // live positions per tile checked through the LDS list
constexpr uint16_t NX_NEAR = 0xFFFD, NX_FAR = 0xFFFE, NX_DEAD = 0xFFFF;

#ifndef DRP_K1G_WAVES
#define DRP_K1G_WAVES 5  // min waves per SIMD for the general claims kernel (edge and dense tiles)
#endif
// the fast form (below), which spec_claims also runs for the stream-edge tiles on its list
struct FastLds;
// spec_claims' image buffer: the tile's image, or the edge form's FastLds (whose own image for the
// per-frame records is IMG + 32 bytes, plus its frame list and the small words)
constexpr uint32_t SPEC_BUF = IMG + 32 + 4 * DRP_SPEC_NT + 256;
enum : uint32_t { FC_OK = 0, FC_DENSE = 1 };
template <bool CF, bool EDGE = false, bool REC = false>
__device__ __forceinline__ uint32_t fast_claims(const DecodeParams &P, const TileGeo &G, uint64_t t, FastLds &S,
                                                uint32_t &eb_o, uint32_t &en_o, uint32_t &ecn_o, uint64_t &cl_o);
__global__ __launch_bounds__(NT, DRP_K1G_WAVES) void spec_claims(DecodeParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[SPEC_BUF];
  __shared__ uint64_t xr[NT / WAVE];
  __shared__ uint32_t xf[NT / WAVE];
  __shared__ uint64_t lmw[NT];
  __shared__ uint16_t loff[NT];
  __shared__ uint32_t xf2[2 * NT / WAVE];
  __shared__ uint64_t xm[4];  // candidate masks (two waves): [w] strong, [2 + w] strong and far
  __shared__ uint16_t lpos[LLCAP], lnx[LLCAP];
  __shared__ uint8_t lal[LLCAP];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u, wid = tid >> 6;
  uint64_t tl_ = P.stats && tid == 0 ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t ntiles = P.tile_prefix[P.nstreams];
  // With a work list (the fast kernel ran first): the edge and dense tiles it listed, a few per
  // workgroup; without one: every tile, one per workgroup.
  const uint32_t nwork = P.work ? *P.work_n : 0u;
  for (uint32_t wi = blockIdx.x; P.work ? wi < nwork : wi == blockIdx.x; wi += gridDim.x) {
  const uint64_t t = P.work ? P.work[wi] : wi;
  bsync();  // the previous tile's LDS reads are done
  const TileGeo G = tile_geo(P, t);  // (its loads go out with the tile count's)
  if (t >= ntiles) continue;  // (whole workgroup)
  // a stream-edge tile claims_fast listed: the fast form with the stream's bounds (its LDS in buf;
  // one with more than FCAP live positions goes on below)
  if (P.work && (G.A < G.so || G.A + IMG > G.se)) {
    uint32_t eb, en, ecn;
    uint64_t cl;
    if (fast_claims<true, true>(P, G, t, *reinterpret_cast<FastLds *>(buf), eb, en, ecn, cl) != FC_DENSE) continue;
    bsync();  // (its LDS reads are done before stage_live writes buf)
  }
  const uint64_t live = stage_live(P, G, buf);
  const Img m{buf, P.bytes, G.A, G.se};
  const uint64_t lb = G.A + (uint64_t)tid * SEGB, s1 = lb + SEGB;
  PHASE(0);

  // ---- strong candidate: the first live position whose chain survives, preferring chains
  // that can be checked inside the LDS image (shadow headers whose varint swallows a real
  // header jump ~10 KB+: checking them would cost a random HBM read each) ---------------------
  uint64_t g = NONE, R = NONE;
  uint32_t n = 0;
  bool far = false;
  uint64_t defer = 0;  // candidates whose check leaves the LDS image (decided in HBM if needed)
  // Survival of every live position of the tile, load-balanced: the positions go to an LDS
  // list, each is parsed once (its successor's list index, or "out"), then KSTRONG - 1 rounds
  // of look-ups propagate death back along the chains. lal: 0 dead, 1 strong, 2 undecided (the
  // chain leaves the LDS image: checked in HBM only if a restart needs it, see below).
  const uint32_t cnt = (uint32_t)__builtin_popcountll(live);
  const uint32_t cpre = wave_incl_scan32(cnt);
  if (lane == 63) xf[wid] = cpre;
  lmw[tid] = live;
  bsync();
  uint32_t off = cpre - cnt, total = 0;
#pragma unroll
  for (uint32_t w = 0; w < NT / WAVE; w++) {
    if (w < wid) off += xf[w];
    total += xf[w];
  }
  loff[tid] = (uint16_t)off;
  bsync();  // (xf is reused below)
  if (total <= LLCAP) {
    {
      uint64_t bits = live;
      uint32_t i = off;
      while (bits) {
        lpos[i++] = (uint16_t)(tid * SEGB + (uint32_t)__builtin_ctzll(bits));
        bits &= bits - 1;
      }
    }
    bsync();
    // tile-relative 32-bit arithmetic: the stream end as an offset from A (clamped), and the
    // one-byte-length header (every C2 frame) parsed inline; longer varints take parse_win
    const uint32_t se_rel = (uint32_t)umin64(G.se - G.A, 0x7FFFFFFFull);
    for (uint32_t i = tid; i < total; i += NT) {
      const uint32_t o = lpos[i] & 0x7FFFu;
      uint64_t w0, w1;
      lds_win16(buf, o, w0, w1);  // o < TILE: the 16-byte window is inside the image
      bool valid, near;  // near: the frame ends at or past the stream end
      uint32_t sr;       // successor offset from A (saturated)
      const uint32_t b0 = (uint32_t)(w0 & 0xFFu), id = (uint32_t)((w0 >> 8) & 0xFFu);
      if (b0 < 0x80u && se_rel - o >= 2u) {  // same grammar as parse_win's one-byte branch
        sr = id == 0 ? o + 2u : o + 1u + b0;
        valid = id < 3u && (id == 0 || (b0 != 0 && b0 <= se_rel - o - 1u));
        near = sr >= se_rel;  // (se_rel is exact whenever it can be reached from here)
      } else {
        const Hdr h = parse_win(w0, w1, G.A + o, G.se);
        valid = h.kind == H_VALID;
        sr = (uint32_t)umin64(h.succ - G.A, 0xFFFFFFFFull);
        near = h.succ >= G.se;
      }
      uint16_t code = NX_DEAD;
      uint8_t a = 0;
      if (valid && sr >= TILE) lpos[i] |= 0x8000u;  // first frame leaves the tile
      if (valid) {
        if (near) {
          code = NX_NEAR;  // the stream end: survived
          a = 1;
        } else if (sr >= TILE) {
          code = NX_FAR;   // past the tile: undecided (a restart that needs it checks in HBM)
          a = 2;
        } else {
          const uint32_t q = sr, th = q / SEGB, b = q % SEGB;
          const uint64_t lw = lmw[th];
          if ((lw >> b) & 1ull) {
            code = (uint16_t)(loff[th] + __builtin_popcountll(lw & ((1ull << b) - 1)));
            a = 1;
          }
        }
      }
      lnx[i] = code;
      lal[i] = a;
    }
    bsync();
    for (int r = 1; r < KSTRONG; r++) {
      for (uint32_t i = tid; i < total; i += NT) {
        const uint16_t v = lnx[i];
        if (lal[i] == 1 && v < NX_NEAR) {
          const uint8_t b = lal[v];
          if (b != 1) lal[i] = b;  // dead or undecided downstream
        }
      }
      bsync();
    }
    // this thread's first strong position; undecided ones are deferred
    for (uint32_t i = off; i < off + cnt; i++) {
      const uint8_t a = lal[i];
      if (a == 1) {
        g = G.A + (lpos[i] & 0x7FFFu);
        far = (lpos[i] & 0x8000u) != 0;
        break;
      }
      if (a == 2) defer |= 1ull << ((lpos[i] & 0x7FFFu) - tid * SEGB);
    }
    if (g != NONE) R = walk<true>(m, g, s1, n);
  } else {  // very dense tile: per-thread checks
    uint64_t bits = live;
    while (bits) {
      const uint32_t o = (uint32_t)__builtin_ctzll(bits);
      bits &= bits - 1;
      uint64_t r;
      uint32_t k;
      bool f;
      const uint32_t st = strong<true>(m, lb + o, s1, r, k, f);
      if (st == S_OK) {
        g = lb + o;
        R = r;
        n = k;
        far = f;
        break;
      }
      if (st == S_HBM) defer |= 1ull << o;
    }
  }
  // A chain that starts by jumping past the whole tile is trusted only when nothing later in
  // the tile could start one: a shadow whose long jump happens to land on a real frame start
  // survives any number of frames, but it jumps over the tile's real (dense) chain. The
  // tile-wide candidate masks (128 bits) are exchanged once; the survivors' mask S is then
  // known to every thread without further barriers.
  uint64_t S0, S1;
  {
    const uint64_t hm = __ballot(g != NONE), fm = __ballot(g != NONE && far);
    uint64_t H0 = hm, H1 = 0, F0 = fm, F1 = 0;  // one wave: its own ballots are the tile's masks
    if constexpr (NT == 2 * WAVE) {
      if (lane == 0) {
        xm[wid] = hm;
        xm[2 + wid] = fm;
      }
      bsync();
      H0 = xm[0];
      H1 = xm[1];
      F0 = xm[2];
      F1 = xm[3];
    }
    const uint64_t L1 = H1 ? ((1ull << (63 - __builtin_clzll(H1))) - 1) : 0ull;  // below the top bit
    const uint64_t L0 = H1 ? ~0ull : (H0 ? ((1ull << (63 - __builtin_clzll(H0))) - 1) : 0ull);
    S0 = H0 & ~(F0 & L0);
    S1 = H1 & ~(F1 & L1);
    if (far && any_above(H0, H1, tid)) {
      g = NONE;
      R = NONE;
      n = 0;
    }
  }
  uint64_t E = g;
  bool rs = false;  // this thread restarts the chain (no chain enters it, or the entering one died)
  PHASE(1);
  // ---- link the threads' chains ------------------------------------------------------------
  link<false>(m, s1, g, NONE, E, R, n, xr, xf, P.overflow, &rs);
  // A thread no chain reaches and without an LDS-decided candidate, with none later in the
  // tile either, decides its deferred candidates in HBM (big frames: the chain from a real
  // frame start leaves the image within a step or two), then the chains are linked again.
  // The first test rides on the reduction that finds the last carrier.
  uint32_t need = (E == NONE && defer && !any_above(S0, S1, tid)) ? 1u : 0u;
  uint32_t js = (is_pos(E) && E < s1) ? tid + 1 : 0u;  // last carrier + 1
  block_max2_u32(need, js, xf2);
  bool moved = false;
  for (uint32_t it = 0; need && it < 3; it++) {
    moved = true;
    if (E == NONE && defer && !any_above(S0, S1, tid)) {
      while (defer) {
        const uint32_t o = (uint32_t)__builtin_ctzll(defer);
        defer &= defer - 1;
        uint64_t r;
        uint32_t k;
        bool f;
        if (strong<false>(m, lb + o, s1, r, k, f, P.kstrong_hbm) == S_OK) {
          g = lb + o;
          E = g;
          R = r;
          n = k;
          break;
        }
      }
    }
    link<false>(m, s1, g, NONE, E, R, n, xr, xf, P.overflow, &rs);
    need = (E == NONE && defer && !any_above(S0, S1, tid)) ? 1u : 0u;
    js = (is_pos(E) && E < s1) ? tid + 1 : 0u;
    block_max2_u32(need, js, xf2);
  }
  PHASE(2);
  // The chain's last frame may jump over threads that hold strong candidates: a shadow that
  // joined the chain can jump far and land on a real frame start past the tile. Build the
  // chain those candidates start as well and keep it when it is the denser one (>= 2
  // frames where the first has one); a real long frame jumps over bytes with no candidate.
  {
    bool after;
    if (!moved) {
      after = any_from(S0, S1, js);  // survivors at or after the last carrier + 1
    } else {  // candidates changed in HBM: count them again
      after = block_max_u32(g != NONE && tid + 1 > js ? 1u : 0u, xf2) != 0;
    }
    if (js && after) {
      const uint64_t Ea = E, Ra = R;
      const uint32_t na = n;
      const bool rsa = rs;
      const bool mine = tid + 1 > js;
      E = NONE;
      R = NONE;
      n = 0;
      link<false>(m, s1, mine ? g : NONE, NONE, E, R, n, xr, xf, P.overflow, &rs);
      // (xf2: link's last reads of xf are not behind a barrier)
      const uint32_t nb = block_sum_u32(mine ? (n & 0xFFFFu) : 0u, xf2);
      if (nb < 2 || !mine) {  // keep the first chain where the dense one does not apply
        E = Ea;
        R = Ra;
        n = na;
        rs = rsa;
      }
    }
  }
  PHASE(3);
  // per-thread record for kernel 2: entry offset (| 0x40 when the thread restarts the chain,
  // 0xFF none), frames and change frames delivered from it
  {
    // (a thread at or past its stream's end gets the chain's end passed on as E: no record, so the
    // records-only check does not read a wrapped entry byte as a restart and relist every stream's
    // last tile)
    const bool carrier = is_pos(E) && E >= lb && E < s1 && E < G.se;
    const uint64_t ix = t * NT + tid;
    P.ent[ix] = carrier ? (uint8_t)((E - lb) | (rs ? 0x40u : 0u)) : (uint8_t)0xFF;
    P.ent_n[ix] = carrier ? (uint8_t)(n & 0xFFFFu) : (uint8_t)0;
    P.ent_c[ix] = carrier ? (uint8_t)(n >> 16) : (uint8_t)0;
  }
  if (tid == NT - 1) P.claim[t] = (R == NONE || ((R & MARK_TERM) && (R & M_ERR))) ? C_ID : R;
  }
}

// ==== kernel 1, fast form: claims of interior tiles ============================================
// Same outputs as spec_claims (claim, per-thread entry records), for the tiles whose LDS image
// [A, A + IMG) lies inside their stream: no stream-start masking, every in-tile header window is
// inside the image and the stream, and all arithmetic is 32-bit and tile-relative. Differences in
// what is *predicted* (never in what is output: verification is exact):
//  * live positions are those of 1..3-byte length varints (frames < 2 MiB); a longer frame's
//    header is no candidate, so a tile whose chain holds one mispredicts and is repaired;
//  * a change frame behind a multi-byte varint that ends inside the image must start with a
//    Change field tag (subset, key, change, from, to, value), not hold a well-formed Change;
//  * every live position is parsed once into an LDS node (successor node and offset, type);
//    chain walks and the threads' link rounds follow nodes and never re-parse a header;
//  * the link's "latest carrier" lookup is a ballot + one lane permute, not a shuffle scan.
// Edge tiles and tiles with more than FCAP live positions are appended to a work list for the
// general kernel, which runs after this one.
#ifndef DRP_FCAP
#define DRP_FCAP 512
#endif
constexpr uint32_t FCAP = DRP_FCAP;
constexpr uint16_t NX_TAILB = 0xFFFB, NX_TAILC = 0xFFFC;  // the node's frame runs past the stream end
// Chain exits (32-bit): a node index | its offset << 16 (offset < 0x4000: the tile and its halo), or
constexpr uint32_t RX_NONE = 0xFFFFFFFFu;  // no chain
constexpr uint32_t RX_DEAD = 0xFFFFFFFEu;  // the chain died (invalid header)
constexpr uint32_t RX_FAR = 0x80000000u;   // | node: that node's frame ends past the listed positions
constexpr uint32_t RX_TERM = 0x40000000u;  // | node: that node's frame is cut by the stream end (tail)
static_assert(IMG < 0x4000, "node offsets are 14-bit");
__device__ __forceinline__ bool rx_node(uint32_t x) { return x < RX_TERM; }
__device__ __forceinline__ uint32_t rx_off(uint32_t x) { return x >> 16; }  // (nodes only)

// 16-byte block -> bit k = MSB of byte k (m), bit k = byte k <= 2 (s); v_dot4 gathers the bits
__device__ __forceinline__ uint32_t le2_bytes(uint32_t x) { return ~(((x | 0x80808080u) - 0x03030303u) | x) & 0x80808080u; }
__device__ __forceinline__ uint32_t gather_msb(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t lo = __builtin_amdgcn_udot4(a, 0x08040201u, __builtin_amdgcn_udot4(b, 0x80402010u, 0u, false), false);
  const uint32_t hi = __builtin_amdgcn_udot4(c, 0x08040201u, __builtin_amdgcn_udot4(d, 0x80402010u, 0u, false), false);
  return (lo >> 7) | (hi << 1);  // (both are 128 x an 8-bit mask)
}
__device__ __forceinline__ uint32_t masks16(const uint4 v) {  // m | s << 16
  constexpr uint32_t H = 0x80808080u;
  const uint32_t m = gather_msb(v.x & H, v.y & H, v.z & H, v.w & H);
  const uint32_t s = gather_msb(le2_bytes(v.x), le2_bytes(v.y), le2_bytes(v.z), le2_bytes(v.w));
  return m | (s << 16);
}


// A Change frame that leaves the listed positions (long frames: C5's 4 KB values) cannot have its
// chain followed in the image. It is strong when its payload parses as a Change in the schema's
// own shape: one-byte tags of the schema with their wire types (length-delimited subset, key and
// value; varint change, from and to of <= 5 bytes), every field header at most 512 bytes past the
// image (read from the batch, not the LDS), the
// required fields present, and the last field ending exactly at the payload end (the value's
// bytes are not read). Random bytes essentially never pass; a real frame in another shape is left
// undecided as before. Prediction only: verification is exact.
__device__ __forceinline__ bool change_fills(const uint32_t *w32, uint32_t po, uint32_t pl, uint32_t lim,
                                             uint32_t off = 0, uint32_t found = 0) {
#pragma unroll 1
  for (uint32_t f = 0; f < 8u && off < pl; f++) {
    const uint32_t q = po + off;
    if (q + 12u > lim) return false;
    const uint32_t d = q >> 2, sh = (q & 3u) * 8u;
    const uint32_t a0 = w32[d], a1 = w32[d + 1], a2 = w32[d + 2];
    const uint32_t w = __builtin_amdgcn_alignbit(a1, a0, sh), wn = __builtin_amdgcn_alignbit(a2, a1, sh);
    const uint32_t b0 = w & 0xFFu, tag = b0 >> 3;
    const bool num = tag - 3u <= 2u;  // change / from / to: varints; subset / key / value: lengths
    if (b0 >= 0x80u || tag - 1u > 5u || (b0 & 7u) != (num ? 0u : 2u)) return false;
    const uint32_t x = __builtin_amdgcn_alignbit(wn, w, 8);  // bytes 1..4
    const uint32_t tm = ~x & 0x80808080u;
    uint32_t k2;
    uint64_t v = (x & 0x7Fu) | ((x >> 1) & 0x3F80u) | ((x >> 2) & 0x1FC000u) | ((x >> 3) & 0xFE00000u);
    if (tm) {
      k2 = ((uint32_t)__builtin_ctz(tm) >> 3) + 1u;
      v &= (1u << (7u * k2)) - 1u;
    } else {
      const uint32_t b5 = (wn >> 8) & 0xFFu;
      if (b5 & 0x80u) return false;
      k2 = 5u;
      v |= (uint64_t)b5 << 28;
    }
    if (k2 + 1u > pl - off) return false;
    if (num) {
      found |= 1u << (tag - 2u);
      off += 1u + k2;
    } else {
      const uint32_t o2 = off + 1u + k2;
      if (v > (uint64_t)(pl - o2)) return false;
      if (tag == 2u) found |= 1u;
      off = o2 + (uint32_t)v;
    }
  }
  return off == pl && found == 15u;
}

// change_fills after the first field, with one load level: the 28 bytes from q = po + off (the
// numeric fields of <= 6 bytes each, then the value's tag and length) are loaded together and parsed
// from registers. The value must end the payload. 1: strong; 0: not a Change of that shape (C2's
// swallowing shadow headers, which read a real frame's fields and then its successor's header,
// stop here after one load instead of six); 2: another shape (a subset before the key): the
// field-by-field check decides.
__device__ __forceinline__ uint32_t change_fills_win(const uint32_t *w32, uint32_t po, uint32_t pl, uint32_t lim,
                                                     uint32_t off, uint32_t found) {
  const uint32_t q = po + off;
  if (q + 36u > lim) return 2u;  // (the nine dwords from q & ~3)
  const uint32_t d = q >> 2, sh = (q & 3u) * 8u;
  uint32_t a[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a[i] = w32[d + i];
  uint64_t x[4];  // bytes q .. q + 31
#pragma unroll
  for (int i = 0; i < 4; i++)
    x[i] = (uint64_t)__builtin_amdgcn_alignbit(a[2 * i + 1], a[2 * i], sh) |
           ((uint64_t)__builtin_amdgcn_alignbit(a[2 * i + 2], a[2 * i + 1], sh) << 32);
  uint32_t used = 0;
#pragma unroll
  for (int f = 0; f < 4; f++) {
    const uint32_t b0 = (uint32_t)x[0] & 0xFFu, tag = b0 >> 3;
    const uint64_t y = x[0] >> 8;  // the varint's bytes (up to 5)
    const uint64_t tm = ~y & 0x8080808080ull;
    if (b0 >= 0x80u || !tm) return 0u;
    const uint32_t k2 = ((uint32_t)__builtin_ctzll(tm) >> 3) + 1u;
    const uint64_t v = ((y & 0x7Full) | ((y >> 1) & 0x3F80ull) | ((y >> 2) & 0x1FC000ull) | ((y >> 3) & 0xFE00000ull) |
                        ((y >> 4) & 0x7F0000000ull)) & ((1ull << (7u * k2)) - 1ull);
    if (tag - 3u <= 2u && (b0 & 7u) == 0u) {  // change / from / to
      found |= 1u << (tag - 2u);
      const uint32_t s = 1u + k2;
      used += s;
      if (off + used > pl) return 0u;
      const uint32_t b = 8u * s;  // (2..6 bytes)
      x[0] = (x[0] >> b) | (x[1] << (64u - b));
      x[1] = (x[1] >> b) | (x[2] << (64u - b));
      x[2] = (x[2] >> b) | (x[3] << (64u - b));
      x[3] >>= b;
      continue;
    }
    if (b0 == 0x32u) {  // the value: it must end the payload
      return (found == 15u && (uint64_t)off + used + 1u + k2 + v == (uint64_t)pl) ? 1u : 0u;
    }
    if (b0 == 0x0Au || b0 == 0x12u) return 2u;  // a length-delimited field before the value
    return 0u;
  }
  return 2u;
}

// Node word: successor code (node index or NX_*) | min(successor offset, 0x3FFF) << 16 | id << 30
// (id 3: the node's own header is invalid).
// Walk from node exit x (offset < s1r) through the thread's bytes: returns the exit (a node whose
// offset is >= s1r, or RX_*); n = frames delivered | change frames << 16.
__device__ __forceinline__ uint32_t fwalk(const uint32_t *lnd, uint32_t x, uint32_t s1r, uint32_t &n) {
  n = 0;
  uint32_t i = x & 0xFFFFu;
#pragma unroll 1
  for (;;) {
    const uint32_t nd = lnd[i], id = nd >> 30, c = nd & 0xFFFFu, q = (nd >> 16) & 0x3FFFu;
    if (id == 3) return RX_DEAD;
    if (c == NX_TAILC) return RX_TERM | i;  // a change frame cut by the stream end is not delivered
    n += 1u + ((id == 1) << 16) - (id == 0);
    if (c == NX_TAILB) return RX_TERM | i;  // a partial blob is delivered and ends the chain
    if (c == NX_FAR || c == NX_NEAR) return RX_FAR | i;
    if (q >= s1r) return c == NX_DEAD ? RX_DEAD : (c | (q << 16));
    if (c == NX_DEAD) return RX_DEAD;
    i = c;
  }
}

// Link rounds (spec mode of link()): a thread's entry is the exit of the latest carrier before it;
// no carrier, or a dead one, restarts the chain at the thread's own strong node g. A correction
// travels one carrier per round, so two chains that never merge (a dense second framing) take a
// round per frame of the tile: with cap, the rounds stop there and flink returns true (E, R, n
// then unsettled; the caller takes claims_fast's pointer-jumping form instead).
__device__ __forceinline__ bool flink(const uint32_t *lnd, uint32_t s1r, uint32_t g, uint32_t &E, uint32_t &R,
                                      uint32_t &n, bool &rs, uint32_t *wl, uint32_t *fl, uint32_t *overflow,
                                      unsigned long long *stats = nullptr, uint32_t cap = ~0u) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll 1
  for (uint32_t round = 0;; round++) {
    const bool carrier = rx_node(E) && rx_off(E) < s1r;
    const uint64_t cm = __ballot(carrier);
    const uint64_t bm = cm & below;
    const uint32_t j = bm ? 63u - (uint32_t)__builtin_clzll(bm) : 0u;
    const uint32_t xj = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(j << 2), (int)R);
    if constexpr (NT == 2 * WAVE) {
      if (lane == 0) wl[wid] = cm ? (uint32_t)__builtin_amdgcn_readlane((int)R, 63 - __builtin_clzll(cm)) : RX_NONE;
      bsync();  // (A) wl visible; fl reads of the last round are done
    }
    const uint32_t prev = (NT == 2 * WAVE && wid == 1) ? wl[0] : RX_NONE;
    const uint32_t ex = bm ? xj : prev;
    const bool r = ex >= RX_DEAD;  // none or dead
    const uint32_t En = r ? g : ex;
    const bool ch = En != E;
    const bool relevant = ch && (carrier || (rx_node(En) && rx_off(En) < s1r));
    const uint64_t any = __ballot(relevant);
    bool more = any != 0;
    if constexpr (NT == 2 * WAVE) {
      if (lane == 0) fl[wid] = any != 0;
      bsync();  // (B) fl visible; wl reads of this round are done
      more = (fl[0] | fl[1]) != 0;
    }
    rs = r;
    if (more && round + 1 >= cap) return true;  // (block-uniform: more is)
    if (!more) {
      if (stats && tid == 0) {  // (DRP_STATS: rounds, their maximum, tiles over 8)
        atomicAdd(&stats[56], (unsigned long long)(round + 1));
        atomicMax(&stats[57], (unsigned long long)(round + 1));
        if (round + 1 > 8) atomicAdd(&stats[58], 1ull);
      }
      if (ch) {  // a non-carrier passes the exit on
        E = En;
        R = En;
        n = 0;
      }
      break;
    }
    if (round > NT + 2) {  // cannot happen: entries settle thread by thread
      if (tid == 0) atomicOr(overflow, F_WAIT);
      break;
    }
    if (ch) {
      E = En;
      if (rx_node(E) && rx_off(E) < s1r) R = fwalk(lnd, E, s1r, n);
      else {
        R = E;
        n = 0;
      }
    }
  }
  return false;
}



constexpr uint32_t HV = HALO / SEGB;  // halo "threads" with nodes
// LDS of the fast claims form
// claims_fast keeps no LDS image of the tile: every live position's header is parsed from the
// L2 lines the tile load just brought in (the byte masks come from the loaded registers), so a
// tile takes 6.2 KB of LDS instead of 15 and the kernel runs at 8 waves/SIMD (52 VGPRs) instead
// of 5: the HBM stream of some workgroups overlaps the instruction-bound work of others
// (C2 100M: 3.37 -> ~2.8 ms; C5: 3.77 -> ~2.4 ms).
struct FastLds {
  union {
    struct {
      uint64_t lmw[NT + HV];   // live masks; then strong masks
      uint64_t dmw[NT];        // undecided masks
      uint16_t loff[NT + HV];  // first list index of each thread
      uint32_t hmx[HALO / 16 + 1];  // halo masks per 16 bytes
      uint16_t lpos[FCAP];
      uint32_t lnd[FCAP > NT + 1 ? FCAP : NT + 1];  // nodes (first: the next-16-byte masks; last: the emit list)
      uint8_t lal[FCAP];  // 0 dead, 1 strong, 2 undecided (leaves the image)
      uint32_t lsucc[FCAP];  // successor offset of the nodes whose frame leaves the list (the claim of a
                             // chain that ends in one: no header re-read from HBM at the tile's end)
    };
    // the per-frame records' image of the tile and its halo, staged from the registers of the tile
    // load once the frames are listed (fast_records: everything above is dead by then)
    __attribute__((aligned(16))) uint8_t img[IMG + 32];
  };
  uint32_t fls[NT];  // fast_records: the tile's delivered frames in chain order (offset | id << 14 | tailb << 16)
  uint32_t xw[8];
  uint32_t xf[2 * NT / WAVE], wl[NT / WAVE], fl[NT / WAVE];
  uint64_t xm[4];  // candidate masks (two waves): [w] strong, [2 + w] strong and far
#ifdef DRP_K1_PAD
  uint8_t pad[DRP_K1_PAD];  // (A/B only: caps the workgroups per CU through LDS)
#endif
};
static_assert(sizeof(FastLds) <= SPEC_BUF, "spec_claims runs the edge form in its image buffer");


// claims_fast when the link rounds do not settle within DRP_FL_CAP rounds (two chains that never
// merge, e.g. tests/_streams.shadow_stream's second framing: ~42 rounds per tile, 77% of the
// kernel on that input). The converged link is the chain from the first thread's strong node,
// node to node by each node's walk through its own thread's bytes (a death restarts at the next
// thread's strong node; the halo, a frame past the image or a tail ends it). Every node's next
// node is computed once, and pointer jumping gives every node its chain's end in log2(hops)
// rounds; the claim is the first strong node's. The deferred restarts and rule 3 are not applied.
// Records: none (0xFF), so the records-only check relists the tile and verify_counts re-walks it
// from its exact entry (on the second framing, the cascade shortcut takes the whole list instead).
#ifndef DRP_FL_CAP
#define DRP_FL_CAP 6  // link rounds before the pointer-jumping form (~0: never); clean C2 tiles settle in <= 5
#endif
constexpr uint32_t JT_C_ID = 2u << 30, JT_TERM = 1u << 30, JT_NONE = 0xFFFFu;
template <uint32_t NTT>
__device__ __forceinline__ uint32_t fast_claims_jump(const DecodeParams &P, uint64_t t, uint64_t A, FastLds &S, uint32_t g,
                                                  uint32_t ttotal, uint32_t total, uint32_t &eb_o, uint32_t &en_o,
                                                  uint32_t &ecn_o, uint64_t &cl_o) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  constexpr uint32_t KPT = FCAP / NTT;
  uint16_t *nx = reinterpret_cast<uint16_t *>(S.lmw);  // (the candidate masks are read: free)
  uint32_t *gl = reinterpret_cast<uint32_t *>(S.dmw);
  uint32_t *lnd = S.lnd;
  if (P.stats && tid == 0) atomicAdd(&P.stats[60], 1ull);  // (DRP_STATS: tiles in this form)
  const uint64_t gm = __ballot(g != RX_NONE);
  if (lane == 0) S.xm[wid] = gm;
  gl[tid] = g;
  bsync();
  const uint64_t G0 = S.xm[0], G1 = NTT == 2 * WAVE ? S.xm[1] : 0ull;
  uint32_t yn[KPT], yt[KPT];
#pragma unroll
  for (uint32_t j = 0; j < KPT; j++) {
    const uint32_t i = tid + j * NTT;
    yn[j] = JT_NONE;
    yt[j] = JT_C_ID;
    if (i < ttotal) {  // a tile node: the exit of the walk through its own thread's bytes
      const uint32_t o = S.lpos[i], th = o / SEGB;
      uint32_t cnt;
      const uint32_t x = fwalk(lnd, i, (th + 1u) * SEGB, cnt);
      if (rx_node(x)) {
        const uint32_t k = x & 0xFFFFu;
        if (S.lpos[k] >= TILE) yt[j] = S.lpos[k];  // (a halo node: the chain leaves the tile there)
        else yn[j] = k;
      } else if (x == RX_DEAD) {  // the next thread with a strong node restarts the chain
        const uint64_t a0 = th + 1u < 64u ? G0 & (~0ull << (th + 1u)) : 0ull;
        const uint64_t a1 = th + 1u < 64u ? G1 : (th + 1u < 128u ? G1 & (~0ull << (th + 1u - 64u)) : 0ull);
        const uint32_t k = a0 ? (uint32_t)__builtin_ctzll(a0) : (a1 ? 64u + (uint32_t)__builtin_ctzll(a1) : NTT);
        if (k < NTT) yn[j] = gl[k] & 0xFFFFu;
      } else if (x & RX_FAR) {
        yt[j] = S.lsucc[x & 0xFFFFu];
      } else if (x & RX_TERM) {
        yt[j] = JT_TERM | S.lpos[x & 0xFFFFu];
      }
    } else if (i < total) {
      yt[j] = S.lpos[i];  // (halo nodes end chains)
    }
  }
  bsync();  // (the walks' reads of lnd are done)
#pragma unroll
  for (uint32_t j = 0; j < KPT; j++) {
    const uint32_t i = tid + j * NTT;
    if (i < total) {
      nx[i] = (uint16_t)yn[j];
      lnd[i] = yt[j];
    }
  }
  bsync();
#pragma unroll 1
  for (uint32_t round = 0; round < 10u; round++) {  // (hops < 2^9: each leaves a thread)
    uint32_t chm = 0;
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++) {
      const uint32_t i = tid + j * NTT;
      if (i < total && nx[i] != JT_NONE) {
        const uint32_t a = nx[i], b = nx[a];
        yn[j] = b;
        yt[j] = b == JT_NONE ? lnd[a] : 0u;
        chm |= 1u << j;
      }
    }
    const uint64_t any = __ballot(chm != 0);
    if (lane == 0) S.fl[wid] = any != 0;
    bsync();  // (this round's reads are done; flags visible)
    uint32_t more = 0;
#pragma unroll
    for (uint32_t w = 0; w < NTT / WAVE; w++) more |= S.fl[w];
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++)
      if ((chm >> j) & 1u) {
        const uint32_t i = tid + j * NTT;
        nx[i] = (uint16_t)yn[j];
        if (yn[j] == JT_NONE) lnd[i] = yt[j];
      }
    bsync();  // (writes visible; flag reads done)
    if (!more) break;
  }
  const uint64_t ix = t * NTT + tid;
  eb_o = 0xFFu;
  en_o = 0;
  ecn_o = 0;
  P.ent[ix] = 0xFF;
  P.ent_n[ix] = 0;
  P.ent_c[ix] = 0;
  cl_o = 0;
  if (tid == NTT - 1) {
    uint64_t cl = C_ID;
    if (G0 | G1) {
      const uint32_t k = G0 ? (uint32_t)__builtin_ctzll(G0) : 64u + (uint32_t)__builtin_ctzll(G1);
      const uint32_t s0 = gl[k] & 0xFFFFu;
      const uint32_t code = nx[s0] == JT_NONE ? lnd[s0] : JT_C_ID;  // (settled: every next is JT_NONE)
      if (code == JT_C_ID) cl = C_ID;
      else if (code & JT_TERM) cl = MARK_TERM | (A + (code & ~JT_TERM));
      else cl = A + code;
    }
    P.claim[t] = cl;
    cl_o = cl;
  }
  return FC_OK;
}

// ---- per-frame records: the wire is read once (C2) ------------------------------------------------
// claims_fast already holds each thread's chain, so after the claim it decodes the Change fields of
// every frame its threads deliver (the exact frames of the tile from verification's entry thread on,
// plus the shadow frames of the threads before it) into CR_WORDS words per frame, and emit_lean
// expands the records of the tiles verification lets it (tile_recok) into columns without staging
// the tile again (decode.js:144-169 / 205-214 deliver the same frames in the same order). Per tile,
// CR_CAP slots in slot order = chain order (the threads' frame counts, prefix-summed), word-major so
// each word of a wave's frames is one coalesced store:
//   w0  payload offset from the tile's first byte (14 bits) | id << 14 | partial (a blob cut by the
//       stream end) << 16 | has value << 17 | key length varint bytes << 18
//   w1  payload length (the header's, as the column)
//   w2  key length | value offset << 16 (payload-relative)
//   w3..w5 change, from, to
// Recorded: blob frames, and Change payloads in protocol-buffers' own shape without a subset: key
// (length varint of <= 2 bytes) change from to [value], one-byte tags, numbers < 2^32, the last field
// ending the payload. Anything else (a subset, longer varints, a field header near the stream end,
// more than CR_CAP frames) leaves the tile without records (tile_rec REC_NONE): emit_lean then decodes
// it from the wire as before, and errors are reported there. The record of a frame is only a
// restatement of its header and fields; verification proves which frames are real.
#ifndef DRP_CREC_STAGE
#define DRP_CREC_STAGE 2  // (A/B builds: 0 stops after the frame list, 1 after the field decode)
#endif
constexpr uint32_t CR_CAP = NT, CR_WORDS = 6, CR_TILE_WORDS = CR_CAP * CR_WORDS;
static_assert(CR_CAP == NT, "one frame per thread in the record decode");

// one frame's fields from the 28 bytes at payload-relative ke (numbers of any width up to 5 bytes,
// value length up to 4 bytes): false when the payload is in another shape
__device__ __forceinline__ bool crec_general(const uint32_t *w32, uint32_t qa, uint32_t ke, uint32_t pl,
                                             uint32_t &num0, uint32_t &num1, uint32_t &num2, uint32_t &vo, bool &hv) {
  const uint32_t d = qa >> 2, sh = (qa & 3u) * 8u;
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = w32[d + i];
  uint64_t x[4];  // bytes qa .. qa + 27 (x[3]: 4 bytes)
#pragma unroll
  for (int i = 0; i < 3; i++)
    x[i] = (uint64_t)__builtin_amdgcn_alignbit(a[2 * i + 1], a[2 * i], sh) |
           ((uint64_t)__builtin_amdgcn_alignbit(a[2 * i + 2], a[2 * i + 1], sh) << 32);
  x[3] = __builtin_amdgcn_alignbit(a[7], a[6], sh);
  uint32_t used = 0, nums[3];
#pragma unroll
  for (int f = 0; f < 3; f++) {
    const uint32_t b0 = (uint32_t)x[0] & 0xFFu;
    const uint64_t y = x[0] >> 8;
    const uint64_t tm = ~y & 0x8080808080ull;
    if (b0 != 0x18u + 8u * (uint32_t)f || !tm) return false;
    const uint32_t k2 = ((uint32_t)__builtin_ctzll(tm) >> 3) + 1u;
    const uint64_t v = ((y & 0x7Full) | ((y >> 1) & 0x3F80ull) | ((y >> 2) & 0x1FC000ull) | ((y >> 3) & 0xFE00000ull) |
                        ((y >> 4) & 0x7F0000000ull)) & ((1ull << (7u * k2)) - 1ull);
    if (v >> 32) return false;
    nums[f] = (uint32_t)v;
    const uint32_t s = 1u + k2, b = 8u * s;  // (2..6 bytes)
    used += s;
    x[0] = (x[0] >> b) | (x[1] << (64u - b));
    x[1] = (x[1] >> b) | (x[2] << (64u - b));
    x[2] = (x[2] >> b) | (x[3] << (64u - b));
    x[3] >>= b;
  }
  num0 = nums[0];
  num1 = nums[1];
  num2 = nums[2];
  if (ke + used > pl) return false;
  hv = ke + used != pl;
  vo = 0;
  if (!hv) return true;
  const uint32_t b0 = (uint32_t)x[0] & 0xFFu;
  const uint64_t y = x[0] >> 8;
  const uint64_t tm = ~y & 0x80808080ull;
  if (b0 != 0x32u || !tm) return false;
  const uint32_t k2 = ((uint32_t)__builtin_ctzll(tm) >> 3) + 1u;
  const uint64_t v = ((y & 0x7Full) | ((y >> 1) & 0x3F80ull) | ((y >> 2) & 0x1FC000ull) | ((y >> 3) & 0xFE00000ull)) &
                     ((1ull << (7u * k2)) - 1ull);
  vo = ke + used + 1u + k2;
  return vo <= pl && v == (uint64_t)(pl - vo) && vo < 0x10000u;
}

// The record of the delivered frame whose header is at tile-relative offset o (id from its node;
// tailb: a blob cut by the stream end). w32: the tile's first byte; bytes up to se_rel are readable.
// false: the frame is not in the record's shape (the tile takes the wire-reading emission).
__device__ __forceinline__ bool crec_frame(const uint32_t *w32, uint32_t o, uint32_t se_rel, uint32_t id, bool tailb,
                                           uint32_t (&w)[CR_WORDS]) {
  const uint32_t d = o >> 2, sh = (o & 3u) * 8u;
  const uint32_t a0 = w32[d], a1 = w32[d + 1], a2 = w32[d + 2];
  const uint32_t h = __builtin_amdgcn_alignbit(a1, a0, sh), hn = __builtin_amdgcn_alignbit(a2, a1, sh);
  const uint32_t k = ((uint32_t)__builtin_ctz((~h & 0x808080u) | 0x80000000u) >> 3) + 1u;
  const uint32_t L = ((h & 0x7Fu) | ((h >> 1) & 0x3F80u) | ((h >> 2) & 0x1FC000u)) & ((1u << (7u * k)) - 1u);
  const uint32_t po = o + k + 1u, pl = L - 1u;
  w[0] = po | (id << 14) | ((tailb ? 1u : 0u) << 16);
  w[1] = pl;
  w[2] = w[3] = w[4] = w[5] = 0;
  if (id != 1u) return true;
  const uint64_t x = (((uint64_t)hn << 32) | h) >> (8u * (k + 1u));  // payload bytes 0 .. 6 - k
  const uint32_t b1 = (uint32_t)(x >> 8) & 0xFFu, b2 = (uint32_t)(x >> 16) & 0xFFu;
  const uint32_t kb = b1 < 0x80u ? 1u : (b2 < 0x80u ? 2u : 0u);
  const uint32_t klen = kb == 1u ? b1 : (b1 & 0x7Fu) | (b2 << 7);
  const uint32_t ke = 1u + kb + klen;  // the key's end, payload-relative
  uint32_t n0 = 0, n1 = 0, n2 = 0, vo = 0;
  bool hv = false, ok = ((uint32_t)x & 0xFFu) == 0x12u && kb && ke + 6u <= pl;
  const uint32_t qa = po + ke;
  ok = ok && qa + 36u <= se_rel;  // (the general form's 8 dwords from qa & ~3)
  if (ok) {
    const uint32_t e = qa >> 2, s2 = (qa & 3u) * 8u;
    const uint32_t c0 = w32[e], c1 = w32[e + 1], c2 = w32[e + 2], c3 = w32[e + 3];
    const uint64_t y = (uint64_t)__builtin_amdgcn_alignbit(c1, c0, s2) | ((uint64_t)__builtin_amdgcn_alignbit(c2, c1, s2) << 32);
    const uint32_t y8 = __builtin_amdgcn_alignbit(c3, c2, s2) & 0xFFu;
    // one-byte change / from / to: 18 a 20 b 28 c, then [32 d (d1)] or the payload's end
    const bool one = (y & 0xFFull) == 0x18u && ((y >> 16) & 0xFFull) == 0x20u && ((y >> 32) & 0xFFull) == 0x28u &&
                     (y & 0x0000800080008000ull) == 0;
    if (one) {
      n0 = (uint32_t)(y >> 8) & 0xFFu;
      n1 = (uint32_t)(y >> 24) & 0xFFu;
      n2 = (uint32_t)(y >> 40) & 0xFFu;
      if (ke + 6u != pl) {
        const uint32_t d0 = (uint32_t)(y >> 56), vh = d0 < 0x80u ? 2u : (y8 < 0x80u ? 3u : 0u);
        const uint32_t vl = vh == 2u ? d0 : (d0 & 0x7Fu) | (y8 << 7);
        vo = ke + 6u + vh;
        hv = true;
        ok = ((uint32_t)(y >> 48) & 0xFFu) == 0x32u && vh && vo <= pl && vl == pl - vo && vo < 0x10000u;
      }
    } else {
      ok = crec_general(w32, qa, ke, pl, n0, n1, n2, vo, hv);
    }
  }
  w[0] |= ((hv ? 1u : 0u) << 17) | (kb << 18);
  w[2] = klen | (vo << 16);
  w[3] = n0;
  w[4] = n1;
  w[5] = n2;
  return ok;
}

// Records of the tile's delivered frames (after the claim; whole workgroup). E / nf: this thread's
// settled entry and frame count (0 for a non-carrier), exactly as its per-thread record has them.
// v / hv: this thread's 64 bytes of the tile and (threads < HALO / 16) 16 bytes of the halo, still
// in the registers of the tile load: they become an LDS image of the tile (over the node tables,
// dead once the frames are listed), so the field decode reads no memory (re-reading the tile from
// the batch at this point, long after its load, cost claims_fast ~135 B per frame of fabric reads).
__device__ __forceinline__ void fast_records(const DecodeParams &P, uint64_t t, FastLds &S, uint32_t E, uint32_t nf,
                                             uint32_t s1r, uint32_t se_rel, const uint4 (&v)[SEGB / 16],
                                             const uint4 &hv) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  const uint32_t ip = wave_scan_dpp(nf);
  if (lane == 63) S.xw[4 + wid] = ip;
  bsync();
  const uint32_t tot = NT == 2 * WAVE ? S.xw[4] + S.xw[5] : S.xw[4];
  if (tot > CR_CAP) return;  // (uniform: tile_rec stays REC_NONE)
  uint32_t bad = 0;
  if (nf) {  // this thread's frames in chain order, as fwalk counts them
    uint32_t slot = ip - nf + (wid ? S.xw[4] : 0u), cnt = 0, i = E & 0xFFFFu;
#pragma unroll 1
    for (uint32_t g = 0; g < 64u; g++) {
      const uint32_t nd = S.lnd[i], id = nd >> 30, c = nd & 0xFFFFu, q = (nd >> 16) & 0x3FFFu;
      if (id == 3u || c == NX_TAILC) break;
      if (id != 0u) {
        if (cnt < nf) S.fls[slot + cnt] = (uint32_t)S.lpos[i] | (id << 14) | ((c == NX_TAILB ? 1u : 0u) << 16);
        cnt++;
      }
      if (c >= NX_TAILB || q >= s1r) break;  // (NX_TAILB, NX_TAILC, NX_NEAR, NX_FAR, NX_DEAD)
      i = c;
    }
    bad = cnt != nf;
  }
  bsync();  // (the node tables are dead: the image goes over them)
  if (DRP_CREC_STAGE == 0) return;
  uint4 *im = reinterpret_cast<uint4 *>(S.img);
#pragma unroll
  for (uint32_t k = 0; k < SEGB / 16; k++) im[tid * (SEGB / 16) + k] = v[k];
  if (tid < HALO / 16) im[TILE / 16 + tid] = hv;
  if (tid < 2) im[IMG / 16 + tid] = make_uint4(0, 0, 0, 0);  // (the slack: no stale bytes)
  bsync();
  if (tid < tot && !bad) {
    const uint32_t f = S.fls[tid];
    uint32_t w[CR_WORDS];
    bad = !crec_frame(reinterpret_cast<const uint32_t *>(S.img), f & 0x3FFFu, min(se_rel, IMG), (f >> 14) & 3u,
                      (f >> 16) & 1u, w);
    uint32_t *rr = P.rec + t * CR_TILE_WORDS + tid;
    if (DRP_CREC_STAGE == 1) {  // (A/B: keep the decode, store nothing)
      if ((w[0] ^ w[2] ^ w[3] ^ w[4] ^ w[5]) == 0x7FFFFFFFu && !bad) rr[0] = w[1];
      bad = true;
    }
    if (!bad) {
      rr[0] = w[0];
      rr[CR_CAP] = w[1];
      if ((w[0] >> 14 & 3u) == 1u) {
#pragma unroll
        for (uint32_t k = 2; k < CR_WORDS; k++) rr[k * CR_CAP] = w[k];
      }
    }
  }
  const uint64_t bm = __ballot(bad);
  if (lane == 0) S.xw[6 + wid] = bm != 0;
  bsync();
  if (tid == 0) P.tile_rec[t] = (NT == 2 * WAVE ? S.xw[6] | S.xw[7] : S.xw[6]) ? REC_NONE : 0u;
}

// bits of the 64 positions from base (tile-relative) that lie in [lo, hi)
__device__ __forceinline__ uint64_t range_bits(uint32_t base, uint32_t lo, uint32_t hi) {
  const uint32_t a = lo > base ? min(lo - base, 64u) : 0u, z = hi > base ? min(hi - base, 64u) : 0u;
  const uint64_t za = z >= 64u ? ~0ull : ((1ull << z) - 1ull), aa = a >= 64u ? ~0ull : ((1ull << a) - 1ull);
  return za & ~aa;
}

// The fast claims of interior tile t: writes the per-thread records (P.ent*) and P.claim[t], and
// returns this thread's record (eb, en, ecn) and, in thread NT - 1, the claim. FC_DENSE: more than
// FCAP live positions (the tile went to the general kernel's work list; nothing written).
// EDGE: a stream-edge tile (the stream starts after A, or ends before A + IMG), run from
// spec_claims' list: loads bounds-checked at the batch end, live positions only in [e0, se) (the
// stream's exact entry on, its end before), the last 3 positions before se always listed and
// every header whose 16-byte window crosses se parsed by the exact grammar (a header cut by the
// stream end is a tail, as parse_win has it); FC_DENSE lists nothing (the caller goes on).
template <bool CF, bool EDGE, bool REC>
__device__ __forceinline__ uint32_t fast_claims(const DecodeParams &P, const TileGeo &G, uint64_t t, FastLds &S,
                                                uint32_t &eb_o, uint32_t &en_o, uint32_t &ecn_o, uint64_t &cl_o) {
  uint8_t *buf = nullptr;
  uint64_t *lmw = S.lmw, *dmw = S.dmw, *xm = S.xm;
  uint16_t *loff = S.loff, *lpos = S.lpos;
  uint32_t *hmx = S.hmx, *lnd = S.lnd, *xw = S.xw, *xf = S.xf, *wl = S.wl, *fl = S.fl;
  uint8_t *lal = S.lal;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  // ---- stage, masks, live positions (varints of 1..3 bytes) --------------------------------
  uint4 v[SEGB / 16], hv;
  if (EDGE) {
    load_image(P, G, v, hv);  // (bounds-checked near the batch end)
  } else {
    const uint4 *q = reinterpret_cast<const uint4 *>(P.bytes + G.A + (uint64_t)tid * SEGB);
#pragma unroll
    for (int k = 0; k < (int)(SEGB / 16); k++) v[k] = q[k];
    hv = tid < HALO / 16 ? *reinterpret_cast<const uint4 *>(P.bytes + G.A + TILE + tid * 16) : make_uint4(0, 0, 0, 0);
  }
  uint32_t mk[4];
#pragma unroll
  for (int k = 0; k < 4; k++) mk[k] = masks16(v[k]);
  uint32_t *mx = lnd;  // next-16-byte masks of every thread (thread NT-1: the halo's first bytes)
  mx[tid] = mk[0];
  if (tid < HALO / 16) {
    const uint32_t hmk = masks16(hv);
    hmx[tid] = hmk;
    if (tid == 0) mx[NT] = hmk;
  }
  if (tid == HALO / 16) hmx[HALO / 16] = 0xFFFFu;  // (past the image: no terminators)
  bsync();
  const uint32_t nx = mx[tid + 1];
  const uint64_t M0 = (uint64_t)(mk[0] & 0xFFFFu) | ((uint64_t)(mk[1] & 0xFFFFu) << 16) |
                      ((uint64_t)(mk[2] & 0xFFFFu) << 32) | ((uint64_t)(mk[3] & 0xFFFFu) << 48);
  const uint64_t S0 = (uint64_t)(mk[0] >> 16) | ((uint64_t)(mk[1] >> 16) << 16) | ((uint64_t)(mk[2] >> 16) << 32) |
                      ((uint64_t)(mk[3] >> 16) << 48);
  const uint64_t M1 = nx & 0xFFFFu, S1 = nx >> 16;
  const uint64_t X0 = ~M0 & ((S0 >> 1) | (S1 << 63));  // varint terminator followed by an id <= 2
  const uint64_t X1 = ~M1 & (S1 >> 1);
  const uint64_t Xs1 = (X0 >> 1) | (X1 << 63), Xs2 = (X0 >> 2) | (X1 << 62), Ms1 = (M0 >> 1) | (M1 << 63);
  uint64_t live = X0 | (M0 & (Xs1 | (Ms1 & Xs2)));
  // (edge tiles) the stream's positions [lo_rel, hi_rel) only; the last 3 before its end always
  uint32_t lo_rel = 0, hi_rel = IMG, fo_rel = IMG;
  if (EDGE) {
    lo_rel = G.e0 > G.A ? (uint32_t)umin64(G.e0 - G.A, IMG) : 0u;
    hi_rel = (uint32_t)umin64(G.se - G.A, IMG);
    fo_rel = hi_rel < IMG ? max(lo_rel, hi_rel >= 3u ? hi_rel - 3u : 0u) : IMG;
    live = (live & range_bits(tid * SEGB, lo_rel, hi_rel)) | range_bits(tid * SEGB, fo_rel, hi_rel);
  }
  // Halo nodes (DRP_HALO_NODES): the halo's live positions join the list as HV more "threads", so
  // the survival check of the tile's last frames does not stop at the tile end (their chains
  // would otherwise leave the list within KSTRONG frames and stay undecided, and the link would
  // reach their threads one round at a time). Lanes 0..HV-1 of wave 0 build their masks.
  uint64_t hlive = 0;
  if (tid < HV) {
    uint32_t hk[5];
#pragma unroll
    for (int k = 0; k < 5; k++) hk[k] = hmx[tid * 4 + k];
    const uint64_t hM0 = (uint64_t)(hk[0] & 0xFFFFu) | ((uint64_t)(hk[1] & 0xFFFFu) << 16) |
                         ((uint64_t)(hk[2] & 0xFFFFu) << 32) | ((uint64_t)(hk[3] & 0xFFFFu) << 48);
    const uint64_t hS0 = (uint64_t)(hk[0] >> 16) | ((uint64_t)(hk[1] >> 16) << 16) | ((uint64_t)(hk[2] >> 16) << 32) |
                         ((uint64_t)(hk[3] >> 16) << 48);
    const uint64_t hM1 = hk[4] & 0xFFFFu, hS1 = hk[4] >> 16;
    const uint64_t hX0 = ~hM0 & ((hS0 >> 1) | (hS1 << 63)), hX1 = ~hM1 & (hS1 >> 1);
    const uint64_t hXs1 = (hX0 >> 1) | (hX1 << 63), hXs2 = (hX0 >> 2) | (hX1 << 62), hMs1 = (hM0 >> 1) | (hM1 << 63);
    hlive = hX0 | (hM0 & (hXs1 | (hMs1 & hXs2)));
    if (EDGE)
      hlive = (hlive & range_bits(TILE + tid * SEGB, lo_rel, hi_rel)) | range_bits(TILE + tid * SEGB, fo_rel, hi_rel);
    if (tid == HV - 1) hlive &= (1ull << (SEGB - 16)) - 1ull;  // (the image's last 16 bytes: no lookahead)
  }
  // ---- the tile's (and halo's) live positions as an LDS list -----------------------------------
  const uint32_t cnt = (uint32_t)__builtin_popcountll(live);
  const uint32_t cpre = wave_scan_dpp(cnt);
  const uint32_t hcnt = (uint32_t)__builtin_popcountll(hlive);
  uint32_t hpre = 0;
  if (wid == 0) hpre = wave_scan_dpp(hcnt);  // (the halo's threads are wave 0's: wave-uniform)
  if (lane == 63) xw[wid] = cpre;
  if (tid == 63) xw[2] = hpre;
  lmw[tid] = live;
  if (tid < HV) lmw[NT + tid] = hlive;
  bsync();  // (also: mx reads done)
  const uint32_t off = cpre - cnt + (wid ? xw[0] : 0u);
  const uint32_t ttotal = NT == 2 * WAVE ? xw[0] + xw[1] : xw[0];  // the tile's nodes
  const uint32_t total = ttotal + xw[2];
  if (total > FCAP) {  // very dense tile: the general kernel's per-thread checks
    if (!EDGE) push_work(P, t);
    return FC_DENSE;
  }
  loff[tid] = (uint16_t)off;
  {
    uint64_t bits = live;
    uint32_t i = off;
    while (bits) {
      lpos[i++] = (uint16_t)(tid * SEGB + (uint32_t)__builtin_ctzll(bits));
      bits &= bits - 1;
    }
  }
  if (tid < HV) {
    uint64_t bits = hlive;
    uint32_t i = ttotal + hpre - hcnt;
    loff[NT + tid] = (uint16_t)i;
    while (bits) {
      lpos[i++] = (uint16_t)(TILE + tid * SEGB + (uint32_t)__builtin_ctzll(bits));
      bits &= bits - 1;
    }
  }
  bsync();
  // ---- parse every node once --------------------------------------------------------------------
  const uint32_t se_rel = (uint32_t)umin64(G.se - G.A, 0x7FFFFFFFull);  // >= IMG
  constexpr uint32_t KPT = FCAP / NT;  // nodes per thread (at most)
  uint32_t ncode[KPT], npos[KPT];
  uint32_t na[KPT];
  uint32_t chained = 0;  // this thread's nodes whose successor is a node (in the image)
  uint32_t cfw[KPT];  // a Change frame leaving the image: payload offset | length << 14
  uint32_t cff[KPT];  // its first field's bytes | key seen << 20
  const uint32_t *w32 = reinterpret_cast<const uint32_t *>(P.bytes + G.A);  // (L2: the tile was just read)
#pragma unroll
  for (uint32_t j = 0; j < KPT; j++) {
    const uint32_t i = tid + j * NT;
    ncode[j] = NX_DEAD;
    na[j] = 0;
    npos[j] = 0;
    cfw[j] = 0;
    cff[j] = 0;
    if (i < total) {
      const uint32_t o = lpos[i];
      uint32_t w, wn, k, L, id, succ;
      bool valid, tail, exact = false;
      if (EDGE && o + 16u > se_rel) {  // (edge tiles) the window crosses the stream end: parse_win's grammar
        const Hdr h = hdr_global(P.bytes, G.A + o, G.se);
        exact = true;
        tail = h.kind == H_TAIL_HDR || h.kind == H_TAIL_CHANGE || h.kind == H_TAIL_BLOB;
        valid = h.kind == H_VALID || tail;
        id = h.kind == H_TAIL_HDR ? 1u : h.id;  // (a cut header delivers nothing, as a cut change frame)
        k = h.vlen;
        L = (uint32_t)umin64(h.L, 0xFFFFFFFFull);
        succ = h.kind == H_VALID ? (uint32_t)(h.succ - G.A) : o + 1u;
        w = wn = 0;
      } else {
        const uint32_t d = o >> 2, sh = (o & 3u) * 8u;
        const uint32_t a0 = w32[d], a1 = w32[d + 1], a2 = w32[d + 2];
        w = __builtin_amdgcn_alignbit(a1, a0, sh);
        wn = __builtin_amdgcn_alignbit(a2, a1, sh);
        const uint32_t tm = ~w & 0x808080u;  // live => a terminator in bytes 0..2
        k = ((uint32_t)__builtin_ctz(tm | 0x80000000u) >> 3) + 1u;
        const uint32_t L3 = (w & 0x7Fu) | ((w >> 1) & 0x3F80u) | ((w >> 2) & 0x1FC000u);
        L = L3 & ((1u << (7u * k)) - 1u);
        id = (w >> (8u * k)) & 0xFFu;
        succ = o + k + (id ? L : 1u);
        const uint32_t avail = se_rel - o;  // >= IMG - o (interior); > 0 (edge: o < se)
        valid = id <= 2u && (id == 0u || L != 0u);
        tail = valid && id != 0u && L > avail - k;
      }
      uint32_t c = NX_DEAD, a = 0;
      if (valid && !tail && !exact && id == 1u && k >= 2u && succ <= IMG) {  // Change field tag first
        const uint32_t pb = k == 3u ? (wn & 0xFFu) : (w >> (8u * (k + 1u))) & 0xFFu;
        constexpr uint64_t TAGS = (1ull << 0x0a) | (1ull << 0x12) | (1ull << 0x18) | (1ull << 0x20) | (1ull << 0x28) |
                                  (1ull << 0x32);
        valid = pb < 64u && ((TAGS >> pb) & 1ull);
      }
      if (!valid) {
        c = NX_DEAD;
      } else if (tail) {
        c = id == 2u ? NX_TAILB : NX_TAILC;
      } else if (succ >= se_rel) {
        c = NX_NEAR;  // ends at the stream end: survived
        a = 1;
        S.lsucc[i] = succ;
      } else if (succ >= IMG - 16) {
        c = NX_FAR;   // past the listed positions: undecided (a restart that needs it checks in HBM),
        a = 2;        // unless it is a Change frame whose fields fill it exactly (below)
        S.lsucc[i] = succ;
        // (halo nodes: only frames longer than the halo, so C2's short frames there never pay for
        // it; C5's long ones do, so a tile's last real frame is not left undecided by its successor)
        // The first field is checked here from the header's own bytes (no load): subset or key
        // (protocol-buffers writes fields in schema order), a length of <= 3 bytes, inside the
        // payload. ~99% of shadow headers stop here, so change_fills' loads are rare on C2.
        if (CF && id == 1u && (o < TILE || L > HALO) && L - 1u < (1u << 18)) {
          const uint32_t x = k + 1u < 4u ? __builtin_amdgcn_alignbit(wn, w, 8u * (k + 1u)) : wn;  // bytes k+1..k+4
          const uint32_t tg = x & 0xFFu, lt = ~(x >> 8) & 0x808080u;
          if ((tg == 0x0Au || tg == 0x12u) && lt) {
            const uint32_t nb = ((uint32_t)__builtin_ctz(lt) >> 3) + 1u, y = x >> 8;
            const uint32_t v = ((y & 0x7Fu) | ((y >> 1) & 0x3F80u) | ((y >> 2) & 0x1FC000u)) & ((1u << (7u * nb)) - 1u);
            const uint32_t f1 = 1u + nb + v;  // the first field's bytes
            if (f1 < L - 1u) cfw[j] = (o + k + 1u) | ((L - 1u) << 14), cff[j] = f1 | ((tg == 0x12u ? 1u : 0u) << 20);
          }
        }
      } else {
        const uint32_t th = succ / SEGB, b = succ % SEGB;
        const uint64_t lw = lmw[th];
        if ((lw >> b) & 1ull) {
          c = loff[th] + (uint32_t)__builtin_popcountll(lw & ((1ull << b) - 1ull));
          a = 1;
        }
      }
      lnd[i] = c | (min(succ, 0x3FFFu) << 16) | ((valid ? id : 3u) << 30);
      lal[i] = (uint8_t)a;
      ncode[j] = c;
      na[j] = a;
      npos[j] = o;
      chained += c < NX_TAILB;
    }
  }
  // Change frames that leave the image are strong by structure when their fields fill them
  // exactly (change_fills). A loop of its own after the parse: inside it, its dependent loads kept
  // the parse's loads of later nodes from being issued together (C2: claims 2.8 -> 5.2 ms). Only
  // a wave whose bytes chain few frames inside the image runs it (C5: two real frames per tile,
  // their chains leave the image; C2: ~47 per wave, predicted without it).
  if (CF && wave_sum_dpp(chained) < 16u) {
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++) {
      // (field headers may lie past the image, up to 512 bytes: a halo frame's key runs past it;
      // w32 reads the batch, which holds them: interior tiles end >= IMG before the stream end)
      uint32_t cr = 0;
      if (cfw[j]) {
        // (the LDS-image build reads its IMG + 32 bytes only; the default reads the batch)
        const uint32_t lim = min(se_rel, IMG + 512u), po = cfw[j] & 0x3FFFu,
                       pl = cfw[j] >> 14;
        cr = change_fills_win(w32, po, pl, lim, cff[j] & 0xFFFFFu, cff[j] >> 20);
        if (cr == 2u) cr = change_fills(w32, po, pl, lim, cff[j] & 0xFFFFFu, cff[j] >> 20) ? 1u : 0u;
      }
      if (cr == 1u) {
        na[j] = 1;
        lal[tid + j * NT] = 1;
      }
    }
  }
  bsync();
  lmw[tid] = 0;  // (now the strong masks)
  dmw[tid] = 0;
  // ---- survival: KSTRONG - 1 rounds propagate death / undecided back along the chains ------------
#pragma unroll 1
  for (int r = 1; r < KSTRONG; r++) {
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++) {
      if (na[j] == 1u && ncode[j] < NX_NEAR) {
        const uint32_t b = lal[ncode[j]];
        if (b != 1u) {
          na[j] = b;
          lal[tid + j * NT] = (uint8_t)b;
        }
      }
    }
    bsync();
  }
#pragma unroll
  for (uint32_t j = 0; j < KPT; j++) {
    if (na[j] && npos[j] < TILE) {
      const uint32_t o = npos[j];
      atomicOr((unsigned long long *)(na[j] == 1u ? &lmw[o / SEGB] : &dmw[o / SEGB]), 1ull << (o % SEGB));
    }
  }
  bsync();
  // ---- this thread's strong candidate g (the first strong node of its bytes) -------------------
  const uint64_t sm = lmw[tid];
  const uint32_t lb = tid * SEGB, s1r = lb + SEGB;
  uint32_t g = RX_NONE;
  uint64_t defer = dmw[tid];
  bool far = false;
  if (sm) {
    const uint32_t b = (uint32_t)__builtin_ctzll(sm);
    defer &= (1ull << b) - 1ull;
    const uint32_t gi = off + (uint32_t)__builtin_popcountll(live & ((1ull << b) - 1ull));
    g = gi | ((lb + b) << 16);
    const uint32_t gc = lnd[gi] & 0xFFFFu;
    far = gc == NX_FAR || gc == NX_NEAR;
  }
  uint32_t n = 0, R = RX_NONE;
  if (g != RX_NONE) R = fwalk(lnd, g, s1r, n);
  // rule 2: a chain that starts by jumping past the tile only where nothing later can start one
  uint64_t S0m, S1m;
  {
    const uint64_t hm = __ballot(g != RX_NONE), fm = __ballot(g != RX_NONE && far);
    uint64_t H0 = hm, H1 = 0, F0 = fm, F1 = 0;  // one wave: its own ballots are the tile's masks
    if constexpr (NT == 2 * WAVE) {
      if (lane == 0) {
        xm[wid] = hm;
        xm[2 + wid] = fm;
      }
      bsync();
      H0 = xm[0];
      H1 = xm[1];
      F0 = xm[2];
      F1 = xm[3];
    }
    const uint64_t L1 = H1 ? ((1ull << (63 - __builtin_clzll(H1))) - 1) : 0ull;  // below the top bit
    const uint64_t L0 = H1 ? ~0ull : (H0 ? ((1ull << (63 - __builtin_clzll(H0))) - 1) : 0ull);
    S0m = H0 & ~(F0 & L0);
    S1m = H1 & ~(F1 & L1);
    if (far && any_above(H0, H1, tid)) {
      g = RX_NONE;
      R = RX_NONE;
      n = 0;
    }
  }
  uint32_t E = g;
  bool rs = false;
  if (flink(lnd, s1r, g, E, R, n, rs, wl, fl, P.overflow, P.stats, DRP_FL_CAP)) {
    // the rounds did not settle: past P.jump_min such tiles in this launch (an input with a second
    // framing throughout: every tile), pointer jumping; before it (clean streams have a few, whose
    // predictions rely on the restarts and rule 3 below), the rounds go on
    // (an atomic only below the threshold: one word takes ~88 atomics per us, and on a cascade
    // every tile gets here)
    if (tid == 0) {
      uint32_t c = __hip_atomic_load(&P.counter[12], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (c < P.jump_min) c = atomicAdd(&P.counter[12], 1u);
      xw[6] = c;
    }
    bsync();
    if (xw[6] >= P.jump_min) return fast_claims_jump<NT>(P, t, G.A, S, g, ttotal, total, eb_o, en_o, ecn_o, cl_o);
    flink(lnd, s1r, g, E, R, n, rs, wl, fl, P.overflow, P.stats);
  }
  // restarts from deferred candidates, decided in HBM (big frames), as in spec_claims
  const Img m{buf, P.bytes, G.A, G.se, false};
  uint32_t need, js;  // a thread needs a restart; the last carrier + 1
  block_any_last(E == RX_NONE && defer && !any_above(S0m, S1m, tid), rx_node(E) && rx_off(E) < s1r, need, js, xf);
  bool moved = false;
  if (P.stats && tid == 0 && need) atomicAdd(&P.stats[59], 1ull);  // (DRP_STATS: tiles with restarts)
#pragma unroll 1
  for (uint32_t it = 0; need && it < 3; it++) {
    moved = true;
    if (E == RX_NONE && defer && !any_above(S0m, S1m, tid)) {
      while (defer) {
        const uint32_t o = (uint32_t)__builtin_ctzll(defer);
        defer &= defer - 1;
        uint64_t r;
        uint32_t k;
        bool f;
        if (strong<false>(m, G.A + lb + o, G.A + s1r, r, k, f, P.kstrong_hbm) == S_OK) {
          g = (off + (uint32_t)__builtin_popcountll(live & ((1ull << o) - 1ull))) | ((lb + o) << 16);
          E = g;
          R = fwalk(lnd, g, s1r, n);
          break;
        }
      }
    }
    flink(lnd, s1r, g, E, R, n, rs, wl, fl, P.overflow);
    block_any_last(E == RX_NONE && defer && !any_above(S0m, S1m, tid), rx_node(E) && rx_off(E) < s1r, need, js,
                   xf);
  }
  // rule 3: the chain's last frame may jump over threads holding strong candidates; keep the
  // chain they start when it is the denser one (>= 2 frames)
  {
    bool after;
    if (!moved) after = any_from(S0m, S1m, js);
    else after = block_max_u32(g != RX_NONE && tid + 1 > js ? 1u : 0u, xf) != 0;
    if (js && after) {
      const uint32_t Ea = E, Ra = R, na0 = n;
      const bool rsa = rs;
      const bool mine = tid + 1 > js;
      E = RX_NONE;
      R = RX_NONE;
      n = 0;
      flink(lnd, s1r, mine ? g : RX_NONE, E, R, n, rs, wl, fl, P.overflow);
      const uint32_t nb = block_sum_u32(mine ? (n & 0xFFFFu) : 0u, xf);
      if (nb < 2 || !mine) {
        E = Ea;
        R = Ra;
        n = na0;
        rs = rsa;
      }
    }
  }
  // per-thread records for kernel 2 (as spec_claims) and the claim
  {
    const bool carrier = rx_node(E) && rx_off(E) < s1r;
    const uint64_t ix = t * NT + tid;
    eb_o = carrier ? (((rx_off(E) - lb) & 63u) | (rs ? 0x40u : 0u)) : 0xFFu;
    en_o = carrier ? (n & 0xFFFFu) : 0u;
    ecn_o = carrier ? (n >> 16) : 0u;
    P.ent[ix] = (uint8_t)eb_o;
    P.ent_n[ix] = (uint8_t)en_o;
    P.ent_c[ix] = (uint8_t)ecn_o;
  }
  cl_o = 0;
  if (tid == NT - 1) {
    uint64_t cl = C_ID;
    if (R < RX_DEAD && !rx_node(R)) {
      const uint64_t p = G.A + lpos[R & 0xFFFFu];
      if (R & RX_FAR) {
        cl = G.A + S.lsucc[R & 0xFFFFu];  // (the node's header is valid: fwalk gives RX_FAR for NX_FAR / NX_NEAR)
      } else {
        cl = MARK_TERM | p;  // a tail ends the chain
      }
    } else if (rx_node(R)) {
      cl = G.A + rx_off(R);
    }
    P.claim[t] = cl;
    cl_o = cl;
  }
  if (!EDGE && REC) fast_records(P, t, S, E, en_o, s1r, se_rel, v, hv);
  return FC_OK;
}

// CF: with the structural check of frames that leave the image (long frames, C5). Picked per
// launch: the host takes it for a context whose last decode averaged >= 512 bytes per frame (and
// for its first), and large batches take the hop walkers instead when walk_density's sample says
// the stream is sparse; dense streams (C2) are predicted as well without it, and its code costs
// them ~4% (DESIGN.md "Long frames").
#ifndef DRP_K1_REC_WAVES
#define DRP_K1_REC_WAVES 7  // min waves per SIMD for claims_fast with records (the tile's registers live to the end)
#endif
template <bool CF, bool REC>
__global__ __launch_bounds__(NT, REC ? DRP_K1_REC_WAVES : DRP_K1_WAVES) void claims_fast(DecodeParams P) {
  __shared__ FastLds S;
  const uint64_t ntiles = P.tile_prefix[P.nstreams];
  const uint64_t t = blockIdx.x;
  if (REC && t == 0 && threadIdx.x == 0) P.counter[13] = 1u;  // (records may exist: emit_recs runs)
  const TileGeo G = tile_geo(P, t);
  if (t >= ntiles) return;  // (whole workgroup)
  if (G.A < G.so || G.A + IMG > G.se) {  // edge tile: the general kernel
    push_work(P, t);
    return;
  }
  uint32_t eb, en, ecn;
  uint64_t cl;
  (void)fast_claims<CF, false, REC>(P, G, t, S, eb, en, ecn, cl);
}

// ==== kernel 2: exact entries, verification, frame counts =====================================
// e_t = the nearest claim before t that is not identity (or the stream entry); claims are final,
// so nothing here waits. Publishes incl_e[t] = e_{t+1} for kernel 3 and for later tiles.
// ==== kernel 2, records-only form (default): 8 lanes per tile, 32 tiles per workgroup ===========
// verify_counts' fast check from kernel 1's per-thread records alone: e_t from the previous claims
// (up to 32 identity claims back), thread k = the one holding e_t must have it as its predicted
// entry and no later thread may restart the chain; then the tile's counts are the sums of the
// records from thread k on (byte sums with v_dot4). Each lane holds 16 threads' records. A tile
// that does not pass (a re-walk is needed, a miss, a longer identity run) goes to a list that
// verify_counts then takes, so results are verify_counts' in every case. Threads before k are
// left to emit_tiles through tile_k (the records stay as kernel 1 wrote them).
#ifndef DRP_CASCADE_HARD
#define DRP_CASCADE_HARD 1  // (A/B: 0 counts every listed tile toward a cascade, as round 5 did)
#endif
constexpr uint32_t VL_HARD = 1u << 31;  // verify_lite's list entry: the tile's prediction failed
#ifndef DRP_CASCADE_DIV
#define DRP_CASCADE_DIV 8  // verify_counts hands the listed tiles to the segmented repair when more
#endif                     // than 1/8 of the tiles (and P.cascade_min) are listed (0: never)
constexpr uint32_t VL_BLK = 256, VL_G = NT / 16;  // lanes per tile (16 threads' records each)
#ifndef DRP_SP_FRAMES
#define DRP_SP_FRAMES 8  // frames of a sparse tile (0: no sparse emission)
#endif
constexpr uint32_t SP_FRAMES = DRP_SP_FRAMES;
__device__ __forceinline__ uint32_t bytes_from(uint32_t s, uint32_t d) {  // byte mask of dword d: index >= s
  return s <= 4u * d ? 0xFFFFFFFFu : (s >= 4u * d + 4u ? 0u : 0xFFFFFFFFu << (8u * (s - 4u * d)));
}
__device__ __forceinline__ uint32_t restart_bytes(uint32_t x) {  // 4-bit mask: byte b has (b & 0xC0) == 0x40
  const uint32_t y = (x & 0xC0C0C0C0u) ^ 0x40404040u;
  return msb4(~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u);
}
__global__ __launch_bounds__(VL_BLK) void verify_lite(DecodeParams P) {
  const uint32_t tid = threadIdx.x, r = tid & (VL_G - 1u), gb = (tid & 63u) & ~(VL_G - 1u);
  const uint64_t t = ((uint64_t)blockIdx.x * VL_BLK + tid) / VL_G;
  const uint64_t ntiles = P.tile_prefix[P.nstreams];
  if (t >= ntiles) return;  // (whole 8-lane group: no barriers or cross-group exchanges below)
  const TileGeo G = tile_geo(P, t);
  const uint64_t ix = t * NT + 16u * r;
  const uint4 e4 = *reinterpret_cast<const uint4 *>(P.ent + ix);
  const uint4 n4 = *reinterpret_cast<const uint4 *>(P.ent_n + ix);
  const uint4 c4 = *reinterpret_cast<const uint4 *>(P.ent_c + ix);
  const uint64_t claim = P.claim[t];
  uint64_t et = G.e0;
  bool found = t == G.tf;
  for (uint32_t step = 0; !found && step < 4u; step++) {
    const int64_t j = (int64_t)t - 1 - (int64_t)(VL_G * step + r);
    const bool virt = j < (int64_t)G.tf;
    const uint64_t c = virt ? G.e0 : P.claim[j];
    const uint32_t gm = (uint32_t)(__ballot(virt || c != C_ID) >> gb) & ((1u << VL_G) - 1u);
    if (gm) {
      const uint32_t src = gb + (uint32_t)__builtin_ctz(gm);
      et = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(c >> 32), (int)src, WAVE) << 32) |
           (uint32_t)__shfl((int)(uint32_t)c, (int)src, WAVE);
      found = true;
    }
  }
  const bool bogus = is_pos(et) && et < G.A;
  const bool inside = is_pos(et) && !bogus && et < G.A + TILE;
  const uint32_t k = inside ? (uint32_t)((et - G.A) / SEGB) : NT;
  const uint32_t kr = k / 16u, ki = k % 16u;
  const uint32_t ew[4] = {e4.x, e4.y, e4.z, e4.w}, nw[4] = {n4.x, n4.y, n4.z, n4.w}, cw[4] = {c4.x, c4.y, c4.z, c4.w};
  uint32_t bad = 0, sf = 0, sc = 0, rsm = 0, multi = 0, sb = 0;
  const uint32_t s = r > kr ? 0u : (r == kr ? ki : 16u);  // this lane's threads from k on
#pragma unroll
  for (uint32_t d = 0; d < 4; d++) {
    const uint32_t m = bytes_from(s, d);
    sf = __builtin_amdgcn_udot4(nw[d] & m, 0x01010101u, sf, false);
    sc = __builtin_amdgcn_udot4(cw[d] & m, 0x01010101u, sc, false);
    sb = __builtin_amdgcn_udot4(nw[d] & ~m, 0x01010101u, sb, false);  // (frames before e_t's thread)
    rsm |= restart_bytes(ew[d]) << (4u * d);
    multi |= nw[d] & m & 0xFEFEFEFEu;  // a thread from k on with more than one frame
  }
  if (inside) {
    if (r == kr) {
      const uint32_t b = (ew[ki >> 2] >> (8u * (ki & 3u))) & 0xFFu;
      bad = (b & 0x80u) || (b & 63u) != (uint32_t)((et - G.A) % SEGB) || (rsm >> ki) > 1u;
    } else if (r > kr) {
      bad = rsm != 0;
    }
  }
#pragma unroll
  for (uint32_t d = 1; d < VL_G; d <<= 1) {
    sf += shfl_xor32(sf, d);
    sc += shfl_xor32(sc, d);
    sb += shfl_xor32(sb, d);
    bad |= shfl_xor32(bad, d);
    multi |= shfl_xor32(multi, d);
  }
  const bool miss = !inside && !bogus && claim != C_ID && claim != et;
  // verify_counts decides the tiles listed here; one atomic per wave (a cascade lists every tile,
  // and one counter word takes ~88 atomics per us: 207K single appends cost 0.3 ms)
  const bool lst = r == 0 && (!found || bad || bogus || miss || (inside && claim == C_ID));
  // a listed tile a prediction failed on (every reason but !found: a tile deep inside a long
  // payload, more than 32 identity claims after the last frame start, only needs a longer
  // look-back) carries VL_HARD in its list entry; verify_counts decides a cascade from a sample of
  // the entries (no counter: one atomic per listing wave cost 0.2 ms on C2)
  // (!found: et is only the stream entry, so bogus and miss mean nothing there)
  const bool hard = DRP_CASCADE_HARD && found && (bad || bogus || miss || (inside && claim == C_ID));
  const uint64_t lm = __ballot(lst);
  if (lm) {
    const uint32_t lane = threadIdx.x & 63u, ld = (uint32_t)__builtin_ctzll(lm);
    uint32_t base = 0;
    if (lane == ld) base = atomicAdd(P.vlist_n, (uint32_t)__builtin_popcountll(lm));
    base = (uint32_t)__shfl((int)base, (int)ld, WAVE);
    if (lst) P.vlist[base + (uint32_t)__builtin_popcountll(lm & ((1ull << lane) - 1ull))] = (uint32_t)t | (hard ? VL_HARD : 0u);
  }
  if (r != 0 || lst) return;
  // the record emission takes the tile when the claims kernel recorded every frame its threads
  // deliver: the tile's rows are its records from slot sb on (sb = the frames of the threads before
  // e_t's), kept here as sb + 1
  const bool recok = P.tile_recok && inside && sb < 255u && P.tile_rec[t] != REC_NONE;
  if (P.tile_recok) P.tile_recok[t] = recok ? (uint8_t)(sb + 1u) : 0;
  P.tile_exit[t] = inside ? claim : et;
  P.tile_count[t] = sf;
  P.tile_nch[t] = sc;
  P.tile_k[t] = (uint8_t)k;
  if (P.tile_sparse) P.tile_sparse[t] = (!multi && sf <= SP_FRAMES && !recok) ? 1 : 0;
}

__global__ __launch_bounds__(NT) void verify_counts(DecodeParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[IMG + 32];
  __shared__ uint64_t xr[NT / WAVE];
  __shared__ uint32_t xf[NT / WAVE], xs[NT / WAVE];
  __shared__ uint64_t sh_e;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u, wid = tid >> 6;
  uint64_t tl_ = P.stats && tid == 0 ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t ntiles = P.tile_prefix[P.nstreams];
  // every tile (one per workgroup), or the tiles verify_lite listed (a few per workgroup)
  const uint32_t nwork = P.vlist ? *P.vlist_n : 0u;
  if (P.pass_id == 1 && P.vlist && !P.vlist_ovf && blockIdx.x == 0 && tid == 0)
    P.counter[14] = nwork;  // (the head's relisted tiles, for drp_timing.verify_relisted)
  if (P.vlist_ovf && (*P.vlist_ovf || nwork > P.dlist_cap)) {  // an incomplete dirty list: the host
    if (blockIdx.x == 0 && tid == 0) {                          // runs a full pass next
      atomicOr(P.dlist_n + 2, 1u);
      atomicOr(P.overflow, F_MISS);
    }
    return;
  }
  // A cascade: verify_lite listed more than 1 / DRP_CASCADE_DIV of the tiles as failed predictions
  // (and at least P.cascade_min, 4096 unless DRP_CASCADE_MIN says otherwise; tiles listed only for
  // a longer look-back do not count: C3's 1 MiB blobs list ~90% of the tiles that way, and taking
  // them for a cascade cost a segmented repair, 110 ms per 0.34 GB), i.e. the prediction followed a
  // second framing through the stream (tests/_streams.shadow_stream). Re-walking every listed tile only to find them missed costs
  // as much as the segmented repair that follows (1.7 GB dense cascade: 2.4 of 11.7 ms), so the
  // list goes to that repair directly: each stream's first listed tile in first_miss (every tile
  // before it passed the records-only proof, so its entry is exact) and F_CASCADE for the host.
  // Only in the head's pass (pass_id 1).
  // (the share of failed predictions among the listed tiles, from 64 entries spread over the list:
  // every workgroup reads the same sample and takes the same decision)
  bool cascade = DRP_CASCADE_DIV && P.pass_id == 1 && P.vlist && !P.vlist_ovf && nwork >= P.cascade_min &&
                 (uint64_t)nwork * DRP_CASCADE_DIV > ntiles;
  if (cascade && DRP_CASCADE_HARD) {
    const uint32_t e = P.vlist[(uint64_t)nwork * lane / WAVE];
    const uint32_t nh = (uint32_t)__builtin_popcountll(__ballot(wid == 0 && (e & VL_HARD)));
    if (wid == 0 && lane == 0) xs[0] = nh;
    bsync();
    // the hard entries extrapolated: a cascade when they alone are over the threshold
    cascade = (uint64_t)nwork * xs[0] / WAVE >= P.cascade_min && (uint64_t)nwork * xs[0] / WAVE * DRP_CASCADE_DIV > ntiles;
    bsync();
  }
  if (cascade) {
    // one stream: a wave minimum, one atomic per wave; several: one atomic per listed tile
    uint32_t tmin = ~0u;
    for (uint32_t wi = blockIdx.x * NT + tid; wi < nwork; wi += gridDim.x * NT) {
      const uint32_t t = P.vlist[wi] & ~VL_HARD;
      if (P.nstreams == 1) tmin = min(tmin, t);
      else atomicMin((unsigned long long *)&P.first_miss[P.tile_stream[t]], (unsigned long long)t);
    }
    if (P.nstreams == 1) {
      tmin = wave_min_dpp(tmin);
      if (lane == 0 && tmin != ~0u) atomicMin((unsigned long long *)&P.first_miss[0], (unsigned long long)tmin);
    }
    if (blockIdx.x == 0 && tid == 0) atomicOr(P.overflow, F_MISS | F_CASCADE);
    return;
  }
  for (uint32_t wi = blockIdx.x; P.vlist ? wi < nwork : wi == blockIdx.x; wi += gridDim.x) {
  const uint64_t t = P.vlist ? P.vlist[wi] & ~VL_HARD : wi;
  bsync();  // the previous tile's LDS reads are done
  const TileGeo G = tile_geo(P, t);  // (its loads go out with the tile count's)
  if (t >= ntiles) continue;  // (whole workgroup)
  const uint64_t lb = G.A + (uint64_t)tid * SEGB, s1 = lb + SEGB;
  // every load this tile needs goes out first (their latencies overlap)
  const uint64_t ix = t * NT + tid;
  const uint8_t eb = P.ent[ix];
  const uint8_t en = P.ent_n[ix], ecn = P.ent_c[ix];
  const uint64_t claim = P.claim[t];
  const uint64_t cprev = t != G.tf ? P.claim[t - 1] : C_ID;
  PHASE(8);
  if (t != G.tf && cprev != C_ID) {
    // the common case: the previous tile's claim is its exit (a published incl_e of a
    // non-identity tile always equals its claim), so e_t needs no look-back
    if (tid == 0) sh_e = cprev;
  } else if (wid == 0) {
    uint64_t e = G.e0;
    if (t != G.tf) {
      int64_t j0 = (int64_t)t - 1;
      for (;;) {
        const int64_t j = j0 - (int64_t)lane;
        const bool virt = j < (int64_t)G.tf;
        uint64_t ie = 0, cl = C_ID;
        if (!virt) {
          ie = ld_agent(&P.incl_e[j]);
          if (!ie) cl = P.claim[j];
        }
        const uint64_t sm = __ballot(virt || ie || cl != C_ID);
        if (sm) {
          const uint32_t k = (uint32_t)__builtin_ctzll(sm);
          e = readlane64(virt ? G.e0 : (ie ? (ie & ~RDY) : cl), k);
          if (lane < k) st_agent(&P.incl_e[j], e | RDY);  // helping: identity tiles pass e on
          break;
        }
        j0 -= WAVE;  // 64 identity claims: keep looking back
      }
    }
    if (lane == 0) sh_e = e;
  }
  bsync();
  const uint64_t et = sh_e;
  if (tid == NT - 1) st_agent(&P.incl_e[t], (claim == C_ID ? et : claim) | RDY);
  PHASE(9);
  // Fast check from kernel 1's per-thread records (no tile bytes): when the thread holding e_t
  // has e_t as its predicted entry and no later thread restarted the predicted chain, the
  // walks from there on are the exact walks (same entries, and no prediction-only deaths), so
  // the predicted entries, counts and exit are exact.
  // e_t < A: an identity-claimed tile before this one passed on an entry that lies inside it. That
  // tile misses (an identity claim never verifies on its own entry) and is repaired, so this pass
  // proves nothing here: no miss, no repair of this tile's claim (it is re-verified next pass).
  const bool bogus = is_pos(et) && et < G.A;
  const bool inside = is_pos(et) && !bogus && et < G.A + TILE;
  const uint32_t k = inside ? (uint32_t)((et - G.A) / SEGB) : NT;
  uint32_t bad = 0;
  if (inside) {
    if (tid == k && ((eb & 0x80) || (eb & 63) != (uint32_t)((et - G.A) % SEGB))) bad = 1;
    if (tid > k && eb != 0xFF && (eb & 0x40)) bad = 1;
    if (claim == C_ID) bad = 1;
  }
  // one exchange: any thread disagrees (max), and the fast path's frame and change counts
  const bool mine = tid >= k && eb != 0xFF;
  uint32_t cnt_f = mine ? en : 0u, cnt_c = mine ? ecn : 0u;
  {
    cnt_f = wave_sum32(cnt_f);
    cnt_c = wave_sum32(cnt_c);
#pragma unroll
    for (uint32_t d = 1; d < WAVE; d <<= 1) bad = max(bad, shfl_xor32(bad, d));
    if (lane == 0) {
      xr[wid] = ((uint64_t)cnt_c << 32) | cnt_f;
      xf[wid] = bad;
    }
    bsync();
    uint64_t acc = 0;
    uint32_t b = 0;
#pragma unroll
    for (uint32_t w = 0; w < NT / WAVE; w++) {
      acc += xr[w];
      b = max(b, xf[w]);
    }
    bsync();
    cnt_f = (uint32_t)acc;
    cnt_c = (uint32_t)(acc >> 32);
    bad = b;
  }
  const bool fast = !bad;
  uint32_t count_t, nch_t;
  uint64_t exit_t;
  bool miss;
  if (fast) {
    count_t = cnt_f;
    nch_t = cnt_c;
    if (tid < k) {
      P.ent[ix] = 0xFF;
      P.ent_n[ix] = 0;
    }
    exit_t = inside ? claim : et;  // pass-through tiles keep the entry
    miss = !inside && !bogus && claim != C_ID && claim != et;  // (a chain that rejoined the stream's one)
  } else {
    const uint64_t live = stage_live(P, G, buf);
    const Img m{buf, P.bytes, G.A, G.se};
    // the exact chain from e_t, seeded with the predicted chain's per-thread entries
    uint64_t E = !(eb & 0x80) ? lb + (eb & 63) : (live ? lb + (uint32_t)__builtin_ctzll(live) : NONE);
    uint32_t n = 0;
    uint64_t R = walk(m, E, s1, n);
    link<true>(m, s1, NONE, et, E, R, n, xr, xf, P.overflow);
    if (P.tile_rec && tid == 0) P.tile_rec[t] = REC_NONE;  // (the records below are not the claims kernel's)
    const bool carrier = is_pos(E) && E >= lb && E < s1 && E < G.se;  // (as spec_claims' records)
    P.ent[ix] = carrier ? (uint8_t)(E - lb) : (uint8_t)0xFF;  // exact, for kernel 3
    P.ent_n[ix] = carrier ? (uint8_t)(n & 0xFFFFu) : (uint8_t)0;
    P.ent_c[ix] = carrier ? (uint8_t)(n >> 16) : (uint8_t)0;  // (a repair pass may take the fast check)
    count_t = block_sum_u32(n & 0xFFFFu, xs);  // (xs: link's last reads of xf are not behind a barrier)
    nch_t = block_sum_u32(n >> 16, xs);
    // the last thread's R is the tile's exact exit; it must be what the claim predicted (an
    // error on the exact chain never is: predictions restart after errors)
    xr[0] = 0;
    bsync();
    if (tid == NT - 1) xr[0] = R;
    bsync();
    const uint64_t Rl = xr[0];
    exit_t = (Rl & MARK_TERM) ? (Rl & ~M_ERR) : Rl;
    const uint64_t want = claim == C_ID ? et : claim;
    // an error on the exact chain is a miss unless the claim already ends the chain there (a
    // repaired claim, or the segmented repair's): then the tile's exit is exact
    miss = exit_t != want || ((Rl & MARK_TERM) && (Rl & M_ERR) && claim != exit_t);
  }
  PHASE(10);
  if (tid == NT - 1) {
    // the stream's last tile: no later tile takes its claim as its entry (the next stream starts at
    // its own e0), so a miss there rewrites its claim in place instead of asking for a pass (a
    // stream cut mid-frame can end in a chain too short to be strong before its tail: the
    // prediction leaves that tile unclaimed). A later repair that changes its entry relists it.
    if (miss && t + 1 == P.tile_prefix[G.s + 1]) {
      P.claim[t] = inside ? exit_t : C_ID;
      miss = false;
    }
    if (miss) {
      atomicOr(P.overflow, F_MISS);
      // repair: the claim becomes the exit of the chain from this pass's entry. The first
      // missed tile's entry is exact (induction), so each verify pass fixes at least that tile;
      // the host re-runs verify until a pass has no miss (claims are only written on a miss,
      // so a miss-free pass saw a constant claim array and its proof holds).
      P.claim[t] = inside ? exit_t : C_ID;
      if (P.first_miss) atomicMin((unsigned long long *)&P.first_miss[G.s], (unsigned long long)t);
      if (P.dlist) {
        // the tiles whose entry this repair changes: t + 1 and, through identity claims, up to
        // the first later tile with a claim of its own (a longer run: the next pass is a full one)
        const uint64_t tend = P.tile_prefix[G.s + 1];
        uint64_t j = t + 1;
        uint32_t r = 0;
        for (; j < tend && r < 64u; j++, r++) {
          // once per tile per list: two workgroups verifying one tile in the same pass would race
          // on its records (the slow path rewrites them while the other reads them)
          if (atomicMax(&P.dstamp[j], P.pass_id) < P.pass_id) {
            const uint32_t q = atomicAdd(P.dlist_n, 1u);
            if (q < P.dlist_cap) P.dlist[q] = (uint32_t)j;
          }
          if (P.claim[j] != C_ID) break;
        }
        if (r == 64u) atomicOr(P.dlist_n + 2, 1u);  // (the list's overflow word)
      }
      if (P.stats) {  // debug capture (DRP_STATS=1): the first misses
        const unsigned long long q = atomicAdd(&P.stats[0], 1ull);
        if (q < 5) {
          P.stats[1 + 6 * q] = t;
          P.stats[2 + 6 * q] = et;
          P.stats[3 + 6 * q] = claim;
          P.stats[4 + 6 * q] = exit_t;
        }
      }
    }
    P.tile_exit[t] = exit_t;
    P.tile_count[t] = count_t;
    P.tile_nch[t] = nch_t;
    if (P.tile_k) P.tile_k[t] = 0;  // (this kernel rewrote the records of the threads before e_t)
    if (P.tile_recok) P.tile_recok[t] = 0;  // (the wire-reading emission takes it)
    if (P.tile_sparse) P.tile_sparse[t] = 0;  // (its records may be the slow path's: emit_tiles takes it)
  }
  }
}

// ==== scan: tile_base = exclusive prefix of tile_count (reduce, top, down-sweep) ================
constexpr uint32_t SCAN_BLK = 1024, SCAN_PER = 4, SCAN_SPAN = SCAN_BLK * SCAN_PER;

__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t *sw, uint64_t &total) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  uint64_t x = v;
#pragma unroll
  for (uint32_t d = 1; d < WAVE; d <<= 1) {
    const uint64_t y = shfl_up64(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) sw[wid] = x;
  __syncthreads();
  uint64_t off = 0;
  total = 0;
  for (uint32_t w = 0; w < blockDim.x / WAVE; w++) {
    if (w < wid) off += sw[w];
    total += sw[w];
  }
  __syncthreads();
  return off + x - v;
}

__global__ __launch_bounds__(SCAN_BLK) void scan_reduce(const uint64_t *cnt, const uint64_t *tile_prefix,
                                                         uint64_t nstreams, uint64_t *bsum) {
  __shared__ uint64_t sw[SCAN_BLK / WAVE];
  const uint64_t nt = tile_prefix[nstreams];
  const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_SPAN + threadIdx.x * SCAN_PER;
  uint64_t v = 0;
  for (uint32_t k = 0; k < SCAN_PER; k++)
    if (i0 + k < nt) v += cnt[i0 + k];
  uint64_t total;
  (void)block_excl_scan64(v, sw, total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(SCAN_BLK) void scan_top(uint64_t *bsum, uint64_t nb) {
  __shared__ uint64_t sw[SCAN_BLK / WAVE];
  uint64_t carry = 0;
  for (uint64_t c0 = 0; c0 < nb; c0 += SCAN_BLK) {
    const uint64_t i = c0 + threadIdx.x;
    const uint64_t v = i < nb ? bsum[i] : 0;
    uint64_t total;
    const uint64_t ex = block_excl_scan64(v, sw, total);
    if (i < nb) bsum[i] = carry + ex;
    carry += total;
  }
}

// ONE: a single block covers every tile (no reduce / top passes: its offset is 0)
template <bool ONE>
__global__ __launch_bounds__(SCAN_BLK) void scan_down(const uint64_t *cnt, const uint64_t *tile_prefix,
                                                       uint64_t nstreams, const uint64_t *bsum, uint64_t *base,
                                                       uint64_t cap, uint32_t *overflow) {
  __shared__ uint64_t sw[SCAN_BLK / WAVE];
  const uint64_t nt = tile_prefix[nstreams];
  const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_SPAN + threadIdx.x * SCAN_PER;
  uint64_t c[SCAN_PER], v = 0;
  for (uint32_t k = 0; k < SCAN_PER; k++) {
    c[k] = i0 + k < nt ? cnt[i0 + k] : 0;
    v += c[k];
  }
  uint64_t total;
  uint64_t o = (ONE ? 0ull : bsum[blockIdx.x]) + block_excl_scan64(v, sw, total);
  for (uint32_t k = 0; k < SCAN_PER; k++) {
    if (i0 + k < nt) {
      base[i0 + k] = o;
      if (i0 + k == nt - 1 && o + c[k] > cap) atomicOr(overflow, 1u);
    }
    o += c[k];
  }
}

// ==== kernel 3: emission ========================================================================
// Frame-major: the tile's frame starts go to an LDS list (thread order = stream order), then
// thread i decodes frames i, i + NT, ... so every column store is a contiguous run.
#ifndef DRP_LCAP
#define DRP_LCAP 1024
#endif
constexpr uint32_t LCAP = DRP_LCAP;  // frames per tile listed in LDS (denser tiles emit per thread)

__device__ __noinline__ ChangeCols decode_change_hbm(const uint8_t *g, uint64_t se, uint64_t po, uint64_t pl) {
  const GlobalReader gr{g, se};
  return decode_change(gr, po, pl);
}

// The header at absolute p, 32-bit fast form for 1..3-byte length varints whose 16-byte window is
// inside the image and the stream (same results as Img::at); anything else takes Img::at.
__device__ __forceinline__ Hdr hdr_fast(const Img &m, uint64_t p) {
  const uint32_t o = (uint32_t)(p - m.A);
  if (p + 16 <= m.A + IMG && p + 16 <= m.se) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(m.lds) + (o >> 2);
    const uint32_t w = __builtin_amdgcn_alignbit(q[1], q[0], (o & 3u) * 8u);
    const uint32_t tm = ~w & 0x808080u;
    if (tm) {
      const uint32_t k = ((uint32_t)__builtin_ctz(tm) >> 3) + 1u;
      const uint32_t L = ((w & 0x7Fu) | ((w >> 1) & 0x3F80u) | ((w >> 2) & 0x1FC000u)) & ((1u << (7u * k)) - 1u);
      const uint32_t id = (w >> (8u * k)) & 0xFFu;
      Hdr h;
      h.succ = 0;
      h.L = L;
      h.vlen = k;
      h.id = id;
      if (id >= 3u) h.kind = H_ERR_TYPE;
      else if (id == 0u) {
        h.kind = H_VALID;
        h.succ = p + k + 1u;
      } else if (L == 0u) h.kind = H_ERR_LEN;
      else if ((uint64_t)L > m.se - p - k) h.kind = id == 1u ? H_TAIL_CHANGE : H_TAIL_BLOB;
      else {
        h.kind = H_VALID;
        h.succ = p + k + L;
      }
      return h;
    }
  }
  return m.at(p);
}

__device__ __forceinline__ void emit_frame(const DecodeParams &P, const Img &m, uint64_t p, uint64_t f,
                                           uint32_t &nch, uint32_t &nbl, uint64_t &badf) {
  const Hdr h = hdr_fast(m, p);
  const uint64_t po = p + h.vlen + 1;
  const uint64_t pl = h.L - 1;
  if (h.id == 1) nch++; else nbl++;
  if (f >= P.cap) return;
  const DecodeParams *K = &P;
  K->payload_off[f] = po;
  K->payload_len[f] = pl > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)pl;
  K->type[f] = (uint8_t)(h.id | (h.kind == H_TAIL_BLOB ? DRP_FRAME_PARTIAL : 0u));
  if (h.id != 1) return;
  const LdsReader rd{m.lds, m.A, umin64(m.A + IMG, m.se)};
  ChangeCols c = decode_change(rd, po, pl);
  if (c.err == ERR_UNREACHABLE) c = decode_change_hbm(P.bytes, m.se, po, pl);
  K->key_off[f] = c.key_off;
  K->key_len[f] = c.key_len;
  K->subset_off[f] = c.subset_off;
  K->subset_len[f] = c.subset_len;
  K->value_off[f] = c.value_off;
  K->value_len[f] = c.value_len;
  K->change[f] = c.change;
  K->from[f] = c.from;
  K->to[f] = c.to;
  uint32_t fl = c.flags;
  if (c.err == DRP_ERR_REQUIRED) fl |= DRP_F_MISSING;
  K->flags[f] = (uint8_t)fl;
  if (c.err) badf = f < badf ? f : badf;
}

// Output columns at a tile's first row: emit_lean stores at a uniform column pointer plus a 32-bit
// byte offset (SGPR base + VGPR offset addressing).
struct RowCols {
  uint64_t *poff;
  uint32_t *plen;
  uint8_t *type;
  uint32_t *ko, *kl, *so, *sl, *vo, *vl;
  uint64_t *ch, *fr, *to;
  uint8_t *fl;
  uint32_t lim;  // rows the tile may write (the capacity left)
};
__device__ __forceinline__ RowCols row_cols(const DecodeParams &P, uint64_t base) {
  RowCols r;
  r.poff = P.payload_off + base;
  r.plen = P.payload_len + base;
  r.type = P.type + base;
  r.ko = P.key_off + base;
  r.kl = P.key_len + base;
  r.so = P.subset_off + base;
  r.sl = P.subset_len + base;
  r.vo = P.value_off + base;
  r.vl = P.value_len + base;
  r.ch = P.change + base;
  r.fr = P.from + base;
  r.to = P.to + base;
  r.fl = P.flags + base;
  r.lim = base >= P.cap ? 0u : (uint32_t)umin64(P.cap - base, 0xFFFFFFFFull);
  return r;
}

// ---- sparse tiles: frames decoded from HBM, no staging ---------------------------------------
// A tile whose threads from tile_k on each deliver at most one frame (at the thread's entry, from
// verification's records) and at most SP_FRAMES in all (long frames: C5's 4 KB Changes, blob
// payloads) needs no walk and no LDS image: its frame starts are the entries themselves. Eight
// lanes read a tile's records (16 threads each), the frames go to an LDS list, and every thread
// then decodes one frame through 16-byte windows of the batch (header, then the Change field
// headers: string and bytes contents are skipped, so a 4 KB value costs nothing). The columns
// are decode_change's. A frame whose entry is not a delivered header (an id-0 header before it)
// clears the tile's mark and emit_tiles takes the whole tile as before.
struct GlobalWinReader {
  static constexpr bool kFast = true;
  const uint8_t *g;
  uint64_t lim;  // the stream end
  __device__ __forceinline__ bool ok(uint64_t p, uint64_t n) const { return p + n <= lim; }
  __device__ __forceinline__ void win(uint64_t p, uint64_t &w0, uint64_t &w1) const {
    const uint64_t a = p & ~15ull;
    const uint4 u = ld16(g, a, lim), v = ld16(g, a + 16, lim);
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
  }
  __device__ __forceinline__ void win8(uint64_t p, uint32_t &w, uint32_t &wn) const {
    uint64_t w0, w1;
    win(p, w0, w1);
    w = (uint32_t)w0;
    wn = (uint32_t)(w0 >> 32);
  }
};

// change_canon for a payload in HBM, in two dependent reads instead of one per field: the key
// field from a window at the payload start, then change / from / to and the value header from a
// 32-byte window after the key, parsed in registers. Canonical shape only (key first, varints of
// <= 7 bytes, the value last); false: decode_change decides (same columns wherever this accepts).
__device__ __forceinline__ bool change_canon_g(const GlobalWinReader &rd, uint64_t po, uint64_t pl, ChangeCols &c) {
  c.subset_off = c.subset_len = c.value_off = c.value_len = 0;
  c.change = c.from = c.to = 0;
  c.flags = 0;
  c.err = 0;
  if (pl < 8 || pl > 0x7FFFFFFFull || !rd.ok(po, pl)) return false;
  uint64_t w0, w1;
  rd.win(po, w0, w1);
  if ((w0 & 0xFFu) != 0x12u) return false;
  const uint32_t b1 = (uint32_t)(w0 >> 8) & 0xFFu, b2 = (uint32_t)(w0 >> 16) & 0xFFu;
  uint32_t kl, ko;
  if (b1 < 0x80u) {
    kl = b1;
    ko = 2;
  } else {
    if (b2 >= 0x80u) return false;
    kl = (b1 & 0x7Fu) | (b2 << 7);
    ko = 3;
  }
  const uint64_t q = (uint64_t)ko + kl;
  if (q >= pl) return false;
  c.key_off = ko;
  c.key_len = kl;
  uint64_t x[4];
  rd.win(po + q, x[0], x[1]);
  rd.win(po + q + 16, x[2], x[3]);
  uint64_t used = 0;
  uint64_t v[3];
#pragma unroll
  for (uint32_t f = 0; f < 3; f++) {
    if ((x[0] & 0xFFu) != 0x18u + 8u * f) return false;
    const uint64_t y = x[0] >> 8;  // the varint's bytes (up to 7)
    const uint64_t tm = ~y & 0x80808080808080ull;
    if (!tm) return false;
    const uint32_t k = ((uint32_t)__builtin_ctzll(tm) >> 3) + 1u;
    v[f] = ((y & 0x7Full) | ((y >> 1) & 0x3F80ull) | ((y >> 2) & 0x1FC000ull) | ((y >> 3) & 0xFE00000ull) |
            ((y >> 4) & 0x7F0000000ull) | ((y >> 5) & 0x3F800000000ull) | ((y >> 6) & 0x1FC0000000000ull)) &
           ((1ull << (7u * k)) - 1ull);
    const uint32_t sb = 8u * (1u + k);  // (2..8 bytes)
    used += 1u + k;
    if (q + used > pl) return false;
    x[0] = sb == 64 ? x[1] : (x[0] >> sb) | (x[1] << (64u - sb));
    x[1] = sb == 64 ? x[2] : (x[1] >> sb) | (x[2] << (64u - sb));
    x[2] = sb == 64 ? x[3] : (x[2] >> sb) | (x[3] << (64u - sb));
    x[3] = sb == 64 ? 0ull : x[3] >> sb;
  }
  c.change = v[0];
  c.from = v[1];
  c.to = v[2];
  if (q + used == pl) return true;  // (no value)
  if ((x[0] & 0xFFu) != 0x32u) return false;
  const uint64_t y = x[0] >> 8;
  const uint64_t tm = ~y & 0x80808080ull;  // a value length of <= 4 bytes
  if (!tm) return false;
  const uint32_t k = ((uint32_t)__builtin_ctzll(tm) >> 3) + 1u;
  const uint64_t vl =
      ((y & 0x7Full) | ((y >> 1) & 0x3F80ull) | ((y >> 2) & 0x1FC000ull) | ((y >> 3) & 0xFE00000ull)) &
      ((1ull << (7u * k)) - 1ull);
  const uint64_t vo = q + used + 1u + k;
  if (vo + vl != pl) return false;
  c.value_off = (uint32_t)vo;
  c.value_len = (uint32_t)vl;
  c.flags = DRP_F_VALUE;
  return true;
}

constexpr uint32_t SP_TPB = 64;  // tiles per workgroup
__global__ __launch_bounds__(256) void emit_sparse(DecodeParams P) {
  __shared__ uint32_t lst[SP_TPB * SP_FRAMES];  // tile (in the workgroup) << 16 | thread << 8 | rank
  __shared__ uint32_t nl;
  __shared__ uint32_t fail[SP_TPB];
  if (*P.overflow & (F_MISS | F_WAIT)) return;  // (a failed prediction: emitted after its repair)
  const uint32_t tid = threadIdx.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * SP_TPB;
  const uint64_t ntiles = P.tile_prefix[P.nstreams];
  if (tid == 0) nl = 0;
  if (tid < SP_TPB) fail[tid] = 0;
  __syncthreads();
  // records: VL_G lanes per tile (16 threads each), 256 / VL_G tiles per pass
  constexpr uint32_t PER = 256 / VL_G;
  for (uint32_t pass = 0; pass < SP_TPB / PER; pass++) {
    const uint32_t j = pass * PER + tid / VL_G, r = tid % VL_G;
    const uint64_t t = t0 + j;
    const bool sp = t < ntiles && P.tile_sparse[t];
    uint32_t fm = 0;  // this lane's threads that deliver a frame at their entry
    if (sp) {
      const uint32_t k0 = P.tile_k[t];
      const uint4 e4 = *reinterpret_cast<const uint4 *>(P.ent + t * NT + 16u * r);
      const uint4 n4 = *reinterpret_cast<const uint4 *>(P.ent_n + t * NT + 16u * r);
      const uint32_t ew[4] = {e4.x, e4.y, e4.z, e4.w}, nw[4] = {n4.x, n4.y, n4.z, n4.w};
#pragma unroll
      for (uint32_t b = 0; b < 16; b++) {
        const uint32_t e = (ew[b >> 2] >> (8u * (b & 3u))) & 0xFFu, n = (nw[b >> 2] >> (8u * (b & 3u))) & 0xFFu;
        if (16u * r + b >= k0 && e < 0x80u && n == 1u) fm |= 1u << b;
      }
    }
    const uint32_t c = (uint32_t)__builtin_popcount(fm);
    uint32_t pre = c;  // inclusive prefix over the tile's 8 lanes
#pragma unroll
    for (uint32_t d = 1; d < VL_G; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)pre, d, VL_G);
      if (r >= d) pre += y;
    }
    uint32_t rank = pre - c;
    if (c) {
      uint32_t q = atomicAdd(&nl, c);
      for (uint32_t bits = fm; bits; bits &= bits - 1, q++, rank++)
        if (q < SP_TPB * SP_FRAMES) lst[q] = (j << 16) | ((16u * r + (uint32_t)__builtin_ctz(bits)) << 8) | rank;
    }
  }
  __syncthreads();
  const uint32_t n = min(nl, SP_TPB * SP_FRAMES);  // (<= SP_FRAMES per tile: never cut)
  for (uint32_t i = tid; i < n; i += 256) {
    const uint32_t e = lst[i], j = e >> 16, th = (e >> 8) & 0xFFu, rank = e & 0xFFu;
    const uint64_t t = t0 + j;
    const TileGeo G = tile_geo(P, t);
    const uint64_t p = G.A + (uint64_t)th * SEGB + (P.ent[t * NT + th] & 63u);
    const GlobalWinReader rd{P.bytes, G.se};
    uint64_t w0, w1;
    rd.win(p, w0, w1);
    const Hdr h = parse_win(w0, w1, p, G.se);
    if (!((h.kind == H_VALID && h.id != 0) || h.kind == H_TAIL_BLOB)) {
      fail[j] = 1;  // (an id-0 header at the entry: the delivered frame is further on)
      continue;
    }
    const uint64_t f = P.tile_base[t] + rank;
    if (f >= P.cap) continue;
    const uint64_t po = p + h.vlen + 1, pl = h.L - 1;
    P.payload_off[f] = po;
    P.payload_len[f] = pl > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)pl;
    P.type[f] = (uint8_t)(h.id | (h.kind == H_TAIL_BLOB ? DRP_FRAME_PARTIAL : 0u));
    if (h.id != 1) continue;
    ChangeCols cc;
    if (!change_canon_g(rd, po, pl, cc)) cc = decode_change(rd, po, pl);
    P.key_off[f] = cc.key_off;
    P.key_len[f] = cc.key_len;
    P.subset_off[f] = cc.subset_off;
    P.subset_len[f] = cc.subset_len;
    P.value_off[f] = cc.value_off;
    P.value_len[f] = cc.value_len;
    P.change[f] = cc.change;
    P.from[f] = cc.from;
    P.to[f] = cc.to;
    uint32_t fl = cc.flags;
    if (cc.err == DRP_ERR_REQUIRED) fl |= DRP_F_MISSING;
    P.flags[f] = (uint8_t)fl;
    if (cc.err) atomicMin((unsigned long long *)&P.payload_err[G.s], (unsigned long long)f);
  }
  __syncthreads();
  if (tid < SP_TPB && fail[tid]) P.tile_sparse[t0 + tid] = 0;  // ((t0 + tid < ntiles: fail is only set for tiles)
}


// The general emit: the tiles emit_lean / emit_sparse list (P.vlist; null: every tile), each
// re-emitted whole from its verified entries with the general Change decoder (decode_change: any
// field order, repeated or unknown fields, errors).
__global__ __launch_bounds__(NT, DRP_EMIT_WAVES) void emit_tiles(DecodeParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[IMG + 32];
  __shared__ uint16_t lst[LCAP];
  __shared__ uint32_t wsum[NT / WAVE];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u, wid = tid >> 6;
  uint64_t tl_ = P.stats && tid == 0 ? __builtin_amdgcn_s_memtime() : 0;
  if (*P.overflow & (F_MISS | F_WAIT)) return;  // (a failed prediction: emitted after its repair)
  const uint64_t ntiles = P.tile_prefix[P.nstreams];
  const uint32_t nwork = P.vlist ? *P.vlist_n : 0u;
  for (uint32_t wi = blockIdx.x; P.vlist ? wi < nwork : wi == blockIdx.x; wi += gridDim.x) {
  const uint64_t t = P.vlist ? P.vlist[wi] & ~VL_HARD : wi;
  bsync();  // the previous tile's LDS reads are done
  const TileGeo G = tile_geo(P, t);  // (its loads go out with the tile count's)
  if (t >= ntiles) continue;  // (whole workgroup)
  const uint64_t se = G.se, A = G.A;
  // the records load with the tile bytes, not after them
  const uint64_t base = ldc(P.tile_base + t);
  const uint32_t k0 = P.tile_k ? P.tile_k[t] : 0u;  // threads before e_t's (verify_lite)
  const uint8_t eb = tid < k0 ? (uint8_t)0xFF : P.ent[t * NT + tid];  // exact entry of this thread's bytes
  const uint8_t en = P.ent_n[t * NT + tid];   // exact frames from it (kernel 2)
  stage_glds(P, G, buf);
  const Img m{buf, P.bytes, A, se};
  const uint64_t lb = A + (uint64_t)tid * SEGB, s1 = lb + SEGB;
  const uint64_t E = !(eb & 0x80) ? lb + (eb & 63) : NONE;
  PHASE(11);
  const uint32_t n = (eb & 0x80) ? 0u : en;
  const uint32_t ni = wave_incl_scan32(n);
  if (lane == 63) wsum[wid] = ni;
  bsync();
  uint32_t woff = 0, count_t = 0;
#pragma unroll
  for (int w = 0; w < NT / WAVE; w++) {
    if ((uint32_t)w < wid) woff += wsum[w];
    count_t += wsum[w];
  }
  PHASE(12);
  uint32_t nch = 0, nbl = 0;
  uint64_t badf = ~0ull;
  const bool listed = count_t <= LCAP;
  // this thread's frames, in order: list them (or, for very dense tiles, emit them here)
  if (n) {
    uint32_t i = woff + ni - n;
    uint64_t p = E;
    while (p < s1 && p < se) {
      const Hdr h = hdr_fast(m, p);
      if (h.kind != H_VALID && h.kind != H_TAIL_BLOB) break;
      if (h.id != 0) {
        if (listed) lst[i] = (uint16_t)(p - A);
        else emit_frame(P, m, p, base + i, nch, nbl, badf);
        i++;
      }
      if (h.kind != H_VALID) break;
      p = h.succ;
    }
  }
  if (listed) {
    bsync();
    for (uint32_t i = tid; i < count_t; i += NT) emit_frame(P, m, A + lst[i], base + i, nch, nbl, badf);
  }
  PHASE(13);
  (void)nch;
  (void)nbl;
  badf = lane_min64(badf);
  if (lane == 0 && badf != ~0ull) atomicMin((unsigned long long *)&P.payload_err[G.s], (unsigned long long)badf);
  }
}

// ---- the lean fast emit ------------------------------------------------------------------------
// Most tiles hold only Change payloads in protocol-buffers@2's own field order with short varints
// (the shape every encoder writes) and at most a few frames per 64-byte thread segment. For those,
// emit_lean walks each thread's frames from its verified entry and decodes each one in place from
// the LDS image: the header from one 8-byte window, the fields in canonical order (one window per
// field, or one window for change / from / to / the value header when their varints are one byte),
// 32-bit image offsets, and column stores at the tile's row base plus a 32-bit byte offset. Any
// other shape (field order, repeated or unknown fields, varints of more than 5 bytes, headers
// near the image end, length varints of more than 3 bytes) sends the whole tile to the general
// kernel (emit_tiles over P.vlist), which writes the same columns for the rest.
#ifndef DRP_EMIT_LEAN_WAVES
#define DRP_EMIT_LEAN_WAVES 6
#endif
// bytes o .. o + 7 of the image (three dword reads; the image has 32 bytes of slack)
__device__ __forceinline__ uint64_t lds_u64(const uint8_t *lds, uint32_t o) {
  const uint32_t *q = reinterpret_cast<const uint32_t *>(lds) + (o >> 2);
  const uint32_t sh = (o & 3u) * 8u, a0 = q[0], a1 = q[1], a2 = q[2];
  return (uint64_t)__builtin_amdgcn_alignbit(a1, a0, sh) | ((uint64_t)__builtin_amdgcn_alignbit(a2, a1, sh) << 32);
}
// a varint of 1..5 bytes at the start of x: its length (0: none ends within 5 bytes) and value
__device__ __forceinline__ uint32_t vint5(uint64_t x, uint64_t &v) {
  const uint64_t tm = ~x & 0x8080808080ull;
  if (!tm) return 0;
  const uint32_t k = ((uint32_t)__builtin_ctzll(tm) >> 3) + 1u;
  v = ((x & 0x7Full) | ((x >> 1) & 0x3F80ull) | ((x >> 2) & 0x1FC000ull) | ((x >> 3) & 0xFE00000ull) |
       ((x >> 4) & 0x7F0000000ull)) &
      ((1ull << (7u * k)) - 1ull);
  return k;
}
// a length-delimited field (tag already checked) at image offset q: its content offset and length;
// false when the header leaves [0, lim) or the content leaves the payload (ending at end)
__device__ __forceinline__ bool ld_field(uint64_t x, uint32_t q, uint32_t end, uint32_t lim, uint32_t &o2,
                                         uint32_t &len) {
  uint64_t v;
  const uint32_t k = vint5(x >> 8, v);
  o2 = q + 1u + k;
  if (!k || o2 > lim || o2 > end || v > (uint64_t)(end - o2)) return false;
  len = (uint32_t)v;
  return true;
}
// a varint field (tag already checked) at q: its value; false as above
__device__ __forceinline__ bool vi_field(uint64_t x, uint32_t q, uint32_t end, uint32_t lim, uint32_t &q2,
                                         uint64_t &v) {
  const uint32_t k = vint5(x >> 8, v);
  q2 = q + 1u + k;
  return k && q2 <= lim && q2 <= end;
}
// The canonical Change at image offset po (pl bytes; the payload may run past the image, its
// field headers may not): [0x0a subset] 0x12 key 0x18 change 0x20 from 0x28 to [0x32 value],
// ending exactly at the payload end. Offsets relative to the payload, as decode_change's.
__device__ __forceinline__ bool change_canon(const uint8_t *lds, uint32_t po, uint32_t pl, uint32_t lim,
                                             ChangeCols &c) {
  const uint32_t end = po + pl;
  c.subset_off = c.subset_len = c.value_off = c.value_len = 0;
  c.flags = 0;
  c.err = 0;
  uint32_t q = po, o2, len;
  uint64_t x = lds_u64(lds, q);
  if ((x & 0xFFu) == 0x0Au) {
    if (!ld_field(x, q, end, lim, o2, len)) return false;
    c.subset_off = o2 - po;
    c.subset_len = len;
    c.flags = DRP_F_SUBSET;
    q = o2 + len;
    if (q >= lim) return false;
    x = lds_u64(lds, q);
  }
  if ((x & 0xFFu) != 0x12u || !ld_field(x, q, end, lim, o2, len)) return false;
  c.key_off = o2 - po;
  c.key_len = len;
  q = o2 + len;
  if (q + 8u <= lim) {
    x = lds_u64(lds, q);
    // change / from / to (and the value header) with one-byte varints: 18 a 20 b 28 c [32 d]
    if ((x & 0x00FF00FF00FF00FFull) == 0x0032002800200018ull && (x & 0x8080808080808080ull) == 0 &&
        q + 8u + (uint32_t)(x >> 56) == end) {
      c.change = (x >> 8) & 0xFFu;
      c.from = (x >> 24) & 0xFFu;
      c.to = (x >> 40) & 0xFFu;
      c.value_off = q + 8u - po;
      c.value_len = (uint32_t)(x >> 56);
      c.flags |= DRP_F_VALUE;
      return true;
    }
  }
  if (q >= lim) return false;
  x = lds_u64(lds, q);
  if ((x & 0xFFu) != 0x18u || !vi_field(x, q, end, lim, q, c.change) || q >= lim) return false;
  x = lds_u64(lds, q);
  if ((x & 0xFFu) != 0x20u || !vi_field(x, q, end, lim, q, c.from) || q >= lim) return false;
  x = lds_u64(lds, q);
  if ((x & 0xFFu) != 0x28u || !vi_field(x, q, end, lim, q, c.to)) return false;
  if (q == end) return true;
  if (q >= lim) return false;
  x = lds_u64(lds, q);
  if ((x & 0xFFu) != 0x32u || !ld_field(x, q, end, lim, o2, len) || o2 + len != end) return false;
  c.value_off = o2 - po;
  c.value_len = len;
  c.flags |= DRP_F_VALUE;
  return true;
}
// a store at a uniform column base plus a 32-bit byte offset (global_store ... saddr)
template <class T>
__device__ __forceinline__ void st_col(T *base, uint32_t i, T v) {
  *reinterpret_cast<T *>(reinterpret_cast<char *>(base) + (uint32_t)(i * (uint32_t)sizeof(T))) = v;
}

// ---- record emission: columns from claims_fast's per-frame records (fast_records) -------------
// The tiles verification lets it take (tile_recok = 1 + the slot of the tile's first row): rows
// [tile_base, + tile_count) from slot tile_recok - 1 on. Reads 24 B per row and writes the columns;
// the wire is not read again.
// one row (i: relative to C's first row): its columns from the record words (the tile's first
// byte at A)
__device__ __forceinline__ void emit_rec_row(const RowCols &C, uint32_t i, uint64_t A, uint32_t w0, uint32_t pl,
                                             uint32_t w2, uint32_t n0, uint32_t n1, uint32_t n2) {
  const uint32_t id = (w0 >> 14) & 3u;
  st_col(C.poff, i, A + (w0 & 0x3FFFu));
  st_col(C.plen, i, pl);
  st_col(C.type, i, (uint8_t)(id | (((w0 >> 16) & 1u) ? DRP_FRAME_PARTIAL : 0u)));
  if (id != 1u) return;
  const uint32_t hv = (w0 >> 17) & 1u, vo = hv ? w2 >> 16 : 0u;
  st_col(C.ko, i, 1u + ((w0 >> 18) & 3u));
  st_col(C.kl, i, w2 & 0xFFFFu);
  st_col(C.so, i, 0u);
  st_col(C.sl, i, 0u);
  st_col(C.vo, i, vo);
  st_col(C.vl, i, hv ? pl - vo : 0u);
  st_col(C.ch, i, (uint64_t)n0);
  st_col(C.fr, i, (uint64_t)n1);
  st_col(C.to, i, (uint64_t)n2);
  st_col(C.fl, i, (uint8_t)(hv ? DRP_F_VALUE : 0u));
}
// Output rows in chunks of 64, each chunk's stores starting at a 64-row boundary of the columns
// (scripts/probe_bw.hip: 62 B-per-row column stores run at 5.8 TB/s from 64-aligned chunks and at
// 2.9 TB/s from chunks shifted off that boundary). chunk_tiles first marks, per chunk, the tile
// holding its first row; the rows of a chunk then lie in that tile and the ones up to the next
// chunk's. A wave per chunk: its lanes' rows, their tiles (the first or the next one in the fast
// path, else a search over the tiles' first rows), and for a tile with records (tile_recok) the
// row's record words, loaded before the row is stored. Rows of tiles without records are left to
// emit_lean.
__global__ __launch_bounds__(256) void chunk_tiles(DecodeParams P) {
  if (!P.counter[13]) return;  // (claims_fast wrote no records: the hop walkers' claims)
  const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (t >= P.tile_prefix[P.nstreams]) return;
  const uint64_t b = P.tile_base[t], n = P.tile_count[t];
  if (!n || b >= P.cap) return;
  const uint64_t e = umin64(b + n, P.cap);
  for (uint64_t c = (b + 63) / 64; c * 64 < e; c++) P.chunk_tile[c] = (uint32_t)t;
}

constexpr uint32_t ER_WAVES = 4;  // chunks (waves) per workgroup
__global__ __launch_bounds__(ER_WAVES * WAVE) void emit_recs(DecodeParams P) {
  if (*P.overflow & (F_MISS | F_WAIT)) return;  // (a failed prediction: emitted after its repair)
  if (!P.counter[13]) return;                     // (claims_fast wrote no records)
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t c = (uint64_t)blockIdx.x * ER_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t ntiles = ldc(P.tile_prefix + P.nstreams);
  if (!ntiles) return;
  const uint64_t total = umin64(ldc(P.tile_base + ntiles - 1) + ldc(P.tile_count + ntiles - 1), P.cap);
  if (c * 64 >= total) return;  // (whole wave)
  const uint64_t r = c * 64 + lane;
  const uint64_t t0 = ldc(P.chunk_tile + c);
  const uint64_t t1 = (c + 1) * 64 < total ? (uint64_t)ldc(P.chunk_tile + c + 1) : ntiles - 1;
  // this lane's tile: the last tile in [t0, t1] whose first row is <= r
  uint64_t t = t0;
  const uint64_t b1 = t1 > t0 ? ldc(P.tile_base + t0 + 1) : ~0ull;
  if (t1 == t0 + 1 || t1 == t0) {  // (nearly always: tiles of more than 64 rows)
    if (r >= b1) t = t0 + 1;
  } else if (r >= b1) {  // (tiles of few rows, or runs of empty tiles: search)
    uint64_t lo = t0 + 1, hi = t1;  // base[lo] <= r; find the last such
    while (lo < hi) {
      const uint64_t mid = (lo + hi + 1) >> 1;
      if (P.tile_base[mid] <= r) lo = mid;
      else hi = mid - 1;
    }
    t = lo;
  }
  if (r >= total) return;
  const uint32_t rk = P.tile_recok[t];
  if (!rk) return;  // (emit_lean writes this row)
  const uint64_t bt = P.tile_base[t];
  const uint32_t *rr = P.rec + t * CR_TILE_WORDS + (uint32_t)(r - bt) + rk - 1u;
  uint32_t w[CR_WORDS];
#pragma unroll
  for (uint32_t k = 0; k < CR_WORDS; k++) w[k] = rr[k * CR_CAP];
  const uint64_t A = tile_geo(P, t).A;
  const RowCols C = row_cols(P, c * 64);
  emit_rec_row(C, lane, A, w[0], w[1], w[2], w[3], w[4], w[5]);
}

struct LeanLds {
  __attribute__((aligned(16))) uint8_t buf[IMG + 32];
  uint32_t wsum[NT / WAVE];
  uint32_t defer;
  uint64_t todo;  // (long-frame form) the workgroup's tiles that are not sparse
};
__device__ __forceinline__ void emit_lean_tile(const DecodeParams &P, uint64_t t, LeanLds &L);

// Long-frame streams (the context's change_checks form: >= 512 B per frame) leave nearly every
// tile to emit_sparse, and with per-frame records nearly every tile goes to emit_recs, so a
// workgroup per tile would mostly be dispatched to exit: there each
// workgroup takes EMIT_LONG_TPW consecutive tiles (drp_launch_spec_tail sizes the grid), reads
// their marks in one load (a lane each) and runs only the others (8 tiles with a load each in
// turn: C5's emit_lean took 0.116 ms of dependent mark loads). Consecutive, not strided by the
// grid: a tile's halo is its successor's head, and their column lines meet, in one L2 (with every
// tile left to it, the strided order took 4.5 ms on C2 against 2.8 for a workgroup per tile).
constexpr uint32_t EMIT_LONG_TPW = 32;
static_assert(EMIT_LONG_TPW <= WAVE, "one lane per tile's mark");
__global__ __launch_bounds__(NT, DRP_EMIT_LEAN_WAVES) void emit_lean(DecodeParams P) {
  __shared__ LeanLds L;
  if (*P.overflow & (F_MISS | F_WAIT)) return;  // (a failed prediction: emitted after its repair)
  if (P.change_checks || P.rec) {
    const uint64_t ntiles = P.tile_prefix[P.nstreams];
    const uint32_t tid = threadIdx.x;
    if (tid < WAVE) {
      const uint64_t t = (uint64_t)blockIdx.x * EMIT_LONG_TPW + tid;
      const bool run = tid < EMIT_LONG_TPW && t < ntiles && !(P.tile_sparse && P.tile_sparse[t]) &&
                       !(P.tile_recok && P.tile_recok[t]);
      const uint64_t m = __ballot(run);
      if (tid == 0) L.todo = m;
    }
    bsync();
    uint64_t todo = L.todo;
    bool first = true;
    while (todo) {  // (uniform)
      const uint32_t j = (uint32_t)__builtin_ctzll(todo);
      todo &= todo - 1;
      if (!first) bsync();  // (the last tile's LDS reads are done)
      first = false;
      emit_lean_tile(P, (uint64_t)blockIdx.x * EMIT_LONG_TPW + j, L);
    }
    return;
  }
  uint64_t t;
  {  // XCD-contiguous tile order, as the fast emit_tiles
    const uint32_t n = gridDim.x, q = n / 8u, r = n % 8u, x = blockIdx.x % 8u;
    t = (uint64_t)x * q + min(x, r) + blockIdx.x / 8u;
  }
  emit_lean_tile(P, t, L);
}

__device__ __forceinline__ void emit_lean_tile(const DecodeParams &P, uint64_t t, LeanLds &L) {
  uint8_t *buf = L.buf;
  uint32_t *wsum = L.wsum;
  uint32_t &defer = L.defer;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  // emit_sparse wrote it (first: on C5 nearly every tile leaves here, after one load; the mark
  // array covers the grid, and a stale mark past the tile count only ends a tile that ends anyway),
  // or the record emission writes it
  if (P.tile_sparse && P.tile_sparse[t]) return;
  const uint64_t ntiles = P.tile_prefix[P.nstreams];
  const TileGeo G = tile_geo(P, t);
  if (t >= ntiles) return;  // (whole workgroup)
  const uint64_t A = G.A;
  const uint64_t base = ldc(P.tile_base + t);
  const RowCols C = row_cols(P, base);
  const uint32_t se_rel = (uint32_t)umin64(G.se - A, 0x7FFFFFFFull);
  const uint32_t lim = se_rel < IMG ? se_rel : IMG;  // image bytes of the stream
  const uint32_t k0 = P.tile_k ? P.tile_k[t] : 0u;
  const uint8_t eb = tid < k0 ? (uint8_t)0xFF : P.ent[t * NT + tid];  // exact entry of this thread's bytes
  const uint8_t en = P.ent_n[t * NT + tid];                            // frames from it
  if (tid == 0) defer = 0;
  stage_glds(P, G, buf);
  const uint32_t n = (eb & 0x80) ? 0u : en;
  const uint32_t ni = wave_scan_dpp(n);
  if (lane == 63) wsum[wid] = ni;
  bsync();
  uint32_t i = ni - n;
#pragma unroll
  for (uint32_t w = 0; w < NT / WAVE; w++)
    if (w < wid) i += wsum[w];
  bool ok = true;
  if (n) {
    uint32_t o = tid * SEGB + (eb & 63u);
    const uint32_t s1r = tid * SEGB + SEGB;
    while (o < s1r && o < se_rel) {
      if (o + 16u > lim) {  // a header near the image or stream end: the general kernel
        ok = false;
        break;
      }
      const uint32_t w = (uint32_t)lds_u64(buf, o);
      const uint32_t tm = ~w & 0x808080u;
      if (!tm) {  // a length varint of 4 bytes or more
        ok = false;
        break;
      }
      const uint32_t k = ((uint32_t)__builtin_ctz(tm) >> 3) + 1u;
      const uint32_t L = ((w & 0x7Fu) | ((w >> 1) & 0x3F80u) | ((w >> 2) & 0x1FC000u)) & ((1u << (7u * k)) - 1u);
      const uint32_t id = (w >> (8u * k)) & 0xFFu;
      if (id == 0u) {  // (a type-0 header: nothing delivered, the next header follows its id byte)
        o += k + 1u;
        continue;
      }
      if (id > 2u || L == 0u) break;  // a protocol error ends the chain here (finalize reports it)
      const uint32_t po = o + k + 1u, pl = L - 1u;
      const bool tail = L > se_rel - o - k;  // cut by the stream end
      if (tail && id == 1u) break;           // (a Change cut by the stream end is carried, not delivered)
      if (i < C.lim) {
        st_col(C.poff, i, A + po);
        st_col(C.plen, i, pl);
        st_col(C.type, i, (uint8_t)(id | (tail ? DRP_FRAME_PARTIAL : 0u)));
        if (id == 1u) {
          ChangeCols c;
          c.change = c.from = c.to = 0;
          if (!change_canon(buf, po, pl, lim, c)) {
            ok = false;
            break;
          }
          st_col(C.ko, i, c.key_off);
          st_col(C.kl, i, c.key_len);
          st_col(C.so, i, c.subset_off);
          st_col(C.sl, i, c.subset_len);
          st_col(C.vo, i, c.value_off);
          st_col(C.vl, i, c.value_len);
          st_col(C.ch, i, c.change);
          st_col(C.fr, i, c.from);
          st_col(C.to, i, c.to);
          st_col(C.fl, i, (uint8_t)c.flags);
        }
      }
      i++;
      if (tail) break;
      o += k + L;
    }
  }
  if (!ok) defer = 1;
  bsync();
  if (defer && tid == 0) P.vlist[atomicAdd(P.vlist_n, 1u)] = (uint32_t)t;
}

// ==== segmented repair: exact claims for an unsettled stream range ==============================
// Verify passes fix only the first tile of a run of wrong predictions that agree with each other
// (each pass proves one more entry), so a stream crafted with a second valid framing beside the
// real one (tests/_streams.shadow_stream) would need one pass per tile. After a few passes the
// host recomputes the claims of such a stream from its first missed tile t0 on, by exact chain
// walks, in three launches:
//   1. seg_walk    per segment of G tiles: up to 64 candidate entries near the segment start
//                  (positions of its first tile whose header and next header parse; segment 0
//                  also takes e_t0), walked in parallel, one lane each, through the segment's
//                  tiles staged in LDS (tiles no chain starts a frame in are skipped); their
//                  exits at the segment end.
//   2. seg_stitch  one wave, segment by segment: the exact entry is one of the candidates (its
//                  exit is the next entry) or is walked from global memory (rare: an entry
//                  deeper in the segment than its first tile, inside a long blob).
//   3. seg_claims  per segment, the one exact chain from its entry: each tile's claim (the first
//                  chain position past it, the chain's end, or identity).
// A verify pass then proves the new claims as usual. Cost: two streaming passes over the range
// spread over the CUs plus a short serial stitch, however the predictions failed.
constexpr uint32_t SEG_CAND = 64, SEG_GMAX = 1024;  // candidates per segment, tiles per segment (max)
constexpr uint32_t CT_SKIP = 0xFFFFFFFFu, CT_END = 0xFFFFFFFEu, CT_PAST = 0xFFFFFFFDu;  // (ctile markers)
static_assert((uint64_t)SEG_GMAX * TILE < (1ull << 32), "seg_walk: 32-bit offsets in a segment");
constexpr uint64_t SEG_NMAX = 8192;  // segments per repair (max)
#ifndef DRP_SEG_NTARGET
#define DRP_SEG_NTARGET 2048
#endif
constexpr uint64_t SEG_NTARGET = DRP_SEG_NTARGET;  // segments per repair (aimed at)
constexpr uint64_t SEG_GMIN = 4;     // tiles per segment (min)
struct SegRange {
  uint64_t s, t0, tl, G, nseg;  // stream, tiles [t0, tl), tiles per segment, segments
  uint64_t tend;                // the stream's tile end (tl < tend: the range was clamped)
  uint64_t *cand;               // per segment: 64 starts, then 64 exits
  uint64_t *seg_entry;          // [nseg + 1] exact entry of each segment (and the final exit)
  uint8_t *nidx;                // [nseg][64] seg_link: the next segment's candidate each exit is
  uint8_t *seg_lane;            // [nseg] seg_stitch: the candidate that is the exact chain (0xFF: serial)
  uint32_t *ctile;              // [tiles of the range][64] seg_walk: each candidate's position entering
                                // each walked tile, from the segment start (CT_* markers), or null
};

__device__ __forceinline__ TileGeo seg_geo(const DecodeParams &P, uint64_t s) {
  TileGeo G;
  G.s = s;
  G.tf = P.tile_prefix[s];
  G.so = P.stream_off[s];
  G.se = P.stream_off[s + 1];
  G.A = 0;
  G.e0 = G.so + (P.entry ? P.entry[s] : 0ull);
  return G;
}
__device__ __forceinline__ uint64_t seg_tile_a(const TileGeo &G, uint64_t u) {
  return (G.so & ~(uint64_t)(TILE - 1)) + (u - G.tf) * TILE;
}
// the segment's end: the next segment's first tile, or the stream end
__device__ __forceinline__ uint64_t seg_end(const TileGeo &G, const SegRange &R, uint64_t seg) {
  const uint64_t tb = umin64(R.t0 + (seg + 1) * R.G, R.tl);
  return tb >= R.tend ? G.se : seg_tile_a(G, tb);
}
// chain step inside the staged tile: advance p while it starts a frame before lim (the tile end,
// or the segment end); a header that ends the chain returns MARK_TERM (| M_ERR) | p
__device__ __forceinline__ uint64_t seg_advance(const Img &m, uint64_t p, uint64_t lim) {
  while (is_pos(p) && p < lim && p < m.se) {
    const Hdr h = hdr_fast(m, p);  // (1..3-byte varints parsed in 32 bits; others as Img::at)
    if (h.kind != H_VALID) return term_of(h, p);
    p = h.succ;
  }
  return p;
}
// seg_advance, counting the headers parsed (steps)
__device__ __forceinline__ uint64_t seg_advance_n(const Img &m, uint64_t p, uint64_t lim, uint32_t &steps) {
  while (is_pos(p) && p < lim && p < m.se) {
    const Hdr h = hdr_fast(m, p);
    steps++;
    if (h.kind != H_VALID) return term_of(h, p);
    p = h.succ;
  }
  return p;
}

// One tile of seg_walk's chains by table (the candidates' serial walks cost one header parse per
// frame, and a lane on a dense shadow chain walks ~80 frames per tile): every live position of the
// tile is parsed once into a node (its successor node, or its exit: a position at or past lim,
// or the chain's terminal), then pointer jumping gives every node its exit in log2(chain length)
// rounds, and each lane of wave 0 looks its chain's exit up. A successor that is not a live
// position (a header with a varint of more than 3 bytes, or none) continues serially from there,
// as does a tile with more than SW_CAP live positions. Same exits as seg_advance.
constexpr uint32_t SW_CAP = 512, SW_KW = SW_CAP / NT;
constexpr uint32_t SW_TERM = 0xFFFFFFFFu, SW_CONT = 0xFFFFFFFEu;  // (node codes below SW_CONT)
constexpr uint32_t SW_STEPS = 40;  // headers per tile above which the next tile is walked by table
struct SegWalkLds {
  uint64_t lmw[NT];
  uint64_t val[SW_CAP];
  uint32_t nx[SW_CAP];
  uint16_t dist[SW_CAP];  // headers from the node to its value (its chain's steps)
  uint16_t loff[NT];
  uint16_t lpos[SW_CAP];
  uint32_t xw[NT / WAVE], fl[NT / WAVE];
};
__device__ __forceinline__ uint64_t seg_tile_walk(const DecodeParams &P, const TileGeo &G, const uint8_t *buf,
                                                  SegWalkLds &T, uint64_t pos, uint64_t lim, uint32_t &steps) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  const Img mt{buf, P.bytes, G.A, G.se};
  const uint64_t live = live_lds(G, buf);
  const uint32_t cnt = (uint32_t)__builtin_popcountll(live);
  const uint32_t pre = wave_scan_dpp(cnt);
  if (lane == 63) T.xw[wid] = pre;
  T.lmw[tid] = live;
  bsync();
  const uint32_t off = pre - cnt + (wid ? T.xw[0] : 0u);
  const uint32_t total = NT == 2 * WAVE ? T.xw[0] + T.xw[1] : T.xw[0];
  const bool mine = wid == 0 && is_pos(pos) && pos >= G.A && pos < lim;  // (this lane's chain is here)
  if (total > SW_CAP) {  // dense tile: serial walks
    if (mine) pos = seg_advance_n(mt, pos, lim, steps);
    return pos;
  }
  T.loff[tid] = (uint16_t)off;
  {
    uint64_t bits = live;
    uint32_t i = off;
    while (bits) {
      T.lpos[i++] = (uint16_t)(tid * SEGB + (uint32_t)__builtin_ctzll(bits));
      bits &= bits - 1;
    }
  }
  bsync();
#pragma unroll
  for (uint32_t k = 0; k < SW_KW; k++) {
    const uint32_t i = tid + k * NT;
    if (i < total) {
      const uint64_t p = G.A + T.lpos[i];
      const Hdr h = hdr_fast(mt, p);
      uint32_t nx = SW_TERM;
      uint64_t v = 0;
      if (h.kind != H_VALID) {
        v = term_of(h, p);
      } else if (h.succ >= lim || h.succ >= mt.se) {
        v = h.succ;
      } else {
        const uint32_t rel = (uint32_t)(h.succ - G.A), th = rel / SEGB, b = rel % SEGB;
        const uint64_t lw = T.lmw[th];
        if ((lw >> b) & 1ull) {
          nx = T.loff[th] + (uint32_t)__builtin_popcountll(lw & ((1ull << b) - 1ull));
        } else {
          nx = SW_CONT;
          v = h.succ;
        }
      }
      T.nx[i] = nx;
      T.val[i] = v;
      T.dist[i] = 1;
    }
  }
  bsync();
  // pointer jumping: a node's (next, value) becomes its next node's, until every next is a code
  for (uint32_t round = 0;; round++) {
    uint32_t nn[SW_KW], dd[SW_KW];
    uint64_t vv[SW_KW];
    uint32_t chm = 0;
#pragma unroll
    for (uint32_t k = 0; k < SW_KW; k++) {
      const uint32_t i = tid + k * NT;
      nn[k] = 0;
      vv[k] = 0;
      dd[k] = 0;
      if (i < total) {
        const uint32_t j = T.nx[i];
        if (j < SW_CONT) {
          nn[k] = T.nx[j];
          vv[k] = T.val[j];
          dd[k] = (uint32_t)T.dist[i] + T.dist[j];
          chm |= 1u << k;
        }
      }
    }
    const uint64_t b = __ballot(chm != 0);
    if (lane == 0) T.fl[wid] = b != 0;
    bsync();  // this round's reads are done; flags visible
    uint32_t more = 0;
#pragma unroll
    for (uint32_t w = 0; w < NT / WAVE; w++) more |= T.fl[w];
#pragma unroll
    for (uint32_t k = 0; k < SW_KW; k++)
      if ((chm >> k) & 1u) {
        T.nx[tid + k * NT] = nn[k];
        T.val[tid + k * NT] = vv[k];
        T.dist[tid + k * NT] = (uint16_t)min(dd[k], 0xFFFFu);
      }
    bsync();  // writes visible; flag reads done
    if (!more || round > 16) break;  // (chains in a tile are shorter than 2^16 nodes)
  }
  if (mine) {
    const uint32_t rel = (uint32_t)(pos - G.A), th = rel / SEGB, b = rel % SEGB;
    const uint64_t lw = T.lmw[th];
    if ((lw >> b) & 1ull) {
      const uint32_t i = T.loff[th] + (uint32_t)__builtin_popcountll(lw & ((1ull << b) - 1ull));
      const uint32_t c = T.nx[i];
      pos = T.val[i];
      steps += T.dist[i];
      if (c == SW_CONT) pos = seg_advance_n(mt, pos, lim, steps);
    } else {
      pos = seg_advance_n(mt, pos, lim, steps);
    }
  }
  return pos;
}

__global__ __launch_bounds__(NT) void seg_walk(DecodeParams P, SegRange R) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[IMG + 32];
  __shared__ SegWalkLds T;
  __shared__ uint32_t tmode;
  __shared__ uint64_t cpos[SEG_CAND];
  __shared__ uint32_t xw[NT / WAVE];
  __shared__ uint64_t nxt;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
  const uint64_t seg = blockIdx.x;
  TileGeo G = seg_geo(P, R.s);
  const uint64_t ta = R.t0 + seg * R.G, send = seg_end(G, R, seg);
  G.A = seg_tile_a(G, ta);
  uint64_t e0 = NONE;  // segment 0: the exact entry of t0 (nearest non-identity claim before it)
  if (seg == 0) {
    e0 = G.e0;
    for (uint64_t j = R.t0; j > G.tf; j--) {
      const uint64_t c = P.claim[j - 1];
      if (c != C_ID) {
        e0 = c;
        break;
      }
    }
    if (tid == 0) R.seg_entry[0] = e0;
  }
  // candidates: live positions of the first tile whose header, and next header, parse
  const uint64_t live = stage_live(P, G, buf);
  const Img m{buf, P.bytes, G.A, G.se};
  const uint64_t lb = G.A + (uint64_t)tid * SEGB;
  uint64_t ok = 0;
  for (uint64_t bits = live; bits; bits &= bits - 1) {
    const uint32_t o = (uint32_t)__builtin_ctzll(bits);
    const uint64_t p = lb + o;
    const Hdr h = m.at(p);
    bool good = h.kind <= H_TAIL_BLOB;
    if (h.kind == H_VALID && h.succ < G.se && h.succ + 16 <= G.A + IMG) good = m.at(h.succ).kind <= H_TAIL_BLOB;
    if (good) ok |= 1ull << o;
  }
  const uint32_t cnt = (uint32_t)__builtin_popcountll(ok);
  const uint32_t pre = wave_incl_scan32(cnt);
  if (lane == 63) xw[wid] = pre;
  bsync();
  uint32_t idx = pre - cnt + (wid ? xw[0] : 0u);
  const uint32_t first = (seg == 0 && is_pos(e0) && e0 < send) ? 1u : 0u;
  const uint32_t nc = min((uint32_t)SEG_CAND, xw[0] + xw[1] + first);
  if (first && tid == 0) cpos[0] = e0;
  idx += first;
  for (uint64_t bits = ok; bits && idx < SEG_CAND; bits &= bits - 1, idx++)
    cpos[idx] = lb + (uint32_t)__builtin_ctzll(bits);
  bsync();
  uint64_t pos = (wid == 0 && lane < nc) ? cpos[lane] : NONE, start = pos;
  const uint64_t sb0 = seg_tile_a(G, ta);
  if (R.ctile)  // (tiles no chain is in stay CT_SKIP)
    for (uint64_t i = tid; i < (umin64(ta + R.G, R.tl) - ta) * SEG_CAND; i += NT)
      R.ctile[(ta - R.t0) * SEG_CAND + i] = CT_SKIP;
  // walk: the lanes' chains through the segment, tile by tile (a tile only when a chain is in it);
  // the next tile is fetched into registers while wave 0 walks this one (the chains usually go on
  // there), so its load latency is not on the segment's serial path
  uint4 pv[SEGB / 16], ph;
  bool table = false;
  for (;;) {
    TileGeo Gn = G;
    Gn.A = G.A + TILE;
    const bool pre = Gn.A < send;
    if (pre) load_image(P, Gn, pv, ph);
    // (the image of the tile staged last) The walk is by table while the last tile's longest chain
    // took more than SW_STEPS headers (dense chains), frame by frame otherwise.
    uint32_t steps = 0;
    if (R.ctile && wid == 0)  // (each candidate's position entering this tile, for seg_claims_par)
      R.ctile[((G.A - sb0) / TILE + ta - R.t0) * SEG_CAND + lane] =
          !is_pos(pos) ? CT_END : (pos >= send ? CT_PAST : (uint32_t)(pos - sb0));
    if (table) pos = seg_tile_walk(P, G, buf, T, pos, umin64(G.A + TILE, send), steps);
    if (wid == 0) {
      if (!(1 && table)) {
        const Img mt{buf, P.bytes, G.A, G.se};
        pos = seg_advance_n(mt, pos, umin64(G.A + TILE, send), steps);
      }
      // (the wave's lowest chain position, as a 32-bit offset from the segment start: a segment
      // is at most SEG_GMAX tiles)
      const uint64_t sb = seg_tile_a(G, ta);
      const uint32_t mr = wave_min_dpp(is_pos(pos) && pos < send ? (uint32_t)(pos - umin64(pos, sb)) : ~0u);
      const uint32_t smax = wave_max_dpp(steps);
      if (lane == 0) {
        nxt = mr == ~0u ? NONE : sb + mr;
        tmode = smax > SW_STEPS;
      }
    }
    bsync();
    table = tmode != 0;
    const uint64_t q = nxt;
    if (q == NONE) break;
    G.A = seg_tile_a(G, ta + (q - seg_tile_a(G, ta)) / TILE);
    if (pre && G.A == Gn.A) put_image(buf, pv, ph);  // (the barrier above ordered the walk's reads)
    else stage(P, G, buf);
  }
  if (wid == 0) {
    R.cand[seg * 2 * SEG_CAND + lane] = lane < nc ? start : NONE;
    R.cand[seg * 2 * SEG_CAND + SEG_CAND + lane] = pos;
  }
}

// seg_link: for every candidate of segment s, the index of its exit among segment s + 1's candidate
// starts (0xFF: none, or the chain ends or passes over s + 1), so the stitch can follow the chain by
// table lookups instead of a ballot per segment. One wave per segment.
__global__ __launch_bounds__(WAVE) void seg_link(DecodeParams P, SegRange R) {
  __shared__ uint64_t st[SEG_CAND];
  const uint32_t lane = threadIdx.x;
  const uint64_t s = blockIdx.x;
  uint32_t f = 0xFFu;
  if (s + 1 < R.nseg) {
    const TileGeo G = seg_geo(P, R.s);
    const uint64_t send = seg_end(G, R, s + 1);
    const uint64_t ex = R.cand[s * 2 * SEG_CAND + SEG_CAND + lane];
    st[lane] = R.cand[(s + 1) * 2 * SEG_CAND + lane];
    __syncthreads();
    if (is_pos(ex) && ex < send)
      for (uint32_t j = 0; j < SEG_CAND; j++)
        if (st[j] == ex) {
          f = j;
          break;
        }
  }
  R.nidx[s * SEG_CAND + lane] = (uint8_t)f;
}

// The candidate tables of SEG_SB segments at a time are staged in LDS by the whole workgroup
// (double-buffered: the next block loads while wave 0 follows the chain through this one), so
// the serial part is a ballot per segment on LDS data.
// Up to SEG_FAST segments, the chain is followed through seg_link's tables first, in parallel: the
// tables (64 B per segment) go to LDS; each (block of 64 segments, entry candidate) pair is followed
// through its block (all 64 x 32 of them at once), one thread chains the blocks' end maps, each
// block then follows its now-known entry, and the entries are written in parallel. Any segment
// whose entry is not one of its candidates (0xFF on the path) sends the whole range to the serial
// stitch below (1.7 GB dense cascade: 0.47 ms serially, ~0.02 by the tables).
constexpr uint32_t SEG_SB = 64, SEG_STB = 1024;  // segments per staged block, threads
constexpr uint32_t SEG_FAST = 2048, SEG_FB = SEG_FAST / SEG_SB;  // (blocks of 64 segments)
constexpr uint32_t SEG_SMEM_SERIAL = 2 * SEG_SB * 2 * SEG_CAND * 8;  // the serial stitch's tables (128 KB)
constexpr uint32_t SEG_SMEM_FAST = SEG_FAST * SEG_CAND + SEG_FB * SEG_CAND + SEG_FB + SEG_FAST;
constexpr uint32_t SEG_SMEM = SEG_SMEM_SERIAL > SEG_SMEM_FAST ? SEG_SMEM_SERIAL : SEG_SMEM_FAST;
static_assert(SEG_SMEM + 64 <= 160 * 1024, "seg_stitch LDS");
__global__ __launch_bounds__(SEG_STB) void seg_stitch(DecodeParams P, SegRange R) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[SEG_SMEM];
  __shared__ uint32_t bad, idx0;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const TileGeo G = seg_geo(P, R.s);
  if (R.nidx && R.nseg <= SEG_FAST) {
    const uint32_t ns = (uint32_t)R.nseg, nb = (ns + SEG_SB - 1) / SEG_SB;
    uint8_t *nx = smem;                            // [ns][64]
    uint8_t *bend = smem + SEG_FAST * SEG_CAND;    // [nb][64]: block start candidate -> next block's
    uint8_t *bst = bend + SEG_FB * SEG_CAND;       // [nb]: the chain's candidate at each block start
    uint8_t *sidx = bst + SEG_FB;                  // [ns]: the chain's candidate in each segment
    for (uint32_t i = tid; i < ns * SEG_CAND / 16; i += SEG_STB)
      reinterpret_cast<uint4 *>(nx)[i] = reinterpret_cast<const uint4 *>(R.nidx)[i];
    if (tid < WAVE) {  // segment 0's entry among its candidates
      const uint64_t e0 = R.seg_entry[0];
      const uint64_t hit = __ballot(R.cand[lane] == e0);
      if (tid == 0) {
        bad = !(is_pos(e0) && e0 < seg_end(G, R, 0) && hit);
        idx0 = hit ? (uint32_t)__builtin_ctzll(hit) : 0xFFu;
      }
    }
    __syncthreads();
    for (uint32_t p = tid; p < nb * SEG_CAND; p += SEG_STB) {  // each block's end map
      const uint32_t b = p / SEG_CAND, s1 = min(b * SEG_SB + SEG_SB, ns - 1);
      uint32_t x = p % SEG_CAND;
      for (uint32_t s = b * SEG_SB; s < s1 && x != 0xFFu; s++) x = nx[s * SEG_CAND + x];
      bend[p] = (uint8_t)x;
    }
    __syncthreads();
    if (tid == 0) {  // the blocks' entries, in order
      uint32_t x = bad ? 0xFFu : idx0;
      for (uint32_t b = 0; b < nb; b++) {
        bst[b] = (uint8_t)x;
        if (x != 0xFFu) x = bend[b * SEG_CAND + x];
      }
    }
    __syncthreads();
    if (tid < nb) {  // each block from its entry
      const uint32_t s0 = tid * SEG_SB, s1 = min(s0 + SEG_SB, ns);
      uint32_t x = bst[tid];
      for (uint32_t s = s0; s < s1; s++) {
        sidx[s] = (uint8_t)x;
        if (x == 0xFFu) {
          bad = 1;
          break;
        }
        if (s + 1 < ns) x = nx[s * SEG_CAND + x];
      }
    }
    __syncthreads();
    if (!bad) {
      for (uint32_t s = tid; s < ns; s += SEG_STB) {
        const uint32_t x = sidx[s];
        if (R.seg_lane) R.seg_lane[s] = (uint8_t)x;
        R.seg_entry[s] = R.cand[(uint64_t)s * 2 * SEG_CAND + x];
        if (s == ns - 1) R.seg_entry[ns] = R.cand[(uint64_t)s * 2 * SEG_CAND + SEG_CAND + x];
      }
      return;
    }
    __syncthreads();  // (the serial stitch reuses the LDS)
  }
  if (R.seg_lane)  // (the serial stitch: seg_claims walks every segment)
    for (uint64_t s = tid; s < R.nseg; s += SEG_STB) R.seg_lane[s] = 0xFF;
  auto tab = reinterpret_cast<uint64_t (*)[SEG_SB][2 * SEG_CAND]>(smem);  // [2][SEG_SB][128]: 2 x 64 KB
  constexpr uint32_t W = SEG_SB * 2 * SEG_CAND;  // words per block
  // threads [t0, SEG_STB) copy block blk into buffer buf
  auto load = [&](uint64_t blk, uint32_t buf, uint32_t t0) {
    const uint64_t w0 = blk * W, wn = umin64(R.nseg * 2 * SEG_CAND, w0 + W);
    for (uint64_t w = w0 + (tid - t0); w < wn; w += SEG_STB - t0) (&tab[buf][0][0])[w - w0] = R.cand[w];
  };
  const uint64_t nblk = (R.nseg + SEG_SB - 1) / SEG_SB;
  load(0, 0, 0);
  __syncthreads();
  uint64_t e = R.seg_entry[0];
  for (uint64_t blk = 0; blk < nblk; blk++) {
    const uint32_t cur = (uint32_t)(blk & 1);
    if (tid >= WAVE) {
      if (blk + 1 < nblk) load(blk + 1, cur ^ 1u, WAVE);  // (the other waves: the next block)
    } else {
      for (uint32_t k = 0; k < SEG_SB; k++) {
        const uint64_t seg = blk * SEG_SB + k;
        if (seg >= R.nseg) break;
        const uint64_t send = seg_end(G, R, seg);
        if (lane == 0) R.seg_entry[seg] = e;
        if (!is_pos(e) || e >= send) continue;  // the chain ended, or jumps over the segment
        const uint64_t hit = __ballot(tab[cur][k][lane] == e);
        if (hit) {
          e = tab[cur][k][SEG_CAND + (uint32_t)__builtin_ctzll(hit)];
          continue;
        }
        uint64_t p = e;  // not a candidate: walk it (one lane, headers from HBM)
        if (lane == 0) {
          while (p < send && p < G.se) {
            const Hdr h = hdr_global(P.bytes, p, G.se);
            if (h.kind != H_VALID) {
              p = term_of(h, p);
              break;
            }
            p = h.succ;
          }
        }
        e = readlane64(p, 0);
      }
    }
    __syncthreads();  // (the next block is staged; this one's reads are done)
  }
  if (tid == 0) R.seg_entry[R.nseg] = e;
}

// Per tile the chain also gives exact per-thread records (entry byte, frames, change frames), so
// the verify pass after the repair proves such a tile from its records alone (verify_lite) instead
// of re-walking it; a tile where the chain ends (an error or a frame cut by the stream end) keeps
// its records and is re-walked by verify_counts.
__global__ __launch_bounds__(NT) void seg_claims(DecodeParams P, SegRange R) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[IMG + 32];
  __shared__ uint64_t lcl[SEG_GMAX];
  __shared__ uint64_t nxt;
  __shared__ uint8_t re[NT], rn[NT], rc[NT];
  __shared__ uint32_t rok;
  const uint32_t tid = threadIdx.x;
  const uint64_t seg = blockIdx.x;
  if (R.ctile && R.seg_lane[seg] != 0xFF) return;  // (seg_claims_par's)
  TileGeo G = seg_geo(P, R.s);
  const uint64_t ta = R.t0 + seg * R.G, tb = umin64(ta + R.G, R.tl), send = seg_end(G, R, seg);
  for (uint64_t i = tid; i < tb - ta; i += NT) lcl[i] = C_ID;
  const uint64_t t_wg = P.stats && tid == 0 ? __builtin_amdgcn_s_memtime() : 0;  // (DRP_STATS)
  uint64_t c_walk = 0, n_walk = 0, n_tiles = 0;
  uint64_t p = R.seg_entry[seg];
  if (tid == 0) nxt = (is_pos(p) && p < send) ? p : NONE;
  bsync();
  uint4 pv[SEGB / 16], ph;
  uint64_t pa = NONE;  // the tile prefetched into pv / ph
  for (;;) {
    const uint64_t q = nxt;
    if (q == NONE) break;
    const uint64_t u = ta + (q - seg_tile_a(G, ta)) / TILE;
    G.A = seg_tile_a(G, u);
    re[tid] = 0xFF;
    rn[tid] = 0;
    rc[tid] = 0;
    if (G.A == pa) put_image(buf, pv, ph);  // (its barrier also orders the record resets)
    else stage(P, G, buf);
    // the next tile into registers while thread 0 walks this one (the chain usually goes on there)
    {
      TileGeo Gn = G;
      Gn.A = G.A + TILE;
      pa = Gn.A < send ? Gn.A : NONE;
      if (pa != NONE) load_image(P, Gn, pv, ph);
    }
    if (tid == 0) {
      const Img m{buf, P.bytes, G.A, G.se};
      const uint64_t lim = umin64(G.A + TILE, send);
      uint32_t ok = 1;
      const uint64_t t_w = P.stats ? __builtin_amdgcn_s_memtime() : 0;
      p = q;
      // seg_advance, keeping the records of the chain's frames in this tile: positions rise, so
      // the current thread's record is kept in registers and written once when the chain leaves
      // its bytes (LDS writes only: no read-modify-write on the walk's serial path)
      uint32_t cth = NT, ce = 0, cn = 0, cc = 0;
      // 32-bit tile-relative steps while the header's 16-byte window lies in the image and the
      // stream and its varint has 1..3 bytes (hdr_fast's grammar); any other header takes hdr_fast.
      // The step is written without data-dependent branches: the conditions are combined with &
      // and the records are stored on every frame (the last store of a thread's record is its
      // final value)
      {
        const uint32_t lr = (uint32_t)(lim - G.A);  // (q is in [A, lim))
        const uint32_t wr = (uint32_t)umin64(G.se - G.A, IMG), sr = (uint32_t)umin64(G.se - G.A, 0x7FFFFFFFull);
        uint32_t o = (uint32_t)(p - G.A);
        bool term = false, far = false;
        while (o < lr) {
          // (o in a vector register: otherwise the compiler moves this one-lane walk to the scalar
          // unit, which the CU's ~8 walking workgroups share: ~800 cycles per frame)
          asm volatile("" : "+v"(o));
          const uint32_t *qw = reinterpret_cast<const uint32_t *>(buf) + (o >> 2);  // (o < TILE: inside buf)
          const uint32_t w = __builtin_amdgcn_alignbit(qw[1], qw[0], (o & 3u) * 8u);
          const uint32_t tm = ~w & 0x808080u;
          const uint32_t k = ((uint32_t)__builtin_ctz(tm | 0x80000000u) >> 3) + 1u;
          const uint32_t L = ((w & 0x7Fu) | ((w >> 1) & 0x3F80u) | ((w >> 2) & 0x1FC000u)) & ((1u << (7u * k)) - 1u);
          uint32_t id = (w >> (8u * (k & 3u))) & 0xFFu;
          const bool fast = (o + 16u <= wr) & (tm != 0u) & (id < 3u) & ((id == 0u) | ((L != 0u) & (L <= sr - o - k)));
          uint32_t no = o + k + (id ? L : 1u);
          if (__builtin_expect(!fast, 0)) {
            const Hdr h = hdr_fast(m, G.A + o);
            if (h.kind != H_VALID) {
              p = term_of(h, G.A + o);
              ok = 0;
              term = true;
              break;
            }
            id = h.id;
            far = h.succ >= lim;
            p = h.succ;
            no = far ? lr : (uint32_t)(h.succ - G.A);
          }
          const uint32_t th = o / SEGB;
          const bool nw = th != cth;
          ce = nw ? o % SEGB : ce;
          cn = (nw ? 0u : cn) + (id != 0u);
          cc = (nw ? 0u : cc) + (id == 1u);
          cth = th;
          re[th] = (uint8_t)ce;
          rn[th] = (uint8_t)cn;
          rc[th] = (uint8_t)cc;
          o = no;
        }
        if (!term && !far) p = G.A + o;
      }
      if (P.stats) {
        c_walk += __builtin_amdgcn_s_memtime() - t_w;
        n_tiles++;
      }
      if (cth < NT) {
        re[cth] = (uint8_t)ce;
        rn[cth] = (uint8_t)cn;
        rc[cth] = (uint8_t)cc;
      }
      // the tile's claim: the first chain position past it, or where the chain ends in it
      lcl[u - ta] = (p & MARK_TERM) ? (p & ~M_ERR) : p;
      rok = ok && lim == G.A + TILE;  // (a segment end inside the tile: its next segment walks the rest)
      nxt = (is_pos(p) && p < send) ? p : NONE;
    }
    bsync();
    if (rok) {
      const uint64_t ix = u * NT + tid;
      P.ent[ix] = re[tid];
      P.ent_n[ix] = rn[tid];
      P.ent_c[ix] = rc[tid];
    }
    bsync();  // (the records are read before the next tile resets them)
  }
  for (uint64_t i = tid; i < tb - ta; i += NT) P.claim[ta + i] = lcl[i];
  if (P.stats && tid == 0) {  // (DRP_STATS: walk cycles, frames walked, tiles, workgroup cycles)
    atomicAdd(&P.stats[61], (unsigned long long)c_walk);
    atomicAdd(&P.stats[62], (unsigned long long)n_walk);
    atomicAdd(&P.stats[63], (unsigned long long)n_tiles);
    atomicAdd(&P.stats[55], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_wg));
  }
}

// seg_claims for the segments whose exact chain is one of seg_walk's candidates (seg_lane): every
// tile of the range at once, one lane per tile, from that candidate's position entering the tile
// (seg_walk's ctile) through the tile's headers in L2 / HBM, the thread records gathered in LDS
// per wave and written out coalesced. The serial seg_claims walked each segment's ~100 tiles one
// after another in ~2300 workgroups (the LDS per staged tile bounds them).
__global__ __launch_bounds__(WAVE) void seg_claims_par(DecodeParams P, SegRange R) {
  __shared__ uint32_t rec[3][WAVE][NT / 4];  // entry byte, frames, change frames of each thread (24 KB)
  const uint32_t lane = threadIdx.x;
  const uint64_t i = (uint64_t)blockIdx.x * WAVE + lane, n = R.tl - R.t0;
  const uint64_t u = R.t0 + i, seg = i < n ? i / R.G : 0;
  const uint32_t x = i < n ? R.seg_lane[seg] : 0xFFu;
  for (uint32_t w = 0; w < NT / 4; w++) {
    rec[0][lane][w] = 0xFFFFFFFFu;
    rec[1][lane][w] = 0;
    rec[2][lane][w] = 0;
  }
  bool rok = false;
  if (x != 0xFFu) {
    const TileGeo G = seg_geo(P, R.s);
    const uint64_t A = seg_tile_a(G, u), send = seg_end(G, R, seg), sb = seg_tile_a(G, R.t0 + seg * R.G);
    const uint32_t c = R.ctile[i * SEG_CAND + x];
    uint64_t cl = C_ID;
    if (c < CT_PAST && sb + c < A + TILE) {  // (else no chain position in the tile: identity)
      const uint64_t lim = umin64(A + TILE, send);
      uint64_t p = sb + c;
      uint32_t ok = 1;
      uint8_t *r0 = reinterpret_cast<uint8_t *>(rec[0][lane]), *r1 = reinterpret_cast<uint8_t *>(rec[1][lane]),
              *r2 = reinterpret_cast<uint8_t *>(rec[2][lane]);
      uint32_t cth = NT, ce = 0, cn = 0, cc = 0;
      while (is_pos(p) && p < lim && p < G.se) {
        const Hdr h = hdr_global(P.bytes, p, G.se);
        if (h.kind != H_VALID) {
          p = term_of(h, p);
          ok = 0;
          break;
        }
        const uint32_t o = (uint32_t)(p - A), th = o / SEGB;
        const bool nw = th != cth;
        ce = nw ? o % SEGB : ce;
        cn = (nw ? 0u : cn) + (h.id != 0u);
        cc = (nw ? 0u : cc) + (h.id == 1u);
        cth = th;
        r0[th] = (uint8_t)ce;
        r1[th] = (uint8_t)cn;
        r2[th] = (uint8_t)cc;
        p = h.succ;
      }
      cl = (p & MARK_TERM) ? (p & ~M_ERR) : p;
      rok = ok && lim == A + TILE;  // (the stream's last tile keeps its records: verify re-walks it)
    }
    P.claim[u] = cl;
  }
  // the walked tiles' records, a tile at a time by the whole wave (128 B per array per tile)
  uint64_t rm = __ballot(rok);
  while (rm) {
    const uint32_t j = (uint32_t)__builtin_ctzll(rm);
    rm &= rm - 1;
    const uint64_t uj = R.t0 + (uint64_t)blockIdx.x * WAVE + j;
    if (lane < NT / 4) {
      reinterpret_cast<uint32_t *>(P.ent + uj * NT)[lane] = rec[0][j][lane];
      reinterpret_cast<uint32_t *>(P.ent_n + uj * NT)[lane] = rec[1][j][lane];
      reinterpret_cast<uint32_t *>(P.ent_c + uj * NT)[lane] = rec[2][j][lane];
    }
  }
}

// payload bytes of the blob rows among rows [0, n) (a host batch's blob share: drp_api.hip
// stages the next batches in pieces when blobs dominate)
__global__ __launch_bounds__(256) void blob_bytes_kernel(const uint8_t *type, const uint32_t *plen, uint64_t n,
                                                         uint64_t *out) {
  uint64_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    if ((type[i] & 0x3Fu) == DRP_TYPE_BLOB) acc += plen[i];
  acc = wave_sum64(acc);
  if ((threadIdx.x & 63u) == 0 && acc) atomicAdd((unsigned long long *)out, (unsigned long long)acc);
}

// per-stream change / blob counts (one thread per stream)
__global__ void stream_counts_kernel(const uint64_t *tile_prefix, uint64_t nstreams, const uint64_t *count,
                                     const uint64_t *base, const uint64_t *nch, const uint64_t *nch_base,
                                     uint64_t *scount, uint32_t *total) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams) return;
  if (total && s == nstreams - 1) {  // frames of the whole call (the host's density estimate)
    const uint64_t nt = tile_prefix[nstreams];
    const uint64_t f = nt ? base[nt - 1] + count[nt - 1] : 0;
    *total = f > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)f;
  }
  const uint64_t tf = tile_prefix[s], tl = tile_prefix[s + 1];
  uint64_t ch = 0, fr = 0;
  if (tl > tf) {
    ch = nch_base[tl - 1] + nch[tl - 1] - nch_base[tf];
    fr = base[tl - 1] + count[tl - 1] - base[tf];
  }
  scount[2 * s] = ch;
  scount[2 * s + 1] = fr - ch;
}

// tile -> stream (one thread per tile; binary search over tile_prefix)
__global__ void tile_stream_kernel(const uint64_t *tile_prefix, uint64_t nstreams, uint64_t nt_max,
                                   uint32_t *tile_stream) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nt_max) return;
  const uint64_t ntiles = tile_prefix[nstreams];
  if (t >= ntiles) return;
  uint64_t lo = 0, hi = nstreams;
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (tile_prefix[mid] <= t) lo = mid; else hi = mid;
  }
  tile_stream[t] = (uint32_t)lo;
}

}  // namespace spec
}  // namespace drp

using namespace drp;

extern "C" hipError_t drp_launch_tile_scan(const uint64_t *in, const uint64_t *tile_prefix, uint64_t nstreams,
                                           uint64_t nt_max, uint64_t *tmp, uint64_t *out, uint64_t cap,
                                           uint32_t *overflow, hipStream_t st) {
  if (nt_max == 0) return hipSuccess;
  const uint32_t nb = (uint32_t)((nt_max + spec::SCAN_SPAN - 1) / spec::SCAN_SPAN);
  if (nb == 1) {  // (small batches: one launch; a staged piece pays each launch's host cost)
    hipLaunchKernelGGL(spec::scan_down<true>, dim3(1), dim3(spec::SCAN_BLK), 0, st, in, tile_prefix, nstreams,
                       (const uint64_t *)tmp, out, cap, overflow);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(spec::scan_reduce, dim3(nb), dim3(spec::SCAN_BLK), 0, st, in, tile_prefix, nstreams, tmp);
  hipLaunchKernelGGL(spec::scan_top, dim3(1), dim3(spec::SCAN_BLK), 0, st, tmp, (uint64_t)nb);
  hipLaunchKernelGGL(spec::scan_down<false>, dim3(nb), dim3(spec::SCAN_BLK), 0, st, in, tile_prefix, nstreams,
                     (const uint64_t *)tmp, out, cap, overflow);
  return hipGetLastError();
}

extern "C" hipError_t drp_launch_stream_counts(const uint64_t *tile_prefix, uint64_t nstreams, const uint64_t *count,
                                               const uint64_t *base, const uint64_t *nch, const uint64_t *nch_base,
                                               uint64_t *scount, hipStream_t st, uint32_t *total) {
  if (nstreams == 0) return hipSuccess;
  const uint32_t blk = 256;
  hipLaunchKernelGGL(spec::stream_counts_kernel, dim3((uint32_t)((nstreams + blk - 1) / blk)), dim3(blk), 0, st,
                     tile_prefix, nstreams, count, base, nch, nch_base, scount, total);
  return hipGetLastError();
}

extern "C" uint32_t drp_spec_tile_bytes(void) { return spec::TILE; }
extern "C" uint32_t drp_spec_rec_words(void) { return spec::CR_TILE_WORDS; }  // (per tile: fast_records)
extern "C" uint32_t drp_spec_retry_mask(void) { return spec::F_MISS | spec::F_WAIT; }

extern "C" uint32_t drp_spec_miss_bit(void) { return spec::F_MISS; }
extern "C" uint32_t drp_spec_cascade_bit(void) { return spec::F_CASCADE; }

// Claims and verification only (the host checks the prediction before anything is emitted).
extern "C" void drp_dbg_mark(const char *name, hipStream_t st);  // (drp_api.hip: DRP_WATCHDOG)

extern "C" hipError_t drp_launch_spec_head(const DecodeParams *P, uint64_t nt_max, uint64_t nstreams,
                                           uint32_t *tile_stream, hipStream_t st) {
  if (nt_max == 0) return hipSuccess;
  DecodeParams Q = *P;
  Q.tile_stream = nullptr;
  if (nstreams > 1) {
    const uint32_t blk = 256;
    hipLaunchKernelGGL(spec::tile_stream_kernel, dim3((uint32_t)((nt_max + blk - 1) / blk)), dim3(blk), 0, st,
                       P->tile_prefix, nstreams, nt_max, tile_stream);
    drp_dbg_mark("tile_stream_kernel", st);
    Q.tile_stream = tile_stream;
  }
  // interior tiles in the fast form (or by the region walkers); the edge and dense tiles they list
  // in the general one
  if (Q.walk_rp && Q.walk_hop == 2u) {
    // the claims form of a large batch, per launch: a density sample from the streams' exact
    // entries (one small kernel and a 16-byte read back): sparse streams (> HOP_FRAME bytes per
    // frame) take the hop walkers, dense ones claims_fast
    unsigned long long d[2] = {0, 0};
    hipError_t e = drp_launch_walk_density(&Q, st);
    if (e == hipSuccess) e = hipMemcpyAsync(d, Q.walk_dense, 16, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    if (d[0] > (unsigned long long)spec::HOP_FRAME * d[1]) {
      Q.walk_hop = 1u;
      Q.walk_tpr = drp_walk_tiles_per_region(nt_max, 1);  // (the hop walkers' region count)
    } else {
      Q.walk_rp = nullptr;
    }
  }
  if (Q.walk_rp) {
    const hipError_t e = drp_launch_claims_walk(&Q, nt_max, st);
    if (e != hipSuccess) return e;
    drp_dbg_mark("claims_walk", st);
  } else {
    const uint64_t g = nt_max;
    const bool cf = Q.change_checks && !P->walk_rp;
    if (cf && Q.rec)
      hipLaunchKernelGGL((spec::claims_fast<true, true>), dim3((uint32_t)g), dim3(spec::NT), 0, st, Q);
    else if (cf)
      hipLaunchKernelGGL((spec::claims_fast<true, false>), dim3((uint32_t)g), dim3(spec::NT), 0, st, Q);
    else if (Q.rec)
      hipLaunchKernelGGL((spec::claims_fast<false, true>), dim3((uint32_t)g), dim3(spec::NT), 0, st, Q);
    else
      hipLaunchKernelGGL((spec::claims_fast<false, false>), dim3((uint32_t)g), dim3(spec::NT), 0, st, Q);
  }
  drp_dbg_mark("claims_fast", st);
  const uint32_t gw = (uint32_t)(nt_max < 16384 ? nt_max : 16384);
  hipLaunchKernelGGL(spec::spec_claims, dim3(gw), dim3(spec::NT), 0, st, Q);
  drp_dbg_mark("spec_claims", st);
  if (const char *dump = getenv("DRP_DUMP_CLAIMS")) {  // (debugging: the claims kernels' output)
    uint64_t ntl = 0;
    (void)hipStreamSynchronize(st);
    (void)hipMemcpy(&ntl, Q.tile_prefix + nstreams, 8, hipMemcpyDeviceToHost);
    std::vector<uint64_t> cl(ntl);
    std::vector<uint8_t> en(ntl * 128 * 3);
    (void)hipMemcpy(cl.data(), Q.claim, ntl * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(en.data(), Q.ent, ntl * 128, hipMemcpyDeviceToHost);
    (void)hipMemcpy(en.data() + ntl * 128, Q.ent_n, ntl * 128, hipMemcpyDeviceToHost);
    (void)hipMemcpy(en.data() + 2 * ntl * 128, Q.ent_c, ntl * 128, hipMemcpyDeviceToHost);
    if (FILE *f = fopen(dump, "ab")) {
      fwrite(&ntl, 8, 1, f);
      fwrite(cl.data(), 8, ntl, f);
      fwrite(en.data(), 1, ntl * 128 * 3, f);
      fclose(f);
    }
  }
  if (Q.vlist) {  // records-only verification, then verify_counts on the tiles it lists
    const uint64_t nb = (nt_max * spec::VL_G + spec::VL_BLK - 1) / spec::VL_BLK;
    hipLaunchKernelGGL(spec::verify_lite, dim3((uint32_t)nb), dim3(spec::VL_BLK), 0, st, Q);
    drp_dbg_mark("verify_lite", st);
    hipLaunchKernelGGL(spec::verify_counts, dim3((uint32_t)(nt_max < 16384 ? nt_max : 16384)), dim3(spec::NT), 0, st,
                       Q);
    drp_dbg_mark("verify_counts", st);
  } else {
    hipLaunchKernelGGL(spec::verify_counts, dim3((uint32_t)nt_max), dim3(spec::NT), 0, st, Q);
    drp_dbg_mark("verify_counts", st);
  }
  return hipGetLastError();
}

// One more verify pass over the repaired claims (the caller clears incl_e and the flags first).
extern "C" hipError_t drp_launch_spec_verify(const DecodeParams *P, uint64_t nt_max, uint64_t nstreams,
                                             uint32_t *tile_stream, hipStream_t st) {
  if (nt_max == 0) return hipSuccess;
  DecodeParams Q = *P;
  Q.tile_stream = nstreams > 1 ? tile_stream : nullptr;
  if (Q.vlist) {  // records-only verification, verify_counts on the tiles it lists (caller zeroes vlist_n)
    const uint64_t nb = (nt_max * spec::VL_G + spec::VL_BLK - 1) / spec::VL_BLK;
    hipLaunchKernelGGL(spec::verify_lite, dim3((uint32_t)nb), dim3(spec::VL_BLK), 0, st, Q);
    drp_dbg_mark("verify_lite", st);
    hipLaunchKernelGGL(spec::verify_counts, dim3((uint32_t)(nt_max < 16384 ? nt_max : 16384)), dim3(spec::NT), 0, st,
                       Q);
    drp_dbg_mark("verify_counts", st);
  } else {
    hipLaunchKernelGGL(spec::verify_counts, dim3((uint32_t)nt_max), dim3(spec::NT), 0, st, Q);
    drp_dbg_mark("verify_counts", st);
  }
  return hipGetLastError();
}

// A repair pass over the tiles the previous pass listed (P->vlist / P->vlist_n: its dirty list,
// n entries), appending to P->dlist.
extern "C" hipError_t drp_launch_spec_verify_list(const DecodeParams *P, uint64_t n, uint64_t nstreams,
                                                  uint32_t *tile_stream, hipStream_t st) {
  if (n == 0) return hipSuccess;  // (n = ~0: the count is on the device only)
  DecodeParams Q = *P;
  Q.tile_stream = nstreams > 1 ? tile_stream : nullptr;
  const uint64_t g = n == ~0ull ? 1024 : (n < 16384 ? n : 16384);
  hipLaunchKernelGGL(spec::verify_counts, dim3((uint32_t)g), dim3(spec::NT), 0, st, Q);
  drp_dbg_mark("verify_counts", st);
  return hipGetLastError();
}

// Everything after verification: output bases, emission, change-count bases, stream counts.
extern "C" hipError_t drp_launch_spec_tail(const DecodeParams *P, uint64_t nt_max, uint64_t nstreams,
                                           uint32_t *tile_stream, uint64_t *scan_tmp, hipStream_t st) {
  if (nt_max == 0) return hipSuccess;
  DecodeParams Q = *P;
  Q.tile_stream = nstreams > 1 ? tile_stream : nullptr;
  hipError_t e = drp_launch_tile_scan(Q.tile_count, Q.tile_prefix, nstreams, nt_max, scan_tmp, Q.tile_base, Q.cap,
                                      Q.overflow, st);
  if (e != hipSuccess) return e;
  drp_dbg_mark("tile_scan(count)", st);
  if (Q.vlist) {  // the fast kernel, then the general one on the tiles it lists
    e = hipMemsetAsync(Q.vlist_n, 0, 4, st);
    if (e != hipSuccess) return e;
    if (spec::SP_FRAMES && Q.tile_sparse) {  // sparse tiles first (no staging), then every other tile
      hipLaunchKernelGGL(spec::emit_sparse, dim3((uint32_t)((nt_max + spec::SP_TPB - 1) / spec::SP_TPB)), dim3(256),
                         0, st, Q);
      drp_dbg_mark("emit_sparse", st);
    } else {
      Q.tile_sparse = nullptr;
    }
    if (Q.rec)  // (the tiles with records; emit_lean skips them)
    {
      hipLaunchKernelGGL(spec::chunk_tiles, dim3((uint32_t)((nt_max + 255) / 256)), dim3(256), 0, st, Q);
      const uint64_t nchunks = (Q.cap + 63) / 64;
      hipLaunchKernelGGL(spec::emit_recs, dim3((uint32_t)((nchunks + spec::ER_WAVES - 1) / spec::ER_WAVES)),
                         dim3(spec::ER_WAVES * WAVE), 0, st, Q);
    }
    hipLaunchKernelGGL(spec::emit_lean,
                       dim3((uint32_t)(Q.change_checks || Q.rec ? (nt_max + spec::EMIT_LONG_TPW - 1) / spec::EMIT_LONG_TPW
                                                                : nt_max)),
                       dim3(spec::NT), 0, st, Q);
    drp_dbg_mark("emit_fast", st);
    hipLaunchKernelGGL(spec::emit_tiles, dim3((uint32_t)(nt_max < 16384 ? nt_max : 16384)), dim3(spec::NT), 0,
                       st, Q);
    drp_dbg_mark("emit_tiles", st);
  } else {
    Q.vlist = nullptr;  // every tile in the general form
    hipLaunchKernelGGL(spec::emit_tiles, dim3((uint32_t)nt_max), dim3(spec::NT), 0, st, Q);
    drp_dbg_mark("emit_tiles", st);
  }
  e = drp_launch_tile_scan(Q.tile_nch, Q.tile_prefix, nstreams, nt_max, scan_tmp, Q.tile_nch_base, ~0ull, Q.overflow, st);
  if (e != hipSuccess) return e;
  drp_dbg_mark("tile_scan(nch)", st);
  return drp_launch_stream_counts(Q.tile_prefix, nstreams, Q.tile_count, Q.tile_base, Q.tile_nch, Q.tile_nch_base,
                                  Q.scount, st, Q.counter + 3);
}

extern "C" hipError_t drp_launch_blob_bytes(const uint8_t *type, const uint32_t *plen, uint64_t n, uint64_t *out,
                                            hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint64_t nb = (n + 255) / 256;
  hipLaunchKernelGGL(spec::blob_bytes_kernel, dim3((uint32_t)(nb < 1024 ? nb : 1024)), dim3(256), 0, st, type, plen, n,
                     out);
  return hipGetLastError();
}

// Segmented repair of stream s from tile t0 (its first missed tile) to its end (the caller then
// runs a verify pass). scratch: 2 * 64 * SEG_NMAX + SEG_NMAX + 1 words.
extern "C" hipError_t drp_launch_seg_repair(const DecodeParams *P, uint64_t s, uint64_t t0, uint64_t tl,
                                            uint64_t *scratch, uint32_t *ctile, uint64_t ctile_cap, hipStream_t st) {
  if (tl <= t0) return hipSuccess;
  spec::SegRange R;
  R.s = s;
  R.t0 = t0;
  R.tend = tl;
  // at most SEG_NMAX segments of SEG_GMAX tiles (64 GiB of 8 KiB tiles): a longer range is repaired
  // up to there; the verify passes that follow prove the claims past it as before (or fall back).
  // Short segments: a candidate chain walks only its segment (the SIMD's cost is its densest
  // chain), and the segments fill the CUs several workgroups deep.
  const uint64_t n = tl - t0 < spec::SEG_NMAX * spec::SEG_GMAX ? tl - t0 : spec::SEG_NMAX * spec::SEG_GMAX;
  R.tl = t0 + n;
  // ~SEG_NTARGET segments: fewer make each workgroup's walk longer, more make the serial stitch
  // longer (1.7 GB dense cascade: 8192 segments stitch in 1.8 ms)
  const uint64_t g = std::min<uint64_t>((n + spec::SEG_NTARGET - 1) / spec::SEG_NTARGET, spec::SEG_GMAX);
  R.G = g > spec::SEG_GMIN ? g : spec::SEG_GMIN;  // (n <= SEG_NMAX * SEG_GMAX: at most SEG_NMAX segments)
  R.nseg = (n + R.G - 1) / R.G;
  R.cand = scratch;
  R.seg_entry = scratch + 2 * spec::SEG_CAND * spec::SEG_NMAX;
  R.nidx = reinterpret_cast<uint8_t *>(R.seg_entry + spec::SEG_NMAX + 2);  // (SEG_NMAX x 64 B, 16-B aligned)
  R.seg_lane = reinterpret_cast<uint8_t *>(R.seg_entry + spec::SEG_NMAX + 2) + spec::SEG_NMAX * spec::SEG_CAND;
  // (the parallel seg_claims needs the stitch's tables and a position per candidate per tile)
  R.ctile = ctile && ctile_cap >= n * spec::SEG_CAND ? ctile : nullptr;
  DecodeParams Q = *P;
  if (Q.tile_rec) {  // (the repair rewrites these tiles' records: the region walkers' no longer apply)
    const hipError_t e = hipMemsetAsync(Q.tile_rec + t0, 0xFF, (tl - t0) * 4, st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(spec::seg_walk, dim3((uint32_t)R.nseg), dim3(spec::NT), 0, st, Q, R);
  hipLaunchKernelGGL(spec::seg_link, dim3((uint32_t)R.nseg), dim3(WAVE), 0, st, Q, R);
  hipLaunchKernelGGL(spec::seg_stitch, dim3(1), dim3(spec::SEG_STB), 0, st, Q, R);
  if (R.ctile) hipLaunchKernelGGL(spec::seg_claims_par, dim3((uint32_t)((n + WAVE - 1) / WAVE)), dim3(WAVE), 0, st, Q, R);
  hipLaunchKernelGGL(spec::seg_claims, dim3((uint32_t)R.nseg), dim3(spec::NT), 0, st, Q, R);
  return hipGetLastError();
}
