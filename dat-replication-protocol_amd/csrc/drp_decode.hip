// drp_decode.hip — gfx950 decode of varint-length-prefixed multibuffer streams into a
// frame table + Change SoA columns. Replaces the per-frame loop of decode.js
// (Decoder._consume / _onheader / _onchangedata / _onchangeend / _onblobdata,
// decode.js:144-262) and messages.Change.decode (messages/index.js:5).
//
// Algorithm:
//   * One wave (64 lanes) owns one tile of 64*B stream bytes, staged once into LDS.
//     Tiles are handed out by an atomic counter, so every tile a wave waits on has
//     already been taken by a running wave (no deadlock, any grid size).
//   * Lane l owns B bytes. It finds every position whose bytes form a complete header
//     with id <= 2 (bit masks over its bytes), and for each such "live" position computes
//     the lane-local chain function F(p) = (first chain position past the lane, #nodes,
//     #delivered frames) by one descending pass.
//   * A frame chain through the tile is then walked one LANE per step (<= 64 steps),
//     with the per-lane functions read by readlane.
//   * The tile's entry depends on the previous tile's chain (frames have no sync marker).
//     Each tile publishes a speculative exit y (the chain of its best-evidenced candidate
//     entry) and looks back over predecessors: x_t = f_{t-1}(...f_k(x_k)) with
//     f_k(x) = x >= end_k ? x : y_k. With x known it walks its exact chain, checks it
//     against its own y (a mismatch is recorded; the host re-runs from the first such
//     tile with the corrected exit), publishes its exact exit and its frame count, and a
//     second look-back over counts gives its first output slot.
//   * Frames are listed in LDS and decoded round-robin over lanes, so each column store
//     of a wave is one contiguous run.
#include "drp_device.h"
#include "drp_kernels.h"

namespace drp {

constexpr int LMAX = 8;      // live positions per lane kept in registers
constexpr int CMAX = 48;     // speculative candidates tried per tile
constexpr uint32_t EVID = 8; // chain nodes that count as strong evidence
constexpr uint32_t HALO = 256;
constexpr uint32_t SPIN_MAX = 1u << 22;  // bounded waits: ~seconds, then flag and give up



__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

#ifdef DRP_KERNEL_TRACE
#define MARK(stage)                                                                   \
  do {                                                                                \
    if (lane == 0 && P.dbg)                                                           \
      __hip_atomic_store(P.dbg + blockIdx.x * 4, ((uint32_t)t << 8) | (uint32_t)(stage), \
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);                  \
  } while (0)
#else
#define MARK(stage) \
  do {              \
  } while (0)
#endif

// Per-lane chain functions F(p) for the live positions of the lane's B bytes.
struct LaneFns {
  uint32_t meta[LMAX];  // tile-relative pos (14b) | nodes (9b) << 14 | delivered (9b) << 23
  uint64_t ex[LMAX];    // first chain position past the lane, or MARK_TERM | terminal node
  uint32_t cnt, ovf;
};

struct TileCtx {
  const uint8_t *buf;  // LDS image of [A, A + TILE + HALO)
  uint64_t A, ve, se;
};

// F(E) for a wave-uniform E inside the tile: read from the owning lane's list by readlane;
// lanes that dropped positions (list full) are walked directly (uniform).
template <int B>
__device__ __forceinline__ void lane_lookup(const LaneFns &F, const TileCtx &T, uint64_t E, uint64_t &xo,
                                            uint32_t &ndo, uint32_t &dlo) {
  E = uniform64(E);
  const uint32_t prel = (uint32_t)(E - T.A);
  const uint32_t l = uniform32(prel / B);
  bool hit = false;
  uint64_t hx = 0;
  uint32_t hm = 0;
#pragma unroll
  for (int k = 0; k < LMAX; k++)
    if ((uint32_t)k < F.cnt && (F.meta[k] & 0x3FFFu) == prel) { hit = true; hx = F.ex[k]; hm = F.meta[k]; }
  const uint64_t hb = __ballot(hit);
  if ((hb >> l) & 1ull) {
    xo = readlane64(hx, l);
    const uint32_t m = readlane32(hm, l);
    ndo = (m >> 14) & 0x1FFu;
    dlo = m >> 23;
    return;
  }
  if (readlane32(F.ovf, l)) {
    const uint64_t le = umin64(T.A + (uint64_t)(l + 1) * B, T.ve);
    uint64_t cur = E;
    uint32_t nd = 0, dl = 0;
    for (;;) {
      Hdr h = parse_hdr_lds(T.buf, T.A, cur, T.se);
      nd++;
      if (h.kind != H_VALID) {
        dl += (h.kind == H_TAIL_BLOB) ? 1u : 0u;
        xo = MARK_TERM | cur;
        break;
      }
      dl += h.id != 0 ? 1u : 0u;
      cur = uniform64(h.succ);
      if (cur >= le) { xo = cur; break; }
    }
    ndo = uniform32(nd);
    dlo = uniform32(dl);
    return;
  }
  xo = MARK_TERM | E;  // not a live header: the chain ends here (error or tail)
  ndo = 1;
  dlo = 0;
}

// Walk the frame chain from the wave-uniform entry E through the tile, one lane per step.
// rec: lanes on the chain remember their entry (ent) and delivered count (mydl).
template <int B>
__device__ __forceinline__ uint64_t chain_walk(const LaneFns &F, const TileCtx &T, uint64_t E, bool rec,
                                               uint32_t lane, int32_t &ent, uint32_t &mydl, uint32_t &nodes,
                                               uint32_t &del) {
  nodes = 0;
  del = 0;
  E = uniform64(E);
  while (E < T.ve) {
    uint64_t x;
    uint32_t nd, dl;
    lane_lookup<B>(F, T, E, x, nd, dl);
    if (rec) {
      const uint32_t l = uniform32((uint32_t)((E - T.A) / B));
      if (lane == l) { ent = (int32_t)(E - T.A); mydl = dl; }
    }
    nodes = uniform32(nodes + nd);
    del = uniform32(del + dl);
    E = uniform64(x);
  }
  return E;
}

template <int B>
__global__ __launch_bounds__(64) void decode_tiles(DecodeParams P) {
  constexpr uint32_t TILE = 64u * B;
  constexpr uint32_t LBUF = TILE + HALO + 32;
  constexpr uint32_t FL_CAP = TILE / 8;
  constexpr int NW = (B + 16 + 63) / 64;  // 64-bit mask words per lane
  __shared__ __attribute__((aligned(16))) uint8_t buf[LBUF];
  constexpr uint32_t NBW = (TILE + HALO) / 64 + 2;  // bitmap words (+2 zero pad)
  __shared__ uint16_t flist[FL_CAP];
  __shared__ uint64_t mbits[NBW], sbits[NBW];

  const uint32_t lane = lane_id();
  const uint64_t ntiles = P.tile_prefix[P.nstreams];

  for (;;) {
    // Grab the next tile. Every lane executes the atomic (addend 1 on lane 0, 0 elsewhere):
    // a grab under `if (lane == 0)` let the structurizer split this loop so that its inner
    // back-edge skipped the grab and re-processed the same tile forever.
    const uint32_t tt = atomicAdd(P.counter, lane == 0 ? 1u : 0u);
    const uint64_t t = uniform32(readlane32(tt, 0));
    if (t >= ntiles) return;
    MARK(1);

    // ---- which stream / tile ---------------------------------------------------------
    uint64_t lo = 0, hi = P.nstreams;
    while (hi - lo > 1) {
      uint64_t mid = (lo + hi) >> 1;
      if (P.tile_prefix[mid] <= t) lo = mid; else hi = mid;
    }
    const uint64_t s = uniform64(lo);
    const uint64_t tf = P.tile_prefix[s];
    const uint64_t so = P.stream_off[s], se = P.stream_off[s + 1];
    const uint64_t A0 = so & ~(uint64_t)(TILE - 1);
    const uint64_t A = A0 + (t - tf) * TILE;
    const uint64_t vs = umax64(so, A), ve = umin64(se, A + TILE);
    const bool first = (t == tf);
    const uint64_t e0 = so + (P.entry ? P.entry[s] : 0ull);

    // ---- stage the tile (+halo) in LDS; build MSB / (byte <= 2) bitmaps on the way -------
    for (uint32_t i = lane * 16; i < TILE + HALO; i += 64 * 16) {
      const uint64_t p = A + i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (p + 16 <= se) {
        v = *reinterpret_cast<const uint4 *>(P.bytes + p);
      } else if (p < se) {
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < 16 && p + k < se; k++) w[k >> 2] |= (uint32_t)P.bytes[p + k] << (8 * (k & 3));
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
      *reinterpret_cast<uint4 *>(buf + i) = v;
      const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
      uint32_t hm16 = 0, sm16 = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t x = xs[j];
        const uint32_t hm = (x >> 7) & 0x01010101u;                                       // MSB set
        const uint32_t sm = (~((x & 0x7F7F7F7Fu) + 0x7D7D7D7Du) & ~x & 0x80808080u) >> 7;  // byte <= 2
        hm16 |= (((hm * 0x01020408u) >> 24) & 0xFu) << (4 * j);
        sm16 |= (((sm * 0x01020408u) >> 24) & 0xFu) << (4 * j);
      }
      reinterpret_cast<uint16_t *>(mbits)[i / 16] = (uint16_t)hm16;
      reinterpret_cast<uint16_t *>(sbits)[i / 16] = (uint16_t)sm16;
    }
    if (lane < 2) *reinterpret_cast<uint4 *>(buf + TILE + HALO + lane * 16) = make_uint4(0, 0, 0, 0);
    if (lane < 2) { mbits[NBW - 2 + lane] = 0; sbits[NBW - 2 + lane] = 0; }
    __syncthreads();

    MARK(2);
    // ---- lane-local live positions and chain functions ----------------------------------
    const uint64_t ls = A + (uint64_t)lane * B;
    const uint64_t lvs = umax64(ls, vs), lend = umin64(ls + B, ve);
    LaneFns F;
#pragma unroll
    for (int k = 0; k < LMAX; k++) { F.meta[k] = 0; F.ex[k] = 0; }
    F.cnt = 0;
    F.ovf = 0;
    uint32_t &cnt = F.cnt, &ovf = F.ovf;
    uint32_t *meta = F.meta;
    uint64_t *ex = F.ex;
    if (lvs < lend) {
      uint64_t M[NW], S[NW];
#pragma unroll
      for (int w = 0; w < NW; w++) {
        M[w] = mbits[lane * (B / 64) + w];
        S[w] = sbits[lane * (B / 64) + w];
      }
      // terminator t: MSB clear at t and byte t+1 <= 2  (bit t of ~M & (S >> 1))
      uint64_t T[NW];
#pragma unroll
      for (int w = 0; w < NW; w++) {
        uint64_t sh = (S[w] >> 1) | (w + 1 < NW ? (S[w + 1] << 63) : 0ull);
        T[w] = ~M[w] & sh;
      }
      // only terminators that can end a varint starting in [plo, phi)
      const uint32_t plo = (uint32_t)(lvs - ls), phi = (uint32_t)(lend - ls);
      const uint32_t tmax = phi + 9;  // exclusive
#pragma unroll
      for (int w = 0; w < NW; w++) {
        int b0 = w * 64;
        if ((uint32_t)b0 >= tmax) T[w] = 0;
        else if ((uint32_t)(b0 + 64) > tmax) T[w] &= (1ull << (tmax - b0)) - 1;
      }
      // descending over terminators, then over varint start positions
#pragma unroll
      for (int w = NW - 1; w >= 0; w--) {
        uint64_t tw = T[w];
        while (tw) {
          const int tb = 63 - __builtin_clzll(tw);
          tw &= ~(1ull << tb);
          const uint32_t tpos = (uint32_t)(w * 64 + tb);
          uint32_t p = tpos;
          for (;;) {
            if (p < phi && p >= plo && !ovf) {
              const uint64_t abs = ls + p;
              Hdr h = parse_hdr_lds(buf, A, abs, se);
              if (h.kind == H_VALID || h.kind == H_TAIL_BLOB || h.kind == H_TAIL_CHANGE ||
                  h.kind == H_ERR_LEN) {
                uint64_t exv;
                uint32_t nd, dl;
                if (h.kind != H_VALID) {
                  exv = MARK_TERM | abs;
                  nd = 1;
                  dl = (h.kind == H_TAIL_BLOB) ? 1u : 0u;
                } else {
                  dl = h.id != 0 ? 1u : 0u;
                  const uint64_t nx = h.succ;
                  if (nx >= lend) {
                    exv = nx;
                    nd = 1;
                  } else {
                    const uint32_t nrel = (uint32_t)(nx - A);
                    bool f = false;
                    uint64_t fx = 0;
                    uint32_t fm = 0;
#pragma unroll
                    for (int k = 0; k < LMAX; k++)
                      if ((uint32_t)k < cnt && (meta[k] & 0x3FFFu) == nrel) { f = true; fx = ex[k]; fm = meta[k]; }
                    if (f) {
                      exv = fx;
                      nd = 1 + ((fm >> 14) & 0x1FFu);
                      dl += fm >> 23;
                    } else {  // successor is a dead / incomplete header inside this lane
                      exv = MARK_TERM | nx;
                      nd = 2;
                    }
                  }
                }
                if (cnt < (uint32_t)LMAX) {
                  const uint32_t m = (uint32_t)(abs - A) | (umin64(nd, 511) << 14) | (umin64(dl, 511) << 23);
#pragma unroll
                  for (int k = 0; k < LMAX; k++)
                    if ((uint32_t)k == cnt) { meta[k] = m; ex[k] = exv; }
                  cnt++;
                } else {
                  ovf = 1;
                }
              }
            }
            if (p == 0 || p <= plo) break;
            const uint32_t q = p - 1;
            if (!((M[q >> 6] >> (q & 63)) & 1ull) || tpos - q + 1 > 10) break;
            p = q;
          }
        }
      }
    }

    MARK(3);
    // ---- chain walker: one lane per step ---------------------------------------------
    int32_t ent = -1;     // this lane's entry (tile-relative) on the recorded chain
    uint32_t mydl = 0;    // delivered frames of the recorded chain inside this lane
    const TileCtx TC{buf, A, ve, se};
    auto term_is_tail = [&](uint64_t x) -> bool {
      const uint64_t q = x & POS_MASK;
      if (q >= A + TILE) return false;
      Hdr h = parse_hdr_lds(buf, A, q, se);
      return h.kind == H_TAIL_HDR || h.kind == H_TAIL_CHANGE || h.kind == H_TAIL_BLOB;
    };

    // ---- entry: known, looked up early, overridden, or speculated -----------------------
    uint64_t x = 0, y = MARK_NONE;
    bool have_x = false, published = false;
    if (first) {
      x = e0;
      have_x = true;
    } else if (!P.strict) {
      const uint64_t v = ld_agent(&P.inclx[t - 1]);
      if (v) { x = v - 1; have_x = true; }
    }
    if (!have_x && !P.strict) {
      const uint64_t ov = P.yover ? P.yover[t] : 0ull;
      if (ov) {
        y = ov - 1;
      } else {
        // candidates in ascending position order; best = most evidence, earliest on ties
        uint64_t lanes_with = __ballot(cnt > 0);
        int64_t best = -1;
        uint32_t tried = 0;
        bool done = false;
        while (lanes_with && !done) {
          const uint32_t l = (uint32_t)__builtin_ctzll(lanes_with);
          lanes_with &= lanes_with - 1;
          const uint32_t cl = uniform32(readlane32(cnt, l));
          for (int32_t k = (int32_t)cl - 1; k >= 0 && !done; k--) {
            uint32_t msel = 0;
#pragma unroll
            for (int kk = 0; kk < LMAX; kk++) if (kk == k) msel = meta[kk];
            const uint64_t g = uniform64(A + (readlane32(msel, l) & 0x3FFFu));
            uint32_t nodes, del;
            const uint64_t xe = chain_walk<B>(F, TC, g, false, lane, ent, mydl, nodes, del);
            const bool survived = xe < MARK_TERM || (ve == se && term_is_tail(xe));
            if (survived) {
              bool validated = false;
              Hdr h = parse_hdr_lds(buf, A, g, se);
              if (h.kind == H_VALID && h.id == 1) {
                LdsReader rd{buf, A, umin64(A + TILE + HALO, se)};
                ChangeCols c = decode_change(rd, g + h.vlen + 1, h.L - 1);
                validated = (c.err == 0);
              }
              const int64_t score = (int64_t)nodes + (validated ? 1000 : 0);
              if (score > best) { best = score; y = xe; }
              if (nodes >= EVID || validated) done = true;
            }
            if (++tried >= (uint32_t)CMAX) done = true;
          }
        }
      }
      if (lane == 0) st_agent(&P.aggx[t], y + 1);
      published = true;
    }

    MARK(4);
    // ---- exit look-back ----------------------------------------------------------------
    if (!have_x) {
      for (uint32_t spin = 0;; spin++) {
        const int64_t pi = (int64_t)t - 1 - (int64_t)lane;
        const bool inr = pi >= (int64_t)tf;
        const uint64_t vi = inr ? ld_agent(&P.inclx[pi]) : 0ull;
        const uint64_t va = (inr && !P.strict) ? ld_agent(&P.aggx[pi]) : 0ull;
        const uint64_t im = __ballot(vi != 0);
        if (im) {
          const uint32_t ist = (uint32_t)__builtin_ctzll(im);
          const uint64_t am = __ballot(va != 0 && (va - 1) != MARK_NONE);
          const uint64_t need = (ist >= 64) ? ~0ull : ((1ull << ist) - 1);
          if ((am & need) == need) {
            uint64_t xv = readlane64(vi, ist) - 1;
            for (int32_t i = (int32_t)ist - 1; i >= 0; i--) {
              const uint64_t k = t - 1 - (uint64_t)i;
              const uint64_t ce_k = umin64(A0 + (k - tf + 1) * TILE, se);
              const uint64_t yk = readlane64(va, (uint32_t)i) - 1;
              if (xv < ce_k) xv = yk;
            }
            x = xv;
            break;
          }
        }
        if (spin > SPIN_MAX) {  // a predecessor never published: flag, end the chain here
          if (lane == 0) atomicOr(P.overflow, 2u);
          x = MARK_TERM | vs;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }

    MARK(5);
    // ---- exact chain through this tile ---------------------------------------------------
    x = uniform64(x);
    y = uniform64(y);
    uint64_t exit_t;
    uint32_t count_t = 0;
    if (x >= ve) {
      exit_t = x;  // pass-through (inside a long frame) or the chain already ended
    } else {
      uint32_t nodes;
      exit_t = chain_walk<B>(F, TC, x, true, lane, ent, mydl, nodes, count_t);
    }
    exit_t = uniform64(exit_t);
    count_t = uniform32(count_t);
    if (count_t > TILE) {  // impossible for a consistent walk: flag instead of looping on it
      if (lane == 0) atomicOr(P.overflow, 4u);
      count_t = 0;
    }
    if (published && y != MARK_NONE && exit_t != y && x < ve) {
      if (lane == 0) atomicMin(P.misspec, (uint32_t)t);
    }
    if (lane == 0) {
      st_agent(&P.inclx[t], exit_t + 1);
      st_agent(&P.aggc[t], (uint64_t)count_t + 1);
    }

    MARK(6);
    // ---- count look-back -> first output slot ------------------------------------------
    uint64_t base = 0;
    if (t > 0) {
      for (uint32_t spin = 0;;) {
        const int64_t pi = (int64_t)t - 1 - (int64_t)lane;
        uint64_t vi = 0, va = 0;
        if (pi >= 0) {
          vi = ld_agent(&P.inclc[pi]);
          va = ld_agent(&P.aggc[pi]);
        } else if (pi == -1) {
          vi = 1;  // virtual inclusive prefix 0 before tile 0
        }
        const uint64_t im = __ballot(vi != 0);
        if (im) {
          const uint32_t ist = (uint32_t)__builtin_ctzll(im);
          const uint64_t am = __ballot(va != 0);
          const uint64_t need = (1ull << ist) - 1;
          if ((am & need) == need) {
            const uint64_t part = (lane < ist) ? va - 1 : 0ull;
            base = readlane64(vi, ist) - 1 + wave_sum64(part);
            base = uniform64(base);
            break;
          }
        }
        if (++spin > SPIN_MAX) {
          if (lane == 0) atomicOr(P.overflow, 2u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    base = uniform64(base);
    if (lane == 0) st_agent(&P.inclc[t], base + count_t + 1);
    if (base + count_t > P.cap && lane == 0) atomicOr(P.overflow, 1u);

    MARK(7);
    // ---- emit frames ---------------------------------------------------------------------
    MARK(10);
    const uint32_t myoff = wave_incl_scan32(mydl) - mydl;
    MARK(11);
    uint32_t nch = 0, nbl = 0;
    uint64_t badf = ~0ull;
    for (uint32_t r0 = 0; r0 < count_t; r0 += FL_CAP) {
      if (ent >= 0 && mydl) {
        uint64_t cur = A + (uint32_t)ent;
        uint32_t k = 0;
        for (;;) {
          Hdr h = parse_hdr_lds(buf, A, cur, se);
          if (hdr_delivered(h)) {
            const uint32_t rank = myoff + k;
            if (rank >= r0 && rank < r0 + FL_CAP) flist[rank - r0] = (uint16_t)(cur - A);
            k++;
          }
          if (h.kind != H_VALID) break;
          cur = h.succ;
          if (cur >= lend) break;
        }
      }
      MARK(12);
      __syncthreads();
      MARK(13);
      const uint32_t nr = (count_t - r0) < FL_CAP ? (count_t - r0) : FL_CAP;
      for (uint32_t k = lane; k < nr; k += 64) {
        const uint64_t pos = A + flist[k];
        Hdr h = parse_hdr_lds(buf, A, pos, se);
        const uint64_t f = base + r0 + k;
        const uint64_t po = pos + h.vlen + 1;
        const uint64_t pl = h.L - 1;
        uint32_t ty = h.id | (h.kind == H_TAIL_BLOB ? DRP_FRAME_PARTIAL : 0u);
        if (h.id == 1) nch++; else nbl++;
        if (f < P.cap) {
          P.payload_off[f] = po;
          P.payload_len[f] = pl > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)pl;
          P.type[f] = (uint8_t)ty;
          if (h.id == 1) {
            LdsReader rd{buf, A, umin64(A + TILE + HALO, se)};
            ChangeCols c = decode_change(rd, po, pl);
            if (c.err == ERR_UNREACHABLE) {
              GlobalReader gr{P.bytes, se};
              c = decode_change(gr, po, pl);
            }
            P.key_off[f] = c.key_off;
            P.key_len[f] = c.key_len;
            P.subset_off[f] = c.subset_off;
            P.subset_len[f] = c.subset_len;
            P.value_off[f] = c.value_off;
            P.value_len[f] = c.value_len;
            P.change[f] = c.change;
            P.from[f] = c.from;
            P.to[f] = c.to;
            uint32_t fl = c.flags;
            if (c.err == DRP_ERR_REQUIRED) fl |= DRP_F_MISSING;
            P.flags[f] = (uint8_t)fl;
            if (c.err) {
              atomicMin((unsigned long long *)&P.payload_err[s], (unsigned long long)f);
              badf = f < badf ? f : badf;
            }
          }
        }
      }
      MARK(14);
      __syncthreads();
      MARK(15);
    }
    MARK(8);
    nch = wave_sum32(nch);
    nbl = wave_sum32(nbl);
#pragma unroll
    for (uint32_t m = 1; m < WAVE; m <<= 1) {
      const uint64_t o = ((uint64_t)shfl_xor32((uint32_t)(badf >> 32), m) << 32) | shfl_xor32((uint32_t)badf, m);
      badf = o < badf ? o : badf;
    }
    if (lane == 0) {
      if (nch) atomicAdd((unsigned long long *)&P.scount[2 * s], (unsigned long long)nch);
      if (nbl) atomicAdd((unsigned long long *)&P.scount[2 * s + 1], (unsigned long long)nbl);
      P.tile_x[t] = x;
      P.tile_exit[t] = exit_t;
      P.tile_base[t] = base;
      P.tile_count[t] = count_t;
      P.tile_nch[t] = nch;
      P.tile_nbl[t] = nbl;
      P.tile_perr[t] = badf;
    }
    MARK(9);
  }
#ifdef DRP_KERNEL_TRACE
  if (P.dbg && lane == 0)
    __hip_atomic_store(P.dbg + blockIdx.x * 4 + 1, 0xD0Eu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

// Debug: copy the agent-scope progress words of a running decode to host-mapped memory.
__global__ void peek_kernel(const uint32_t *dbg, uint32_t n, uint32_t *out) {
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    out[i] = __hip_atomic_load(dbg + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// tile_prefix[s] = number of tiles of streams < s; tile_prefix[nstreams] = total.
template <int B>
__global__ __launch_bounds__(1024) void tile_prefix_kernel(const uint64_t *stream_off, uint64_t nstreams,
                                                           uint64_t *tile_prefix) {
  constexpr uint64_t TILE = 64ull * B;
  __shared__ uint64_t part[1024];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t c0 = 0; c0 < nstreams; c0 += 1024) {
    const uint64_t s = c0 + threadIdx.x;
    uint64_t n = 0;
    if (s < nstreams) {
      const uint64_t so = stream_off[s], se = stream_off[s + 1];
      if (se > so) n = (((se + TILE - 1) & ~(TILE - 1)) - (so & ~(TILE - 1))) / TILE;
    }
    part[threadIdx.x] = n;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
      uint64_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    if (s < nstreams) tile_prefix[s] = carry + part[threadIdx.x] - n;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) tile_prefix[nstreams] = carry;
}

__device__ Hdr parse_hdr_global(const uint8_t *g, uint64_t p, uint64_t se) {
  GlobalReader gr{g, se};
  uint64_t w0, w1;
  gr.win(p, w0, w1);
  // reuse the LDS parser on a 32-byte private image
  uint8_t img[40];
  for (int i = 0; i < 8; i++) { img[i] = (uint8_t)(w0 >> (8 * i)); img[8 + i] = (uint8_t)(w1 >> (8 * i)); }
  for (int i = 16; i < 40; i++) img[i] = 0;
  return parse_hdr_lds(img, p, p, se);
}

// One thread per stream: turn per-tile records into drp_stream_result.
__global__ void finalize_kernel(const uint8_t *bytes, const uint64_t *stream_off, uint64_t nstreams,
                                const uint64_t *tile_prefix, const uint64_t *tile_exit,
                                const uint64_t *tile_base, const uint64_t *tile_count,
                                const uint64_t *payload_err, const uint64_t *scount,
                                const uint8_t *type, const uint8_t *flags, uint64_t cap,
                                drp_stream_result *res) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams) return;
  const uint64_t ntiles = tile_prefix[nstreams];
  const uint64_t tf = tile_prefix[s], tl = tile_prefix[s + 1];
  const uint64_t so = stream_off[s], se = stream_off[s + 1];
  drp_stream_result r;
  r.frames = r.changes = r.blobs = 0;
  r.consumed = se - so;
  r.blob_remaining = 0;
  r.err_frame = ~0ull;
  r.err_code = DRP_ERR_NONE;
  r.err_detail = 0;
  r.tail_kind = DRP_TAIL_NONE;
  r.reserved = 0;
  if (tf == tl) {
    r.frame_begin = (tf < ntiles) ? tile_base[tf]
                                  : (ntiles ? tile_base[ntiles - 1] + tile_count[ntiles - 1] : 0);
    res[s] = r;
    return;
  }
  const uint64_t fb = tile_base[tf];
  r.frame_begin = fb;
  const uint64_t chain = tile_base[tl - 1] + tile_count[tl - 1] - fb;
  const uint64_t ex = tile_exit[tl - 1];
  uint64_t frames = chain;
  if (ex & MARK_TERM) {
    const uint64_t q = ex & POS_MASK;
    Hdr h = parse_hdr_global(bytes, q, se);
    switch (h.kind) {
      case H_TAIL_HDR: r.tail_kind = DRP_TAIL_HEADER; r.consumed = q - so; break;
      case H_TAIL_CHANGE: r.tail_kind = DRP_TAIL_CHANGE; r.consumed = q - so; break;
      case H_TAIL_BLOB:
        r.tail_kind = DRP_TAIL_BLOB;
        r.consumed = se - so;
        r.blob_remaining = (q + h.vlen + h.L) - se;
        break;
      // an error ends the stream: nothing is carried (consumed = stream length)
      case H_ERR_TYPE: r.err_code = DRP_ERR_TYPE; r.err_detail = h.id; r.err_frame = chain; break;
      case H_ERR_LEN: r.err_code = DRP_ERR_LEN; r.err_detail = h.id; r.err_frame = chain; break;
      default: r.err_code = DRP_ERR_VARINT; r.err_frame = chain; break;
    }
  } else {
    r.consumed = (ex >= se ? se : ex) - so;
  }
  const uint64_t pe = payload_err[s];
  if (pe != ~0ull && pe - fb < r.err_frame) {
    r.err_frame = pe - fb;
    r.err_code = (pe < cap && (flags[pe] & DRP_F_MISSING)) ? DRP_ERR_REQUIRED : DRP_ERR_CHANGE;
    r.err_detail = 0;
    r.tail_kind = DRP_TAIL_NONE;
    r.blob_remaining = 0;
    r.consumed = se - so;
  }
  if (r.err_frame < frames) frames = r.err_frame;
  r.frames = frames;
  if (frames == chain) {
    r.changes = scount[2 * s];
    r.blobs = scount[2 * s + 1];
  } else {
    uint64_t ch = 0, bl = 0;
    for (uint64_t f = fb; f < fb + frames && f < cap; f++) {
      if ((type[f] & 0x3F) == DRP_TYPE_CHANGE) ch++; else bl++;
    }
    r.changes = ch;
    r.blobs = bl;
  }
  res[s] = r;
}

}  // namespace drp

// ---- host-side launchers (called from drp_api.hip) --------------------------------------
using namespace drp;

extern "C" hipError_t drp_launch_tile_prefix(uint32_t B, const uint64_t *stream_off, uint64_t nstreams,
                                             uint64_t *tile_prefix, hipStream_t st) {
  switch (B) {
    case 64: hipLaunchKernelGGL(tile_prefix_kernel<64>, dim3(1), dim3(1024), 0, st, stream_off, nstreams, tile_prefix); break;
    case 128: hipLaunchKernelGGL(tile_prefix_kernel<128>, dim3(1), dim3(1024), 0, st, stream_off, nstreams, tile_prefix); break;
    case 256: hipLaunchKernelGGL(tile_prefix_kernel<256>, dim3(1), dim3(1024), 0, st, stream_off, nstreams, tile_prefix); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t drp_launch_decode(uint32_t B, const DecodeParams *P, uint32_t grid, hipStream_t st) {
  switch (B) {
    case 64: hipLaunchKernelGGL(decode_tiles<64>, dim3(grid), dim3(64), 0, st, *P); break;
    case 128: hipLaunchKernelGGL(decode_tiles<128>, dim3(grid), dim3(64), 0, st, *P); break;
    case 256: hipLaunchKernelGGL(decode_tiles<256>, dim3(grid), dim3(64), 0, st, *P); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t drp_launch_peek(const uint32_t *dbg, uint32_t n, uint32_t *out, hipStream_t st) {
  hipLaunchKernelGGL(peek_kernel, dim3(1), dim3(256), 0, st, dbg, n, out);
  return hipGetLastError();
}

extern "C" hipError_t drp_launch_finalize(const uint8_t *bytes, const uint64_t *stream_off, uint64_t nstreams,
                                          const uint64_t *tile_prefix, const uint64_t *tile_exit,
                                          const uint64_t *tile_base, const uint64_t *tile_count,
                                          const uint64_t *payload_err, const uint64_t *scount,
                                          const uint8_t *type, const uint8_t *flags, uint64_t cap,
                                          drp_stream_result *res, hipStream_t st) {
  const uint32_t blk = 256;
  const uint32_t grid = (uint32_t)((nstreams + blk - 1) / blk);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(finalize_kernel, dim3(grid), dim3(blk), 0, st, bytes, stream_off, nstreams, tile_prefix,
                     tile_exit, tile_base, tile_count, payload_err, scount, type, flags, cap, res);
  return hipGetLastError();
}
