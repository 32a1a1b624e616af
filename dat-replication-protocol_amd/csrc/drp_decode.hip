// drp_decode.hip — gfx950 decode of varint-length-prefixed multibuffer streams into a
// frame table + Change SoA columns. Replaces the per-frame loop of decode.js
// (Decoder._consume / _onheader / _onchangedata / _onchangeend / _onblobdata,
// decode.js:144-262) and messages.Change.decode (messages/index.js:5).
//
// One wave owns one tile of 64*B stream bytes (B bytes per lane), read from HBM once and
// kept in LDS. Frames carry no sync marker, so a tile cannot know where its first frame
// starts until its predecessors are resolved; the kernel therefore splits the work into
// an entry-independent part (almost all of it) and an O(1) entry-dependent part:
//
//   1. live mask   Every byte position whose bytes could start a header with id <= 2
//                  (varint terminator followed by a byte <= 2) — bit-parallel per lane.
//   2. lane DP     Descending over its live positions, each lane sorts every position of
//                  its B bytes into: dead (the chain from it ends inside the lane: error,
//                  tail or non-header) or one of <= 3 "classes" = the distinct positions at
//                  which chains leave the lane. One header parse per live position.
//   3. lane graph  Node (lane, class) -> node holding that class exit in a later lane (or
//                  EXIT / DEAD / UNKNOWN); 6 rounds of pointer doubling in LDS give every
//                  node its tile exit. The tile's transfer function is now known for EVERY
//                  entry position.
//   4. look-back  Tile t publishes Y_t (the distinct exits landing in tile t+1) as soon as
//                  step 3 is done, then agg_t = f_t evaluated on Y_{t-1} (exact, no
//                  speculation). Tile t finds its entry x_t by reading predecessors'
//                  inclusive exits / aggs and composing forward; a miss waits for that
//                  predecessor's exact inclusive exit.
//   5. emit        Marking over the doubling levels gives each lane its entry on the true
//                  chain; lanes walk their own bytes, a second (count) look-back gives the
//                  output slot, and frames are decoded from LDS into the SoA columns.
//
// DESIGN.md §decode has the derivation and the cost model.
#include "drp_device.h"
#include "drp_kernels.h"

namespace drp {

constexpr int NC = 3;                 // surviving exit classes per lane
constexpr uint32_t N_DEAD = 3;        // special graph nodes (class slot 3 of lanes 0 / 1)
constexpr uint32_t N_UNK = 7;
constexpr int LEV = 7;                // doubling levels 0..6 (2^6 = 64 lane hops)
constexpr uint32_t HALO = 512;        // bytes past the tile kept in LDS (straddling frames)
constexpr uint32_t SPIN_MAX = 1u << 22;
constexpr uint64_t READY = 1ull << 63;
constexpr uint32_t V_UNK = 0xFFFFu;   // agg value: not expressible -> wait for inclusive

// Optional per-wave event counters and phase cycle counts (DRP_STATS=1): accumulated in
// registers and flushed with one atomic per counter when the wave exits.
enum : uint32_t {
  ST_LB_ITERS = 0, ST_LB_NOINCL, ST_LB_NOAGG, ST_LB_KEYMISS, ST_LB_VUNK, ST_LB_OK0, ST_LB_OKN,
  ST_Y_SPINS, ST_SERIAL, ST_CNT_SPINS, ST_Y_COUNT, ST_AGG_UNK, ST_TILES, ST_PASS, ST_OVF_LANES,
  ST_T_GRAB, ST_T_STAGE, ST_T_DP, ST_T_Y, ST_T_LB, ST_T_PATH, ST_T_CNT, ST_T_EMIT,
  ST_EV_TILES, ST_EV_SG, ST_SKIPS, ST_PHASEA, ST_RT_CYC, ST_DRAIN_CYC, ST_DP_LIVE, ST_DP_TRIPS,
  ST_T_DPLOOP, ST_EMIT_FRAMES, ST_EMIT_TRIPS, ST_T_DPPARSE, ST_NSTATS
};
#define STAT(k, v)                         \
  do {                                     \
    if (PROF) acc[k] += (uint64_t)(v);     \
  } while (0)
#define TSTAMP(k)                                                               \
  do {                                                                          \
    if (PROF && P.trace && lane == 0) P.trace[t * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define TMARK(k)                             \
  do {                                       \
    if (PROF) {                              \
      const uint64_t now_ = clock64();       \
      acc[k] += now_ - tclk;                 \
      tclk = now_;                           \
    }                                        \
  } while (0)


// ---- tile maps in index form ----------------------------------------------------------
// A tile's map sends the index (0..2) of its entry among the keys Y_{t-1} to the index of its
// exit among Y_t, 2 bits per key; 3 = not expressible (dead path, exit outside Y_t). Maps
// compose in O(1), so a wave scans 64 consecutive tiles' maps in 6 shuffle steps.
constexpr uint32_t MAP_ID = 0x24u;   // identity: 0->0, 1->1, 2->2
constexpr uint32_t MAP_NONE = 0x3Fu;
__device__ __forceinline__ uint32_t map_apply(uint32_t m, uint32_t q) {
  return q >= 3u ? 3u : (m >> (2u * q)) & 3u;
}
// f first, then g
__device__ __forceinline__ uint32_t map_then(uint32_t f, uint32_t g) {
  return map_apply(g, f & 3u) | (map_apply(g, (f >> 2) & 3u) << 2) | (map_apply(g, (f >> 4) & 3u) << 4);
}
// inclusive scan of maps over lanes (lane 0's map applied first)
__device__ __forceinline__ uint32_t map_scan(uint32_t m, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < WAVE; d <<= 1) {
    const uint32_t o = shfl_up32(m, d);
    if (lane >= d) m = map_then(o, m);
  }
  return m;
}

// ---- bit arrays of NW 64-bit words (lane-private, fully unrolled) ---------------------
template <int NW>
__device__ __forceinline__ bool tbit(const uint64_t (&m)[NW], uint32_t o) {
  uint64_t w = m[0];
#pragma unroll
  for (int i = 1; i < NW; i++)
    if ((o >> 6) == (uint32_t)i) w = m[i];
  return (w >> (o & 63)) & 1ull;
}
template <int NW>
__device__ __forceinline__ void sbit(uint64_t (&m)[NW], uint32_t o) {
#pragma unroll
  for (int i = 0; i < NW; i++)
    if ((o >> 6) == (uint32_t)i) m[i] |= 1ull << (o & 63);
}
// right shift (toward lower positions) of an N-word array by d < 64
template <int N>
__device__ __forceinline__ void shr(const uint64_t (&a)[N], uint32_t d, uint64_t (&o)[N]) {
#pragma unroll
  for (int i = 0; i < N; i++) o[i] = (a[i] >> d) | (i + 1 < N ? (a[i + 1] << (64 - d)) : 0ull);
}


__device__ __forceinline__ uint4 load16(const uint8_t *g, uint64_t p, uint64_t se) {
  if (p + 16 <= se) return *reinterpret_cast<const uint4 *>(g + p);
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t k = 0; k < 16; k++)
    if (p + k < se) w[k >> 2] |= (uint32_t)g[p + k] << (8 * (k & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Per-key results of phase 1 that phase 2 needs once the entry is known (the key the entry
// turns out to be selects one row).
enum : uint32_t { KF_KEY = 1, KF_EXIT = 2, KF_COUNT = 4, KF_SERIAL = 8 };
struct KeyRec {
  uint64_t keys;        // Y_{t-1} word (16-bit fields: tile-relative position + 1)
  uint64_t kexit[3];    // exact tile exit of the key's path (KF_EXIT)
  uint32_t kcnt[3];     // frames it delivers in the tile (KF_COUNT)
  uint32_t kfl[3];
  uint8_t ent[3][64];   // per lane: lane-relative entry of the key's path, 0xFF none
};

// Live positions per tile parsed load-balanced across the wave (more: per-lane parsing).
constexpr uint32_t PCAP = 832;
enum : uint32_t { PR_DEAD = 0, PR_IN = 1u << 30, PR_EXIT = 2u << 30, PR_FAR = 3u << 30, PR_OFF = (1u << 30) - 1 };

// LDS of one wave (one tile).
template <int B>
struct WaveLds {
  static constexpr uint32_t TILE = 64u * B;
  static constexpr int NW = B / 64;
  static constexpr int NM = NC + 2;
  uint8_t buf[TILE + HALO + 32] __attribute__((aligned(16)));
  uint64_t lm[64 * NM * NW];  // per lane: class masks, dead mask, live mask
  union {
    struct {                  // lane graph (built after the DP)
      uint64_t exv[256];      // node -> its class exit
      uint8_t jmp[LEV][256];  // doubling levels of the lane graph
      uint8_t mark[256];
      uint16_t nsum[2][256];  // doubling sums of delivered frames along the lane graph
    };
    struct {                  // during the DP: the tile's live positions, parsed load-balanced
      uint16_t ppos[PCAP];    // tile-relative position, lanes in order, ascending in a lane
      uint32_t prec[PCAP];    // its parse: PR_* tag | tile-relative successor / exit
    };
  };
  int32_t entry[64];          // per lane: entry of the tile's path (tile-relative), -1 none
  KeyRec rec[2];              // phase 1 -> phase 2 (two tiles in flight per wave)
};

__device__ __forceinline__ uint64_t lds_ld(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// spin until a sibling's LDS word is non-zero (bounded)
__device__ __forceinline__ uint64_t lds_wait(const uint64_t *p, uint32_t *overflow, uint32_t lane, uint32_t bit = 2u) {
  for (uint32_t spin = 0;; spin++) {
    const uint64_t v = lds_ld(p);
    if (v) return v;
    if (spin > (1u << 24)) {
      if (lane == 0) atomicOr(overflow, bit);
      return 0;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Orders this wave's LDS accesses (a wave's DS instructions execute in order; this keeps
// the compiler from moving them and drains outstanding LDS traffic).
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
}

#ifndef DRP_WPG
#define DRP_WPG 4
#endif
constexpr int WPG = DRP_WPG;  // waves (= consecutive tiles) per workgroup: one grab per group
constexpr int64_t SG = 64;  // tiles per super-group (second look-back level)
#ifndef DRP_NAP
#define DRP_NAP 2  // s_sleep units (64 cycles) between polls of a global look-back word
#endif
#ifndef DRP_EAGER_Y
#define DRP_EAGER_Y 1  // group-first waves wait for Y_{t-1} before looking back (else lazy)
#endif
#ifndef DRP_MIN_WAVES
#define DRP_MIN_WAVES 3  // waves per SIMD the register allocation must allow
#endif

template <int B, bool PROF>
__global__ __launch_bounds__(64 * WPG, DRP_MIN_WAVES) void decode_tiles(DecodeParams P) {
  constexpr uint32_t TILE = 64u * B;
  constexpr int NW = B / 64;           // mask words per lane
  constexpr int NV = B / 16;           // 16-byte loads per lane
  constexpr int NM = NC + 2;           // per lane: class masks, dead mask, live mask
  __shared__ WaveLds<B> wl[WPG];
  __shared__ uint32_t grp_slot;
  // sibling hand-off: the WPG tiles of a group are consecutive, so tile t gets Y_{t-1}, its
  // entry and its output base from the wave before it through LDS (~100 cycles) instead of
  // global round trips (~4 us under load); only the group's first wave looks back globally
  __shared__ uint64_t gyl[WPG], gxl[WPG], gcl[WPG];

  const uint32_t lane = lane_id();
  const uint32_t wid = threadIdx.x >> 6;
  uint8_t *const buf = wl[wid].buf;
  uint64_t *const lm = wl[wid].lm;
  uint64_t *const exv = wl[wid].exv;
  uint8_t(*const jmp)[256] = wl[wid].jmp;
  uint8_t *const mark = wl[wid].mark;
  int32_t *const entry = wl[wid].entry;
  uint16_t(*const nsum)[256] = wl[wid].nsum;
  const uint64_t ntiles = P.tile_prefix[P.nstreams];

  // lm accessors: lane m, mask k (0..NC-1 class, NC dead, NC+1 live), word w
  auto LM = [&](uint32_t m, uint32_t k, uint32_t w) -> uint64_t & { return lm[(m * NM + k) * NW + w]; };

  // profiling counters live in LDS so the profiling build keeps the production occupancy
  // (all updates are wave-uniform: every lane writes the same value)
  __shared__ uint64_t sacc[PROF ? WPG : 1][PROF ? ST_NSTATS : 1];
  uint64_t *const acc = sacc[PROF ? wid : 0];
  if (PROF && lane < ST_NSTATS) acc[lane] = 0;
  uint64_t tclk = PROF ? clock64() : 0;
  uint32_t novf = 0;

  // Software pipeline per wave: phase 1 of the tile just taken (everything that does not
  // depend on its entry: staging, live mask, DP, lane graph, Y_t, agg_t and the lane entries
  // of every key's path), then phase 2 of the tile taken one round earlier (look-back for
  // its entry, lane walks, output slot, emission). By the time a tile reaches phase 2 its
  // predecessors have had a whole phase 1 to publish their maps, so the look-back rarely
  // waits. Phase 1 only ever waits on Y_{t-1} of a tile taken earlier, whose phase 1 starts
  // right after its grab, so the pipeline cannot deadlock.
  uint64_t tp = ~0ull;  // tile whose phase 2 is pending
  uint32_t slot = 0;    // key record of the tile in phase 1 (phase 2 uses slot ^ 1)
  uint64_t c_s = 0, c_tf = 1, c_tl = 0, c_so = 0, c_se = 0, c_e0 = 0;  // cached stream geometry
  for (;;) {
    const uint64_t tgrab = PROF ? __builtin_amdgcn_s_memrealtime() : 0;
    // one atomic grab per group of WPG consecutive tiles; every lane of wave 0 executes
    // the atomic (addend 1 on lane 0) so the grab is never split off the loop
    __syncthreads();
    if (wid == 0) {
      const uint32_t g = atomicAdd(P.counter, lane == 0 ? 1u : 0u);
      if (lane == 0) grp_slot = g;
    }
    if (lane == 0) { gyl[wid] = 0; gxl[wid] = 0; gcl[wid] = 0; }
    __syncthreads();
    const uint64_t g0 = (uint64_t)grp_slot * WPG;
    const uint64_t tn = g0 + wid;
    const bool have = g0 < ntiles && tn < ntiles;

    // ======== phase 1 of tile tn ===========================================================
    if (have) {
    const uint64_t t = tn;
    KeyRec &R = wl[wid].rec[slot];
    // ---- which stream / tile (the last stream's geometry is cached) ------------------------
    if (t < c_tf || t >= c_tl) {
      uint64_t lo = 0, hi = P.nstreams;
      while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (P.tile_prefix[mid] <= t) lo = mid; else hi = mid;
      }
      c_s = uniform64(lo);
      c_tf = uniform64(P.tile_prefix[c_s]);
      c_tl = uniform64(P.tile_prefix[c_s + 1]);
      c_so = uniform64(P.stream_off[c_s]);
      c_se = uniform64(P.stream_off[c_s + 1]);
      c_e0 = uniform64(c_so + (P.entry ? P.entry[c_s] : 0ull));
    }
    const uint64_t s = c_s, tf = c_tf, tl = c_tl, so = c_so, se = c_se;
    const uint64_t A0 = so & ~(uint64_t)(TILE - 1);
    const uint64_t A = A0 + (t - tf) * TILE;
    const uint64_t vs = umax64(so, A), ve = umin64(se, A + TILE);
    const bool first = (t == tf);
    const uint64_t e0 = c_e0;
    (void)tl;
    (void)s;
    (void)vs;
    TMARK(ST_T_GRAB);
    TSTAMP(0);
    if (PROF && P.trace && lane == 0) P.trace[t * 8 + 7] = tgrab;
    // ---- stage: own B bytes (+ the halo) into LDS --------------------------------------
    const uint64_t lb = A + (uint64_t)lane * B;
    uint4 v[NV];
#pragma unroll
    for (int k = 0; k < NV; k++) v[k] = load16(P.bytes, lb + 16 * k, se);
#pragma unroll
    for (int k = 0; k < NV; k++) *reinterpret_cast<uint4 *>(buf + lane * B + 16 * k) = v[k];
    if (lane < HALO / 16)
      *reinterpret_cast<uint4 *>(buf + TILE + lane * 16) = load16(P.bytes, A + TILE + lane * 16, se);
    if (lane < 2) *reinterpret_cast<uint4 *>(buf + TILE + HALO + lane * 16) = make_uint4(0, 0, 0, 0);
    entry[lane] = -1;
    wsync();

    // ---- 1. live mask over the lane's B bytes ----------------------------------------------
    const uint32_t plo = (uint32_t)(vs > lb ? umin64(vs - lb, B) : 0);
    const uint32_t phi = (uint32_t)(ve > lb ? umin64(ve - lb, B) : 0);
    const uint64_t lhi = lb + phi;  // lane's valid end (absolute)
    uint64_t lvm[NW];
    {
      uint64_t M[NW + 1], S[NW + 1];
#pragma unroll
      for (int w = 0; w <= NW; w++) { M[w] = 0; S[w] = 0; }
#pragma unroll
      for (int k = 0; k < NV; k++) {
        uint32_t m16, s16;
        gather16(v[k], m16, s16);
        M[k >> 2] |= (uint64_t)m16 << (16 * (k & 3));
        S[k >> 2] |= (uint64_t)s16 << (16 * (k & 3));
      }
      {
        const uint4 x = *reinterpret_cast<const uint4 *>(buf + lane * B + B);
        uint32_t m16, s16;
        gather16(x, m16, s16);
        M[NW] = m16;
        S[NW] = s16;
      }
      // terminator q: MSB clear at q and byte q+1 <= 2
      uint64_t S1[NW + 1], X[NW + 1], tmp[NW + 1], Mk[NW + 1];
      shr<NW + 1>(S, 1, S1);
#pragma unroll
      for (int w = 0; w <= NW; w++) X[w] = ~M[w] & S1[w];
      // p is live if the run of MSB-set bytes from p ends at a terminator (<= 15 bytes)
#pragma unroll
      for (int w = 0; w <= NW; w++) Mk[w] = M[w];
#pragma unroll
      for (int d = 1; d <= 8; d <<= 1) {
        shr<NW + 1>(X, d, tmp);
#pragma unroll
        for (int w = 0; w <= NW; w++) X[w] |= Mk[w] & tmp[w];
        if (d < 8) {
          shr<NW + 1>(Mk, d, tmp);
#pragma unroll
          for (int w = 0; w <= NW; w++) Mk[w] &= tmp[w];
        }
      }
#pragma unroll
      for (int w = 0; w < NW; w++) {
        const uint32_t b0 = 64u * w;
        uint64_t r = ~0ull;
        if (phi <= b0) r = 0;
        else if (phi < b0 + 64) r = (1ull << (phi - b0)) - 1;
        if (plo >= b0 + 64) r = 0;
        else if (plo > b0) r &= ~((1ull << (plo - b0)) - 1);
        lvm[w] = X[w] & r;
      }
    }

    TMARK(ST_T_STAGE);
    // live masks go to LDS first: an exit that lands on a non-live position of a later lane
    // is a dead end and must not take one of the lane's NC exit classes
#pragma unroll
    for (int w = 0; w < NW; w++) LM(lane, NC + 1, w) = lvm[w];
    wsync();

    // ---- 2. lane DP: classify every live position, descending --------------------------
    if (PROF) {
      uint32_t nl = 0, trips = 0;
#pragma unroll
      for (int w = 0; w < NW; w++) {
        const uint32_t c = (uint32_t)__builtin_popcountll(lvm[w]);
        nl += c;
        uint32_t mx = c;
        for (uint32_t m = 1; m < WAVE; m <<= 1) mx = max(mx, shfl_xor32(mx, m));
        trips += mx;
      }
      STAT(ST_DP_LIVE, wave_sum32(nl));
      STAT(ST_DP_TRIPS, trips);
      TMARK(ST_T_STAGE);
    }
    uint64_t cm[NC][NW], dm[NW];
    uint64_t cex[NC];
    uint32_t ncls = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      cex[c] = 0;
#pragma unroll
      for (int w = 0; w < NW; w++) cm[c][w] = 0;
    }
#pragma unroll
    for (int w = 0; w < NW; w++) dm[w] = 0;
    // 2a. Every live position of the tile is parsed once, spread evenly over the lanes
    // (a lane owns 4 live positions on average but the busiest owns ~4x that): the lanes'
    // positions go to a list, each lane parses list entries lane, lane+64, ..., and the
    // classification below only reads the results back.
    uint32_t nlive = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) nlive += (uint32_t)__builtin_popcountll(lvm[w]);
    const uint32_t pend = wave_incl_scan32(nlive);
    const uint32_t ptotal = readlane32(pend, WAVE - 1);
    const bool balanced = ptotal <= PCAP;
    uint16_t *const ppos = wl[wid].ppos;
    uint32_t *const prec = wl[wid].prec;
    if (balanced) {
      uint32_t i = pend - nlive;
#pragma unroll
      for (int w = 0; w < NW; w++) {
        uint64_t bits = lvm[w];
        while (bits) {
          ppos[i++] = (uint16_t)(lane * B + 64u * w + (uint32_t)__builtin_ctzll(bits));
          bits &= bits - 1;
        }
      }
      wsync();
      for (uint32_t i2 = lane; i2 < ptotal; i2 += WAVE) {
        const uint32_t r = ppos[i2];
        const uint64_t p = A + r;
        const uint64_t mhi = umin64(A + (uint64_t)(r / B + 1) * B, ve);
        const Hdr h = parse_hdr_lds(buf, A, p, se);
        uint32_t code = PR_DEAD;
        if (h.kind == H_VALID) {
          const uint64_t nx = h.succ;
          if (nx < mhi) {
            code = PR_IN | (uint32_t)(nx - A);
          } else {
            bool exit_dead = false;
            if (nx < ve) {
              const uint32_t r2 = (uint32_t)(nx - A);
              exit_dead = !((LM(r2 / B, NC + 1, (r2 % B) >> 6) >> (r2 & 63)) & 1ull);
            } else if (nx < se && nx + 16 <= A + TILE + HALO) {
              const Hdr h2 = parse_hdr_lds(buf, A, nx, se);  // exit into the halo: error header there?
              exit_dead = h2.kind >= H_ERR_VARINT;
            }
            if (!exit_dead) code = nx - A <= PR_OFF ? PR_EXIT | (uint32_t)(nx - A) : PR_FAR;
          }
        }
        prec[i2] = code;
      }
      wsync();
    }
    TMARK(ST_T_DPPARSE);

    // 2b. classification, descending over the lane's live positions
    uint32_t pidx = pend;  // one past the list index of the current position
#pragma unroll
    for (int w = NW - 1; w >= 0; w--) {
      uint64_t bits = lvm[w];
      while (bits) {
        const uint32_t o = 64u * w + (63u - (uint32_t)__builtin_clzll(bits));
        bits &= ~(1ull << (o & 63));
        // successor of position o: dead, inside the lane, or an exit nx >= lhi
        bool dead = true, inl = false;
        uint64_t nx = 0;
        if (balanced) {
          const uint32_t code = prec[--pidx];
          const uint32_t tag = code & PR_FAR;
          dead = tag == PR_DEAD;
          inl = tag == PR_IN;
          nx = A + (code & PR_OFF);
          if (tag == PR_FAR) nx = parse_hdr_lds(buf, A, lb + o, se).succ;
        } else {
          const Hdr h = parse_hdr_lds(buf, A, lb + o, se);
          if (h.kind == H_VALID) {
            nx = h.succ;
            inl = nx < lhi;
            bool exit_dead = false;
            if (nx >= lhi && nx < ve) {
              const uint32_t r2 = (uint32_t)(nx - A);
              exit_dead = !((LM(r2 / B, NC + 1, (r2 % B) >> 6) >> (r2 & 63)) & 1ull);
            } else if (nx >= ve && nx < se && nx + 16 <= A + TILE + HALO) {
              const Hdr h2 = parse_hdr_lds(buf, A, nx, se);  // exit into the halo: error header there?
              exit_dead = h2.kind >= H_ERR_VARINT;
            }
            dead = exit_dead;
          }
        }
        int cls = -1;  // -1 dead, -2 unresolved (class overflow)
        if (!dead) {
          if (!inl) {
            cls = -2;
#pragma unroll
            for (int c = 0; c < NC; c++)
              if ((uint32_t)c < ncls && cex[c] == nx) cls = c;
            if (cls == -2 && ncls < (uint32_t)NC) {
#pragma unroll
              for (int c = 0; c < NC; c++)
                if ((uint32_t)c == ncls) cex[c] = nx;
              cls = (int)ncls;
              ncls++;
            } else if (cls == -2) {
              // table full: evict the farthest exit if this one is nearer. Near exits are
              // checked against live / halo headers; far ones are mostly the 2-byte "shadow"
              // varints that end on a frame's first header byte. Evicted positions become
              // unresolved (a path through them takes the serial walk).
              int far = 0;
#pragma unroll
              for (int c = 1; c < NC; c++)
                if (cex[c] > cex[far]) far = c;
              uint64_t fx = cex[0];
#pragma unroll
              for (int c = 1; c < NC; c++)
                if (c == far) fx = cex[c];
              if (nx < fx) {
#pragma unroll
                for (int c = 0; c < NC; c++)
                  if (c == far) {
                    cex[c] = nx;
#pragma unroll
                    for (int w2 = 0; w2 < NW; w2++) cm[c][w2] = 0;
                  }
                cls = far;
              }
            }
          } else {
            const uint32_t o2 = (uint32_t)(nx - lb);
            if (tbit<NW>(dm, o2) || !tbit<NW>(lvm, o2)) {
              cls = -1;
            } else {
              cls = -2;
#pragma unroll
              for (int c = 0; c < NC; c++)
                if (tbit<NW>(cm[c], o2)) cls = c;
            }
          }
        }
        if (cls == -2) novf++;
        if (cls == -1) sbit<NW>(dm, o);
#pragma unroll
        for (int c = 0; c < NC; c++)
          if (cls == c) sbit<NW>(cm[c], o);
      }
    }
    TMARK(ST_T_DPLOOP);
#pragma unroll
    for (int w = 0; w < NW; w++) {
#pragma unroll
      for (int c = 0; c < NC; c++) LM(lane, c, w) = cm[c][w];
      LM(lane, NC, w) = dm[w];
    }
    wsync();

    // node of an in-tile position q (vs <= q < ve): class node, N_DEAD or N_UNK
    auto resolve = [&](uint64_t q) -> uint32_t {
      const uint32_t r = (uint32_t)(q - A);
      const uint32_t m = r / B, o = r % B;
      const uint32_t w = o >> 6, b = o & 63;
#pragma unroll
      for (int c = 0; c < NC; c++)
        if ((LM(m, c, w) >> b) & 1ull) return m * 4 + c;
      if ((LM(m, NC, w) >> b) & 1ull) return N_DEAD;
      if (!((LM(m, NC + 1, w) >> b) & 1ull)) return N_DEAD;
      return N_UNK;
    };

    // ---- 3. lane graph + pointer doubling ------------------------------------------------
    // Delivered frames of a path inside one lane, walking from position q of lane m up to
    // the lane's end (or the path's end). Used per graph edge and for keys / the entry.
    auto lane_count = [&](uint64_t q) -> uint32_t {
      const uint32_t m = (uint32_t)(q - A) / B;
      const uint64_t mh = umin64(A + (uint64_t)(m + 1) * B, ve);
      uint32_t nd = 0;
      for (uint64_t cur = q; cur < mh;) {
        const Hdr h = parse_hdr_lds(buf, A, cur, se);
        nd += hdr_delivered(h) ? 1u : 0u;
        if (h.kind != H_VALID) break;
        cur = h.succ;
      }
      return nd;
    };
    // Node (lane, class): edge to the node holding the class exit; edge weight = frames
    // delivered in the lane the exit lands in (from the exit to that lane's end).
    uint32_t J[4], Sm[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t n = lane * 4 + c;
      uint32_t j = n;  // self loop: EXIT node, unused slot, or the special nodes 3 / 7
      uint32_t w = 0;
      if ((uint32_t)c < ncls) {
        const uint64_t e = cex[c];
        exv[n] = e;
        if (e < ve) {
          j = resolve(e);
          if (j != N_UNK) w = lane_count(e);
        }
      }
      J[c] = j;
      Sm[c] = w;
      jmp[0][n] = (uint8_t)j;
      nsum[0][n] = (uint16_t)w;
    }
    for (int r = 1; r < LEV; r++) {
      wsync();
#pragma unroll
      for (int c = 0; c < 4; c++) {
        Sm[c] += nsum[(r - 1) & 1][J[c]];
        J[c] = jmp[r - 1][J[c]];
        jmp[r][lane * 4 + c] = (uint8_t)J[c];
        nsum[r & 1][lane * 4 + c] = (uint16_t)Sm[c];
      }
    }
    wsync();
    // frames delivered by the path entering at in-tile position q (valid only when the
    // final node is not N_UNK); q's node n0 = resolve(q)
    auto path_count = [&](uint64_t q, uint32_t n0) -> uint32_t {
      uint32_t c = lane_count(q);
      if (n0 != N_DEAD && n0 != N_UNK) c += nsum[(LEV - 1) & 1][n0];
      return c;
    };
    // J[c] = final node of my class c

    TMARK(ST_T_DP);
    TSTAMP(1);
    // ---- 4a. Y_t: distinct exits of my classes that land in the next tile ----------------
    const bool has_next = (t + 1 < tl);
    uint64_t ywt = READY;  // Y_t (keys of tile t+1), for the index form of agg_t
    if (has_next) {
      uint64_t cand[NC];
#pragma unroll
      for (int c = 0; c < NC; c++) {
        cand[c] = ~0ull;
        if ((uint32_t)c < ncls && J[c] != N_DEAD && J[c] != N_UNK) {
          const uint64_t e = exv[J[c]];
          if (e >= A + TILE && e < A + 2 * TILE && e < se) cand[c] = e;
        }
      }
      uint64_t yw = READY;
      for (int k = 0; k < 3; k++) {
        bool any = false;
        uint64_t mine = ~0ull;
#pragma unroll
        for (int c = 0; c < NC; c++)
          if (cand[c] != ~0ull && !any) { any = true; mine = cand[c]; }
        const uint64_t bm = __ballot(any);
        if (!bm) break;
        const uint64_t y = readlane64(mine, (uint32_t)__builtin_ctzll(bm));
#pragma unroll
        for (int c = 0; c < NC; c++)
          if (cand[c] == y) cand[c] = ~0ull;
        yw |= (y - (A + TILE) + 1) << (16 * k);
        STAT(ST_Y_COUNT, 1);
      }
      ywt = yw;
      if (lane == 0) {
        st_agent(&P.ywd[t], yw);
        lds_st(&gyl[wid], yw);
      }
    } else if (lane == 0) {
      lds_st(&gyl[wid], READY);
    }


    // ---- 4b. keys of this tile: Y_{t-1}, or the stream entry for a stream's first tile ----
    uint64_t keys = READY;
    if (first) {
      if (e0 < ve) keys = READY | (e0 - A + 1);
    } else if (wid > 0) {  // Y_{t-1} from the sibling wave
      keys = uniform64(lds_wait(&gyl[wid - 1], P.overflow, lane, 16u)) | READY;
    } else {
      for (uint32_t spin = 0;; spin++) {
        const uint64_t yk = uniform64(ld_agent(&P.ywd[t - 1]));
        if (yk & READY) { keys = yk; break; }
        STAT(ST_Y_SPINS, 1);
        if (spin > SPIN_MAX) {
          if (lane == 0) atomicOr(P.overflow, 8u);
          break;
        }
        __builtin_amdgcn_s_sleep(DRP_NAP);
      }
    }

    // ---- 4c. per key (lane k < 3): final exit, frames delivered, agg_t = f_t on Y_{t-1} ----
    uint32_t kn = N_DEAD, kf = N_DEAD, kc = 0, kfl = 0, code = V_UNK;
    uint64_t kq = 0, kex = 0;
    {
      const uint32_t rel = lane < 3 ? (uint32_t)(keys >> (16 * lane)) & 0xFFFFu : 0u;
      if (rel) {
        kq = A + rel - 1;
        if (kq >= vs && kq < ve) {
          kfl = KF_KEY;
          kn = resolve(kq);
          kf = (kn != N_DEAD && kn != N_UNK) ? (uint32_t)jmp[LEV - 1][kn] : kn;
          if (kf != N_DEAD && kf != N_UNK) {
            kex = exv[kf];
            kfl |= KF_EXIT;
          }
          if (kn == N_UNK || kf == N_UNK) {
            kfl |= KF_SERIAL;
          } else {
            kc = path_count(kq, kn);
            kfl |= KF_COUNT;
          }
          if ((kfl & KF_EXIT) && kex - (A + TILE) < 0xFFF0ull) code = (uint32_t)(kex - (A + TILE));
        }
      }
      if (PROF) STAT(ST_AGG_UNK, __builtin_popcountll(__ballot(rel != 0 && code == V_UNK)));
      uint32_t ix = 3;
#pragma unroll
      for (int r = 0; r < 3; r++)
        if (code != V_UNK && ((ywt >> (16 * r)) & 0xFFFFu) == code + 1u) ix = (uint32_t)r;
      const uint64_t aw_l = lane < 3 ? ((uint64_t)code << (16 * lane)) | ((uint64_t)ix << (48 + 2 * lane)) : 0ull;
      const uint64_t nw_l = lane < 3 && code != V_UNK ? (uint64_t)kc << (16 * lane) : 0ull;
      const uint64_t aw = READY | readlane64(aw_l, 0) | readlane64(aw_l, 1) | readlane64(aw_l, 2);
      const uint64_t nw = READY | readlane64(nw_l, 0) | readlane64(nw_l, 1) | readlane64(nw_l, 2);
      if (!first && !P.strict && lane == 0) {
        st_agent(&P.aggn[t], nw);
        st_agent(&P.aggv[t], aw);
      }
      if (lane < 3) {
        R.kexit[lane] = kex;
        R.kcnt[lane] = kc;
        R.kfl[lane] = kfl;
      }
      if (lane == 0) R.keys = keys;
    }
    TSTAMP(2);
    // Tile-level evaluation of the exact exit v through tiles j0 .. j0+n-1 of this stream
    // (lanes hold aggv / ywd of tile j0+lane). Returns how many tiles were passed; the exit
    // after tile j0+k is left in lane k's `mine` (value + 1).
    auto eval_tiles = [&](uint64_t &v, uint64_t &cn, int64_t j0, uint32_t n, uint64_t av, uint64_t an,
                          uint64_t yk, uint64_t &mine, uint64_t &minec) -> uint32_t {
      uint32_t k = 0;
      for (; k < n; k++) {
        const uint64_t Aj = A - (uint64_t)((int64_t)t - (j0 + (int64_t)k)) * TILE;
        uint32_t add = 0;
        if (v < Aj + TILE) {
          const uint64_t ai = readlane64(av, k), yi = readlane64(yk, k), ni = readlane64(an, k);
          if (!(ai & READY) || !(yi & READY) || !(ni & READY)) break;
          const uint64_t rel = v - Aj + 1;
          uint32_t code = V_UNK;
#pragma unroll
          for (int q = 0; q < 3; q++)
            if (((yi >> (16 * q)) & 0xFFFFu) == rel) {
              code = (uint32_t)(ai >> (16 * q)) & 0xFFFFu;
              add = (uint32_t)(ni >> (16 * q)) & 0xFFFFu;
            }
          if (code == V_UNK) break;
          v = uniform64(Aj + TILE + code);
        }
        cn += add;
        if (lane == k) { mine = v + 1; minec = (uint64_t)add + 1; }
      }
      return k;
    };
    // Super-group bookkeeping: the last tile of a group of 64 to publish its map composes
    // the group's 64 maps into sagg[g] (keys = Y of the tile before the group).
    const int64_t sg = (int64_t)(t / SG), sg0 = sg * SG;
    const uint64_t sgsize = umin64(SG, ntiles - (uint64_t)sg0);
    auto sg_agg_done = [&]() {
      uint32_t old = 0;
      // relaxed: the words read below are self-validating (READY-tagged), so the last
      // finisher just waits until every one of them is visible
      if (lane == 0) old = __hip_atomic_fetch_add(&P.sgc_agg[sg], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      old = readlane32(old, 0);
      if (old != sgsize - 1) return;
      uint64_t cw = READY | 0xFFFFFFFFFFFFull;  // all V_UNK
      if (sgsize == SG && sg0 > (int64_t)tf && sg0 + SG - 1 < (int64_t)tl && !P.strict) {
        const int64_t j = sg0 + lane;
        uint64_t av = 0, an = 0, yk = 0, yo = 0;
        for (uint32_t w = 0; w < 1u << 16; w++) {  // a tile that never published its map
          av = ld_agent(&P.aggv[j]);                // (resolved early) leaves its codes V_UNK
          an = ld_agent(&P.aggn[j]);
          yk = ld_agent(&P.ywd[j - 1]);
          yo = (lane == SG - 1 && sg0 + SG < (int64_t)tl) ? ld_agent(&P.ywd[j]) : READY;
          if (__ballot(!(av & READY) || !(yk & READY) || !(an & READY) || !(yo & READY)) == 0) break;
          __builtin_amdgcn_s_sleep(DRP_NAP);
        }
        const uint64_t keys = readlane64(yk, 0);
        const uint64_t Ag = A - (uint64_t)((int64_t)t - sg0) * TILE;
        // the group's map in index form: one scan over the 64 tile maps
        const bool rdy = (av & READY) && (an & READY) && (yk & READY) && (yo & READY);
        const uint32_t I = map_scan(rdy ? (uint32_t)(av >> 48) & 63u : MAP_NONE, lane);
        uint32_t E = shfl_up32(I, 1);
        if (lane == 0) E = MAP_ID;
        const uint32_t Ig = readlane32(I, SG - 1);
        const uint64_t ylast = readlane64(yo, SG - 1);
        cw = READY;
        uint64_t nw = READY;
#pragma unroll
        for (int q = 0; q < 3; q++) {
          const uint32_t rel = (uint32_t)(keys >> (16 * q)) & 0xFFFFu;
          uint32_t code = V_UNK;
          uint64_t cq = 0;
          const uint32_t og = map_apply(Ig, (uint32_t)q);
          if (rel && (keys & READY) && og != 3 && ((ylast >> (16 * og)) & 0xFFFFu)) {
            code = (uint32_t)((ylast >> (16 * og)) & 0xFFFFu) - 1u;
            const uint32_t ik = map_apply(E, (uint32_t)q);
            cq = wave_sum32((uint32_t)(an >> (16 * ik)) & 0xFFFFu);
            cw |= (uint64_t)og << (48 + 2 * q);
          } else if (rel && (keys & READY)) {
            uint64_t vq = Ag + rel - 1, d0 = 0, d1 = 0;
            if (eval_tiles(vq, cq, sg0, SG, av, an, yk, d0, d1) == SG &&
                vq - (Ag + (uint64_t)SG * TILE) < 0xFFF0ull)
              code = (uint32_t)(vq - (Ag + (uint64_t)SG * TILE));
          }
          cw |= (uint64_t)code << (16 * q);
          nw |= (code == V_UNK ? 0ull : cq) << (20 * q);
        }
        if (lane == 0) st_agent(&P.saggn[sg], nw);
      }
      if (lane == 0) st_agent(&P.sagg[sg], cw);
    };

    sg_agg_done();
    TMARK(ST_T_Y);

    // ---- 4d. lane entries of every key's path: marking over the doubling levels ----------
    // mark byte of node n = set of keys whose path passes n; after level r it holds the
    // first 2^(r+1) nodes of each path
    {
      uint32_t *const mark32 = reinterpret_cast<uint32_t *>(mark);
      mark32[lane] = 0;
#pragma unroll
      for (int q = 0; q < 3; q++) R.ent[q][lane] = 0xFF;
      wsync();
      if (lane < 3 && (kfl & KF_KEY)) {
        const uint32_t r = (uint32_t)(kq - A);
        R.ent[lane][r / B] = (uint8_t)(r % B);
        if (kn != N_DEAD && kn != N_UNK && !(kfl & KF_SERIAL))
          __hip_atomic_fetch_or(&mark32[kn >> 2], (1u << lane) << (8 * (kn & 3)), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (__ballot(lane < 3 && kn != N_DEAD && kn != N_UNK && !(kfl & KF_SERIAL) && (kfl & KF_KEY))) {
        for (int r = 0; r < LEV - 1; r++) {
          wsync();
          const uint32_t mw = mark32[lane];
          uint32_t tg[4];
#pragma unroll
          for (int c = 0; c < 4; c++) tg[c] = jmp[r][lane * 4 + c];
          wsync();
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const uint32_t bb = (mw >> (8 * c)) & 0xFFu;
            if (bb)
              __hip_atomic_fetch_or(&mark32[tg[c] >> 2], bb << (8 * (tg[c] & 3)), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
        wsync();
        const uint32_t mw = mark32[lane];
#pragma unroll
        for (int c = 0; c < NC; c++) {
          const uint32_t n = lane * 4 + c;
          const uint32_t bb = (mw >> (8 * c)) & 7u;
          if ((uint32_t)c < ncls && bb) {
            const uint32_t nx = jmp[0][n];
            const uint64_t e = cex[c];
            if (e < ve && nx != n) {  // the path continues in a later lane (class or death)
              const uint32_t r = (uint32_t)(e - A);
#pragma unroll
              for (int q = 0; q < 3; q++)
                if ((bb >> q) & 1u) R.ent[q][r / B] = (uint8_t)(r % B);
            }
          }
        }
      }
      wsync();
    }
    }  // phase 1

    // (No grab ahead of phase 2: a group taken before a phase 2 that waits on a
    // predecessor's phase 2 can close a wait cycle — the predecessor's holder may itself be
    // in phase 1 waiting on Y of the group taken early. A group is only ever held while its
    // phase 1 is running or done.)

    // ======== phase 2 of tile tp ===========================================================
    if (tp != ~0ull) {
    const uint64_t t = tp;
    const KeyRec &R = wl[wid].rec[slot ^ 1];
    // ---- which stream / tile (the last stream's geometry is cached) ------------------------
    if (t < c_tf || t >= c_tl) {
      uint64_t lo = 0, hi = P.nstreams;
      while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (P.tile_prefix[mid] <= t) lo = mid; else hi = mid;
      }
      c_s = uniform64(lo);
      c_tf = uniform64(P.tile_prefix[c_s]);
      c_tl = uniform64(P.tile_prefix[c_s + 1]);
      c_so = uniform64(P.stream_off[c_s]);
      c_se = uniform64(P.stream_off[c_s + 1]);
      c_e0 = uniform64(c_so + (P.entry ? P.entry[c_s] : 0ull));
    }
    const uint64_t s = c_s, tf = c_tf, tl = c_tl, so = c_so, se = c_se;
    const uint64_t A0 = so & ~(uint64_t)(TILE - 1);
    const uint64_t A = A0 + (t - tf) * TILE;
    const uint64_t vs = umax64(so, A), ve = umin64(se, A + TILE);
    const bool first = (t == tf);
    const uint64_t e0 = c_e0;
    (void)tl;
    (void)s;
    (void)vs;

    TMARK(ST_T_GRAB);
    // ---- restage: own B bytes (+ the halo); the loads are issued here and land in LDS after
    // the look-back, so the two latencies overlap
    const uint64_t lb = A + (uint64_t)lane * B;
    uint4 rv[NV], rh = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < NV; k++) rv[k] = load16(P.bytes, lb + 16 * k, se);
    if (lane < HALO / 16) rh = load16(P.bytes, A + TILE + lane * 16, se);
    const uint32_t phi = (uint32_t)(ve > lb ? umin64(ve - lb, B) : 0);
    const uint64_t lhi = lb + phi;  // lane's valid end (absolute)

    TMARK(ST_T_STAGE);
    const int64_t sg = (int64_t)(t / SG), sg0 = sg * SG;
    const uint64_t sgsize = umin64(SG, ntiles - (uint64_t)sg0);
    // Tile-level evaluation of the exact exit v through tiles j0 .. j0+n-1 of this stream
    // (lanes hold aggv / ywd of tile j0+lane). Returns how many tiles were passed; the exit
    // after tile j0+k is left in lane k's `mine` (value + 1).
    auto eval_tiles = [&](uint64_t &v, uint64_t &cn, int64_t j0, uint32_t n, uint64_t av, uint64_t an,
                          uint64_t yk, uint64_t &mine, uint64_t &minec) -> uint32_t {
      uint32_t k = 0;
      for (; k < n; k++) {
        const uint64_t Aj = A - (uint64_t)((int64_t)t - (j0 + (int64_t)k)) * TILE;
        uint32_t add = 0;
        if (v < Aj + TILE) {
          const uint64_t ai = readlane64(av, k), yi = readlane64(yk, k), ni = readlane64(an, k);
          if (!(ai & READY) || !(yi & READY) || !(ni & READY)) break;
          const uint64_t rel = v - Aj + 1;
          uint32_t code = V_UNK;
#pragma unroll
          for (int q = 0; q < 3; q++)
            if (((yi >> (16 * q)) & 0xFFFFu) == rel) {
              code = (uint32_t)(ai >> (16 * q)) & 0xFFFFu;
              add = (uint32_t)(ni >> (16 * q)) & 0xFFFFu;
            }
          if (code == V_UNK) break;
          v = uniform64(Aj + TILE + code);
        }
        cn += add;
        if (lane == k) { mine = v + 1; minec = (uint64_t)add + 1; }
      }
      return k;
    };
    uint64_t x = e0;
    if (!first && wid > 0) {  // entry = the sibling's exact exit
      x = uniform64(lds_wait(&gxl[wid - 1], P.overflow, lane, 32u)) - 1;
      STAT(ST_LB_OK0, 1);
    } else if (!first) {
      uint32_t nap = 1;
      int64_t cur = -1;  // tile whose exact exit v is known (-1: none found yet)
      uint64_t v = 0;
      bool force_tile = false;
      for (uint32_t spin = 0;; spin++) {
        STAT(ST_LB_ITERS, 1);
        if (cur < 0) {  // A: nearest published exact exit
          STAT(ST_PHASEA, 1);
          const int64_t lo0 = (int64_t)umax64(tf, (uint64_t)sg0);
          const int64_t j = (int64_t)t - 1 - (int64_t)lane;
          const int64_t b = SG * (sg - (int64_t)lane) - 1;  // last tiles of the 64 previous groups
          uint64_t rt0 = 0;
          if (PROF) {  // drain this wave's outstanding stores first, then time the loads alone
            const uint64_t d0 = clock64();
            __builtin_amdgcn_s_waitcnt(0);
            rt0 = clock64();
            acc[ST_DRAIN_CYC] += rt0 - d0;
          }
          const uint64_t vj = j >= lo0 ? ld_agent(&P.inclx[j]) : 0ull;
          const uint64_t vb = b >= (int64_t)tf ? ld_agent(&P.inclx[b]) : 0ull;
          if (PROF) {
            __builtin_amdgcn_s_waitcnt(0);
            acc[ST_RT_CYC] += clock64() - rt0 + (uint64_t)(__ballot(vj == 12345) & 0);
          }
          {
            const uint64_t im = __ballot(vj != 0);
            if (im) {
              const uint32_t ist = (uint32_t)__builtin_ctzll(im);
              cur = (int64_t)t - 1 - ist;
              v = readlane64(vj, ist) - 1;
            }
          }
          if (cur < 0 && sg0 - 1 >= (int64_t)tf) {
            const uint64_t vi = vb;
            const uint64_t im = __ballot(vi != 0);
            if (im) {
              const uint32_t ist = (uint32_t)__builtin_ctzll(im);
              cur = SG * (sg - (int64_t)ist) - 1;
              v = readlane64(vi, ist) - 1;
            } else if (SG * (sg - 63) - 1 <= (int64_t)tf) {
              const uint64_t vf = uniform64(ld_agent(&P.inclx[tf]));
              if (vf) { cur = (int64_t)tf; v = vf - 1; }
            }
          }
          if (cur < 0) STAT(ST_LB_NOINCL, 1);
        }
        if (P.strict && cur != (int64_t)t - 1) cur = -1;
        // B: evaluate forward from tile cur+1, publishing every exit derived (helping)
        while (cur >= 0 && cur < (int64_t)t - 1) {
          if (!force_tile && (cur + 1) % SG == 0 && cur + SG <= (int64_t)t - 1) {
            // whole super-groups k0 .. k0+m-1
            const int64_t k0 = (cur + 1) / SG;
            const uint32_t m = (uint32_t)min((int64_t)64, ((int64_t)t - 1 - cur) / SG);
            const int64_t gk = k0 + lane;
            const bool inr = lane < m;
            // one round trip: every word this step may need is loaded together
            uint64_t vi = 0, sa = 0, sn = 0, sk = 0;
            if (inr) {
              vi = ld_agent(&P.inclx[SG * gk + SG - 1]);
              sa = ld_agent(&P.sagg[gk]);
              sn = ld_agent(&P.saggn[gk]);
              sk = ld_agent(&P.ywd[SG * gk - 1]);
            }
            const uint64_t im = __ballot(vi != 0);
            if (im) {
              const uint32_t hi = 63u - (uint32_t)__builtin_clzll(im);
              cur = SG * (k0 + hi) + SG - 1;
              v = readlane64(vi, hi) - 1;
              STAT(ST_SKIPS, 1);
              continue;
            }
            uint32_t i = 0;
            uint64_t mine = 0, minec = 0;
            for (; i < m; i++) {
              const uint64_t Ag = A - (uint64_t)((int64_t)t - SG * (k0 + (int64_t)i)) * TILE;
              const uint64_t Aend = Ag + (uint64_t)SG * TILE;
              uint64_t add = 0;
              if (v < Aend) {
                if (v >= Ag + TILE) break;  // lands inside the group: tile level
                const uint64_t ai = readlane64(sa, i), yi = readlane64(sk, i), ni = readlane64(sn, i);
                if (!(ai & READY) || !(yi & READY) || !(ni & READY)) break;
                const uint64_t rel = v - Ag + 1;
                uint32_t code = V_UNK;
#pragma unroll
                for (int q = 0; q < 3; q++)
                  if (((yi >> (16 * q)) & 0xFFFFu) == rel) {
                    code = (uint32_t)(ai >> (16 * q)) & 0xFFFFu;
                    add = (ni >> (20 * q)) & 0xFFFFFull;
                  }
                if (code == V_UNK) break;
                v = uniform64(Aend + code);
              }
              if (lane == i) { mine = v + 1; minec = add + 1; }
            }
            STAT(ST_EV_SG, i);
            if (lane < i) {  // helping: exit of each group's last tile, and the group's count
              st_agent(&P.inclx[SG * gk + SG - 1], mine);
              st_agent(&P.scnt[gk], minec);
            }
            if (i > 0) cur = SG * (k0 + (int64_t)i) - 1;
            if (i < m) force_tile = true;  // next group goes tile by tile
            continue;
          }
          // tile level, up to the end of the super-group holding tile cur+1
          const int64_t j0 = cur + 1;
          const uint32_t n = (uint32_t)min((int64_t)(SG - j0 % SG), (int64_t)t - 1 - cur);
          const int64_t j = j0 + lane;
          const bool inr = lane < n;
          uint64_t vi = 0, av = 0, an = 0, yk = 0, yo = 0;
          if (inr) {  // one round trip for the whole chunk
            vi = ld_agent(&P.inclx[j]);
            if (!P.strict) {
              av = ld_agent(&P.aggv[j]);
              an = ld_agent(&P.aggn[j]);
              yk = ld_agent(&P.ywd[j - 1]);
              yo = ld_agent(&P.ywd[j]);
            }
          }
          const uint64_t im = __ballot(vi != 0);
          if (im) {  // someone already got further: jump to the newest published exit
            const uint32_t hi = 63u - (uint32_t)__builtin_clzll(im);
            cur = j0 + hi;
            v = readlane64(vi, hi) - 1;
            if ((cur + 1) % SG == 0) force_tile = false;
            STAT(ST_SKIPS, 1);
            continue;
          }
          if (!P.strict) {
            // all lanes at once: scan the chunk's maps in index form from v's key index;
            // the exact evaluation below takes over where the index chain breaks
            const uint64_t Aj0 = A - (uint64_t)((int64_t)t - j0) * TILE;
            const uint64_t y0 = readlane64(yk, 0);
            uint32_t i0 = 3;
            if (v >= Aj0 && v < Aj0 + TILE && (y0 & READY)) {
#pragma unroll
              for (int r = 0; r < 3; r++)
                if (((y0 >> (16 * r)) & 0xFFFFu) == v - Aj0 + 1) i0 = (uint32_t)r;
            }
            if (i0 != 3) {
              const bool rdy = inr && (av & READY) && (an & READY) && (yk & READY) && (yo & READY);
              const uint32_t m = rdy ? (uint32_t)(av >> 48) & 63u : MAP_NONE;
              const uint32_t I = map_scan(m, lane);
              uint32_t E = shfl_up32(I, 1);
              if (lane == 0) E = MAP_ID;
              const uint32_t ik = map_apply(E, i0), ok = map_apply(m, ik);
              const uint64_t gm = __ballot(inr && ok != 3);
              const uint32_t k = (~gm) ? (uint32_t)__builtin_ctzll(~gm) : 64u;
              if (k > 0) {
                const uint64_t ex = Aj0 + (uint64_t)(lane + 1) * TILE + ((yo >> (16 * ok)) & 0xFFFFu) - 1;
                if (lane < k) {  // helping: exact exit and frame count of tiles j0 .. j0+k-1
                  st_agent(&P.inclx[j], ex + 1);
                  st_agent(&P.aggc[j], ((an >> (16 * ik)) & 0xFFFFu) + 1);
                }
                STAT(ST_EV_TILES, k);
                v = readlane64(ex, k - 1);
                cur = j0 + (int64_t)k - 1;
                if ((cur + 1) % SG == 0) force_tile = false;
                continue;
              }
            }
          }
          uint64_t mine = 0, minec = 0, cdummy = 0;
          const uint32_t k = eval_tiles(v, cdummy, j0, n, av, an, yk, mine, minec);
          STAT(ST_EV_TILES, k);
          if (lane < k) {  // helping: exact exit and frame count of tiles j0 .. j0+k-1
            st_agent(&P.inclx[j], mine);
            st_agent(&P.aggc[j], minec);
          }
          if (k == 0) { STAT(ST_LB_NOAGG, 1); break; }
          cur = j0 + k - 1;
          if ((cur + 1) % SG == 0) force_tile = false;
          if (k < n) break;  // stuck on a missing map: retry after a nap
        }
        if (cur == (int64_t)t - 1) { x = v; STAT(ST_LB_OKN, 1); break; }
        if (spin > SPIN_MAX) {
          if (lane == 0) atomicOr(P.overflow, 128u);
          x = MARK_TERM | vs;
          break;
        }
        for (uint32_t z = 0; z < nap; z++) __builtin_amdgcn_s_sleep(DRP_NAP);
        nap = nap < 8 ? nap * 2 : 8;
      }
    }
    x = uniform64(x);
#pragma unroll
    for (int k = 0; k < NV; k++) *reinterpret_cast<uint4 *>(buf + lane * B + 16 * k) = rv[k];
    if (lane < HALO / 16) *reinterpret_cast<uint4 *>(buf + TILE + lane * 16) = rh;
    if (lane < 2) *reinterpret_cast<uint4 *>(buf + TILE + HALO + lane * 16) = make_uint4(0, 0, 0, 0);
    entry[lane] = -1;
    wsync();
    TSTAMP(3);
    if (PROF && P.trace && lane == 0)
      P.trace[t * 8 + 6] = (uint64_t)__builtin_amdgcn_s_getreg(4 << 0 | 0 << 6 | 31 << 11) | ((uint64_t)wid << 32) |
                           ((uint64_t)(__builtin_amdgcn_s_getreg(20 << 0 | 0 << 6 | 15 << 11) & 15u) << 40);
    STAT(ST_TILES, 1);
    if (x >= ve) STAT(ST_PASS, 1);

    TMARK(ST_T_LB);
    // ---- 5a. the key x is, and its path's lane entries from phase 1 -----------------------
    int32_t kx = -1;
    if (x < ve) {
#pragma unroll
      for (int q = 0; q < 3; q++)
        if (((R.keys >> (16 * q)) & 0xFFFFu) == x - A + 1 && (R.kfl[q] & KF_KEY)) kx = q;
    }
    const uint32_t xfl = kx >= 0 ? R.kfl[kx] : 0u;
    // the exact exit is known right away unless the path ends inside the tile / is serial:
    // publish it before the lane walks so successors' look-backs advance sooner
    bool early = false, early_cnt = false, graph_exit = false;
    uint32_t gcount = 0;
    uint64_t gexit = 0;
    if (x >= ve) {
      early = early_cnt = true;
      if (lane == 0) {
        st_agent(&P.inclx[t], x + 1);
        lds_st(&gxl[wid], x + 1);
      }
    } else {
      if (xfl & KF_EXIT) {
        early = graph_exit = true;
        gexit = R.kexit[kx];
        if (lane == 0) {
          st_agent(&P.inclx[t], gexit + 1);
          lds_st(&gxl[wid], gexit + 1);
        }
      }
      if (xfl & KF_COUNT) {  // frame count of the path from x, from the graph
        early_cnt = true;
        gcount = R.kcnt[kx];
      }
    }
    auto count_published = [&]() {  // the last tile of the group to get here sums its counts
      uint32_t old = 0;
      if (lane == 0) old = __hip_atomic_fetch_add(&P.sgc_cnt[sg], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      old = readlane32(old, 0);
      if (old == sgsize - 1) {
        uint64_t c = 0;
        for (;;) {  // counts are value + 1: wait until all 64 are visible
          c = lane < sgsize ? ld_agent(&P.aggc[sg0 + lane]) : 1ull;
          if (__ballot(c == 0) == 0) break;
          __builtin_amdgcn_s_sleep(DRP_NAP);
        }
        const uint64_t sum = wave_sum64(c - 1);
        if (lane == 0) st_agent(&P.scnt[sg], sum + 1);
      }
    };
    if (early_cnt) {
      if (lane == 0) st_agent(&P.aggc[t], (uint64_t)gcount + 1);
      count_published();
    }

    if (x < ve) {
      const bool serial = kx < 0 || (xfl & KF_SERIAL);
      if (!serial) {
        const uint32_t o = R.ent[kx][lane];
        entry[lane] = o == 0xFFu ? -1 : (int32_t)(lane * B + o);
      } else {  // class overflow on the path, or an entry that is no key: walk it (rare)
        STAT(ST_SERIAL, 1);
        if (lane == 0) entry[(uint32_t)(x - A) / B] = (int32_t)(x - A);
        uint64_t cur = x;
        for (;;) {
          if (cur >= ve) break;
          const uint32_t r = (uint32_t)(cur - A);
          if (lane == 0 && entry[r / B] < 0) entry[r / B] = (int32_t)r;
          const Hdr h = parse_hdr_lds(buf, A, cur, se);
          if (h.kind != H_VALID) break;
          cur = uniform64(h.succ);
        }
      }
      wsync();
    }
    // ---- 5b. lane walks: delivered frames of the path inside my bytes --------------------
    // The path leaves the last entered lane at wend; if that is still inside the tile (a
    // path that dies at a dead-end exit), the lane holding it walks next.
    int32_t myent = entry[lane];
    uint64_t dmask[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) dmask[w] = 0;
    uint32_t cnt = 0;
    uint64_t wend = 0;
    uint64_t exit_t = x;
    uint32_t count_t = 0;
    if (x < ve) {
      bool walk = myent >= 0;
      for (;;) {
        if (walk) {
          uint64_t cur = A + (uint32_t)myent;
          for (;;) {
            if (cur >= lhi) { wend = cur; break; }
            const Hdr h = parse_hdr_lds(buf, A, cur, se);
            if (hdr_delivered(h)) { sbit<NW>(dmask, (uint32_t)(cur - lb)); cnt++; }
            if (h.kind != H_VALID) { wend = MARK_TERM | cur; break; }
            cur = h.succ;
          }
        }
        const uint64_t em = __ballot(myent >= 0);
        const uint32_t last = 63u - (uint32_t)__builtin_clzll(em);
        exit_t = uniform64(readlane64(wend, last));
        if (exit_t >= ve) break;
        const uint32_t r = (uint32_t)(exit_t - A);
        walk = lane == r / B;
        if (walk) myent = (int32_t)r;
      }
      count_t = wave_sum32(cnt);
      if (graph_exit && exit_t != gexit && lane == 0) atomicOr(P.overflow, 4u);
    }
    exit_t = uniform64(exit_t);
    count_t = uniform32(count_t);
    if (lane == 0 && !early) {
      st_agent(&P.inclx[t], exit_t + 1);
      lds_st(&gxl[wid], exit_t + 1);
    }
    if (early_cnt) {
      if (count_t != gcount && lane == 0) atomicOr(P.overflow, 4u);
    } else {
      if (lane == 0) st_agent(&P.aggc[t], (uint64_t)count_t + 1);
      count_published();
    }

    TMARK(ST_T_PATH);
    // ---- 5c. count look-back -> first output slot ------------------------------------------
    // Same shape as the exit look-back: the nearest inclusive prefix among this group's tiles
    // or the last tiles of the 64 previous groups, then sums forward by whole groups (scnt)
    // and tiles (aggc), publishing the inclusive prefix of every boundary passed (helping).
    uint64_t base = 0;
    if (t > 0 && wid > 0) {  // the sibling's inclusive prefix
      base = uniform64(lds_wait(&gcl[wid - 1], P.overflow, lane, 64u)) - 1;
    } else if (t > 0) {
      uint32_t nap = 1;
      int64_t cur = -2;  // tile whose inclusive prefix v is known (-1: virtual tile before 0)
      uint64_t v = 0;
      bool force_tile = false;
      for (uint32_t spin = 0;;) {
        if (cur < -1) {
          {
            const int64_t j = (int64_t)t - 1 - (int64_t)lane;
            const uint64_t vi = j >= sg0 ? ld_agent(&P.inclc[j]) : 0ull;
            const uint64_t im = __ballot(vi != 0);
            if (im) {
              const uint32_t ist = (uint32_t)__builtin_ctzll(im);
              cur = (int64_t)t - 1 - ist;
              v = readlane64(vi, ist) - 1;
            }
          }
          if (cur < -1) {
            const int64_t b = SG * (sg - (int64_t)lane) - 1;
            const uint64_t vi = b >= 0 ? ld_agent(&P.inclc[b]) : (b == -1 ? 1ull : 0ull);
            const uint64_t im = __ballot(vi != 0);
            if (im) {
              const uint32_t ist = (uint32_t)__builtin_ctzll(im);
              cur = SG * (sg - (int64_t)ist) - 1;
              v = readlane64(vi, ist) - 1;
            }
          }
        }
        while (cur >= -1 && cur < (int64_t)t - 1) {
          if (!force_tile && (cur + 1) % SG == 0 && cur + SG <= (int64_t)t - 1) {
            const int64_t k0 = (cur + 1) / SG;
            const uint32_t m = (uint32_t)min((int64_t)64, ((int64_t)t - 1 - cur) / SG);
            const int64_t gk = k0 + lane;
            const bool inr = lane < m;
            const uint64_t vi = inr ? ld_agent(&P.inclc[SG * gk + SG - 1]) : 0ull;
            const uint64_t im = __ballot(vi != 0);
            if (im) {
              const uint32_t hi = 63u - (uint32_t)__builtin_clzll(im);
              cur = SG * (k0 + hi) + SG - 1;
              v = readlane64(vi, hi) - 1;
              continue;
            }
            const uint64_t sc = inr ? ld_agent(&P.scnt[gk]) : 0ull;
            const uint64_t am = __ballot(sc != 0);
            const uint32_t k = (~am) ? (uint32_t)__builtin_ctzll(~am) : 64u;
            const uint32_t kk = k < m ? k : m;
            if (kk == 0) { force_tile = true; continue; }
            const uint64_t c = lane < kk ? sc - 1 : 0ull;
            uint64_t pre = c;  // inclusive prefix over lanes
#pragma unroll
            for (uint32_t d = 1; d < WAVE; d <<= 1) {
              const uint64_t o = shfl_up64(pre, d);
              if (lane >= d) pre += o;
            }
            if (lane < kk) st_agent(&P.inclc[SG * gk + SG - 1], v + pre + 1);
            v += readlane64(pre, kk - 1);
            cur = SG * (k0 + (int64_t)kk) - 1;
            if (kk < m) force_tile = true;
            continue;
          }
          const int64_t j0 = cur + 1;
          const uint32_t n = (uint32_t)min((int64_t)(SG - j0 % SG), (int64_t)t - 1 - cur);
          const int64_t j = j0 + lane;
          const bool inr = lane < n;
          const uint64_t vi = inr ? ld_agent(&P.inclc[j]) : 0ull;
          const uint64_t im = __ballot(vi != 0);
          if (im) {
            const uint32_t hi = 63u - (uint32_t)__builtin_clzll(im);
            cur = j0 + hi;
            v = readlane64(vi, hi) - 1;
            if ((cur + 1) % SG == 0) force_tile = false;
            continue;
          }
          const uint64_t va = inr ? ld_agent(&P.aggc[j]) : 0ull;
          const uint64_t am = __ballot(va != 0);
          const uint32_t k = (~am) ? (uint32_t)__builtin_ctzll(~am) : 64u;
          const uint32_t kk = k < n ? k : n;
          if (kk == 0) break;
          const uint32_t c = lane < kk ? (uint32_t)(va - 1) : 0u;
          const uint32_t pre = wave_incl_scan32(c);
          if (lane < kk) st_agent(&P.inclc[j], v + pre + 1);
          v += readlane32(pre, kk - 1);
          cur = j0 + kk - 1;
          if ((cur + 1) % SG == 0) force_tile = false;
          if (kk < n) break;
        }
        if (cur == (int64_t)t - 1) { base = v; break; }
        if (++spin > SPIN_MAX) {
          if (lane == 0) atomicOr(P.overflow, 256u);
          break;
        }
        STAT(ST_CNT_SPINS, 1);
        for (uint32_t z = 0; z < nap; z++) __builtin_amdgcn_s_sleep(DRP_NAP);
        nap = nap < 8 ? nap * 2 : 8;
      }
    }
    base = uniform64(base);
    if (lane == 0) {
      st_agent(&P.inclc[t], base + count_t + 1);
      lds_st(&gcl[wid], base + count_t + 1);
    }
    if (base + count_t > P.cap && lane == 0) atomicOr(P.overflow, 1u);

    TMARK(ST_T_CNT);
    TSTAMP(4);
    // ---- 5d. emit ------------------------------------------------------------------------
    const uint32_t myoff = wave_incl_scan32(cnt) - cnt;
    if (PROF) {
      uint32_t mx = cnt;
      for (uint32_t m = 1; m < WAVE; m <<= 1) mx = max(mx, shfl_xor32(mx, m));
      STAT(ST_EMIT_FRAMES, wave_sum32(cnt));
      STAT(ST_EMIT_TRIPS, mx);
    }
    uint32_t nch = 0, nbl = 0, k = 0;
    uint64_t badf = ~0ull;
#pragma unroll
    for (int w = 0; w < NW; w++) {
      uint64_t bits = dmask[w];
      while (bits) {
        const uint32_t o = 64u * w + (uint32_t)__builtin_ctzll(bits);
        bits &= bits - 1;
        const uint64_t pos = lb + o;
        const Hdr h = parse_hdr_lds(buf, A, pos, se);
        const uint64_t f = base + myoff + k;
        k++;
        const uint64_t po = pos + h.vlen + 1;
        const uint64_t pl = h.L - 1;
        const uint32_t ty = h.id | (h.kind == H_TAIL_BLOB ? DRP_FRAME_PARTIAL : 0u);
        if (h.id == 1) nch++; else nbl++;
        if (f < P.cap) {
          P.payload_off[f] = po;
          P.payload_len[f] = pl > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)pl;
          P.type[f] = (uint8_t)ty;
          if (h.id == 1) {
            const LdsReader rd{buf, A, umin64(A + TILE + HALO, se)};
            ChangeCols c = decode_change(rd, po, pl);
            if (c.err == ERR_UNREACHABLE) {
              const GlobalReader gr{P.bytes, se};
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
            if (c.err) badf = f < badf ? f : badf;
          }
        }
      }
    }
    nch = wave_sum32(nch);
    (void)nbl;
#pragma unroll
    for (uint32_t m = 1; m < WAVE; m <<= 1) {
      const uint64_t o = ((uint64_t)shfl_xor32((uint32_t)(badf >> 32), m) << 32) | shfl_xor32((uint32_t)badf, m);
      badf = o < badf ? o : badf;
    }
    if (lane == 0) {
      P.tile_nch[t] = nch;  // per-stream counts: scan + stream_counts (no same-address atomics)
      if (badf != ~0ull) atomicMin((unsigned long long *)&P.payload_err[s], (unsigned long long)badf);
      P.tile_exit[t] = exit_t;
      P.tile_base[t] = base;
      P.tile_count[t] = count_t;
    }
    TMARK(ST_T_EMIT);
    TSTAMP(5);
    }  // phase 2
    if (g0 >= ntiles) break;
    tp = have ? tn : ~0ull;
    slot ^= 1;
  }
  if (PROF) {
    const uint64_t ovl = wave_sum32(novf);
    wsync();
    acc[ST_OVF_LANES] = ovl;
    wsync();
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < (int)ST_NSTATS; i++) atomicAdd(P.stats + i, (unsigned long long)acc[i]);
  }
}

// tile_prefix[s] = number of tiles of streams < s; tile_prefix[nstreams] = total.
template <int B>
__device__ __forceinline__ void tile_prefix_body(const uint64_t *stream_off, uint64_t nstreams,
                                                 uint64_t *tile_prefix);
template <int B>
__global__ __launch_bounds__(1024) void tile_prefix_kernel(const uint64_t *stream_off, uint64_t nstreams,
                                                           uint64_t *tile_prefix) {
  tile_prefix_body<B>(stream_off, nstreams, tile_prefix);
}
// The speculative decode's prologue in one launch: workgroup 0 computes tile_prefix, the others
// fill the per-decode scratch regions (each a multiple of 4 bytes, 4-byte aligned) with their
// byte value: six hipMemsetAsync dispatches cost ~9 us apiece on the decode's serial path.
template <int B>
__global__ __launch_bounds__(1024) void prologue_kernel(const uint64_t *stream_off, uint64_t nstreams,
                                                        uint64_t *tile_prefix, ClearSet cs) {
  if (blockIdx.x == 0) {
    tile_prefix_body<B>(stream_off, nstreams, tile_prefix);
    return;
  }
  const uint64_t stride = (uint64_t)(gridDim.x - 1) * 1024u;
  for (uint32_t r = 0; r < cs.n; r++) {
    uint32_t *p = reinterpret_cast<uint32_t *>(cs.ptr[r]);
    const uint64_t words = cs.bytes[r] / 4;
    const uint32_t v = cs.value[r] * 0x01010101u;
    for (uint64_t i = (uint64_t)(blockIdx.x - 1) * 1024u + threadIdx.x; i < words; i += stride) p[i] = v;
  }
}
template <int B>
__device__ __forceinline__ void tile_prefix_body(const uint64_t *stream_off, uint64_t nstreams,
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
                                drp_stream_result *res, const uint32_t *abort_flag, uint32_t abort_mask) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams) return;
  if (abort_flag && (*abort_flag & abort_mask)) return;  // (a failed prediction: run again after its repair)
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
  r.tail_frame_bytes = 0;
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
      case H_TAIL_CHANGE:
        r.tail_kind = DRP_TAIL_CHANGE;
        r.consumed = q - so;
        r.tail_frame_bytes = h.L > ~0ull - h.vlen ? ~0ull : h.vlen + h.L;  // (saturates)
        break;
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
    r.tail_frame_bytes = 0;
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
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t drp_launch_prologue(uint32_t B, const uint64_t *stream_off, uint64_t nstreams,
                                          uint64_t *tile_prefix, const ClearSet *cs, hipStream_t st) {
  uint64_t mx = 0;
  for (uint32_t r = 0; r < cs->n; r++) mx = cs->bytes[r] > mx ? cs->bytes[r] : mx;
  const uint64_t blocks = (mx / 4 + 4096 - 1) / 4096;  // (4 words per thread and pass at most)
  const uint32_t grid = 1u + (uint32_t)(blocks < 1024 ? (blocks ? blocks : 1) : 1024);
  switch (B) {
    case 64: hipLaunchKernelGGL(prologue_kernel<64>, dim3(grid), dim3(1024), 0, st, stream_off, nstreams, tile_prefix, *cs); break;
    case 128: hipLaunchKernelGGL(prologue_kernel<128>, dim3(grid), dim3(1024), 0, st, stream_off, nstreams, tile_prefix, *cs); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" uint32_t drp_decode_waves_per_group(void) { return WPG; }

extern "C" hipError_t drp_launch_decode(uint32_t B, const DecodeParams *P, uint32_t grid, hipStream_t st) {
  switch (B) {
    case 64:
      if (P->stats) hipLaunchKernelGGL((decode_tiles<64, true>), dim3(grid), dim3(64 * WPG), 0, st, *P);
      else hipLaunchKernelGGL((decode_tiles<64, false>), dim3(grid), dim3(64 * WPG), 0, st, *P);
      break;
    case 128:
      if (P->stats) hipLaunchKernelGGL((decode_tiles<128, true>), dim3(grid), dim3(64 * WPG), 0, st, *P);
      else hipLaunchKernelGGL((decode_tiles<128, false>), dim3(grid), dim3(64 * WPG), 0, st, *P);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t drp_launch_finalize(const uint8_t *bytes, const uint64_t *stream_off, uint64_t nstreams,
                                          const uint64_t *tile_prefix, const uint64_t *tile_exit,
                                          const uint64_t *tile_base, const uint64_t *tile_count,
                                          const uint64_t *payload_err, const uint64_t *scount,
                                          const uint8_t *type, const uint8_t *flags, uint64_t cap,
                                          drp_stream_result *res, const uint32_t *abort_flag,
                                          uint32_t abort_mask, hipStream_t st) {
  const uint32_t blk = 256;
  const uint32_t grid = (uint32_t)((nstreams + blk - 1) / blk);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(finalize_kernel, dim3(grid), dim3(blk), 0, st, bytes, stream_off, nstreams, tile_prefix,
                     tile_exit, tile_base, tile_count, payload_err, scount, type, flags, cap, res, abort_flag,
                     abort_mask);
  return hipGetLastError();
}
