// drp_encode.hip — gfx950 batched Change encode: Encoder.change + Encoder._header
// (encode.js:102-117, 124-137) + messages.Change.encode (messages/index.js:5) for n rows.
//
// Three passes over the rows: (1) frame sizes, (2) exclusive scan of the sizes
// (per-block sums, then a single-block scan of the block sums), (3) one wave per frame
// assembles its bytes: the header and field prefixes are written lane-parallel from varints
// packed in registers (lane j stores byte j), all 64 lanes copy the key / subset / value bytes. Also the per-stream stats and global index scan used by the
// multi-GPU all-gather path.
#include "drp_device.h"
#include "drp_kernels.h"

namespace drp {

__device__ __forceinline__ uint32_t vlen64(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}
__device__ __forceinline__ uint32_t venc(uint64_t v, uint8_t *o) {
  uint32_t n = 0;
  while (v >= 0x80) {
    o[n++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  o[n++] = (uint8_t)v;
  return n;
}

// payload length of row i (protocol-buffers@2 field order: subset?, key, change, from, to, value?)
__device__ __forceinline__ uint64_t payload_len(const drp_change_src &s, uint64_t i) {
  const uint32_t fl = s.flags[i];
  uint64_t n = 0;
  if (fl & DRP_F_SUBSET) n += 1 + vlen64(s.subset_len[i]) + s.subset_len[i];
  n += 1 + vlen64(s.key_len[i]) + s.key_len[i];
  n += 1 + vlen64(s.change[i]) + 1 + vlen64(s.from[i]) + 1 + vlen64(s.to[i]);
  if (fl & DRP_F_VALUE) n += 1 + vlen64(s.value_len[i]) + s.value_len[i];
  return n;
}

constexpr uint32_t SCAN_BLK = 1024;
constexpr uint32_t ENC_F_RANGE = 2u;  // overflow bit: a row's heap range leaves the heap

// [off, off + len) inside [0, heap_bytes) without wrapping
__device__ __forceinline__ bool in_heap(uint64_t off, uint32_t len, uint64_t heap_bytes) {
  return (uint64_t)len <= heap_bytes && off <= heap_bytes - len;
}

__global__ __launch_bounds__(SCAN_BLK) void enc_size_kernel(EncodeParams P) {
  __shared__ uint64_t part[SCAN_BLK];
  const uint64_t i = (uint64_t)blockIdx.x * SCAN_BLK + threadIdx.x;
  uint64_t sz = 0;
  if (i < P.n) {
    const uint64_t pl = payload_len(P.src, i);
    sz = vlen64(pl + 1) + 1 + pl;
    const drp_change_src &s = P.src;
    const uint32_t fl = s.flags[i];
    bool ok = in_heap(s.key_off[i], s.key_len[i], P.heap_bytes);
    if (fl & DRP_F_SUBSET) ok = ok && in_heap(s.subset_off[i], s.subset_len[i], P.heap_bytes);
    if (fl & DRP_F_VALUE) ok = ok && in_heap(s.value_off[i], s.value_len[i], P.heap_bytes);
    if (!ok) atomicOr(P.overflow, ENC_F_RANGE);
  }
  part[threadIdx.x] = sz;
  __syncthreads();
  for (uint32_t d = 1; d < SCAN_BLK; d <<= 1) {
    uint64_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  if (i < P.n) P.frame_off[i] = part[threadIdx.x] - sz;  // block-local exclusive
  if (threadIdx.x == SCAN_BLK - 1) P.block_sum[blockIdx.x] = part[SCAN_BLK - 1];
}

__global__ __launch_bounds__(SCAN_BLK) void enc_blocksum_kernel(EncodeParams P, uint64_t nblk) {
  __shared__ uint64_t part[SCAN_BLK];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t c0 = 0; c0 < nblk; c0 += SCAN_BLK) {
    const uint64_t b = c0 + threadIdx.x;
    const uint64_t v0 = b < nblk ? P.block_sum[b] : 0;
    part[threadIdx.x] = v0;
    __syncthreads();
    for (uint32_t d = 1; d < SCAN_BLK; d <<= 1) {
      uint64_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    if (b < nblk) P.block_sum[b] = carry + part[threadIdx.x] - v0;
    __syncthreads();
    if (threadIdx.x == SCAN_BLK - 1) carry += part[SCAN_BLK - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    // a row outside the heap poisons the total (UINT64_MAX > any cap): nothing is written
    const bool range_bad = (__hip_atomic_load(P.overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ENC_F_RANGE) != 0;
    P.frame_off[P.n] = range_bad ? ~0ull : carry;
    if (range_bad || carry > P.cap) atomicOr(P.overflow, 1u);
  }
}

__global__ __launch_bounds__(SCAN_BLK) void enc_addbase_kernel(EncodeParams P) {
  const uint64_t i = (uint64_t)blockIdx.x * SCAN_BLK + threadIdx.x;
  if (i < P.n) P.frame_off[i] += P.block_sum[blockIdx.x];
}

__device__ __forceinline__ uint64_t enc_funnel(uint64_t lo, uint64_t hi, uint32_t sh) {
  return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 enc_ld(const uint4 *p) {
  return *p;
}
__device__ __forceinline__ void enc_st(uint4 *p, uint4 v) {
  *p = v;
}
// 16 bytes starting `sh` bytes into lo (the next bytes from hi)
__device__ __forceinline__ uint4 enc_shift(uint4 lo, uint4 hi, uint32_t sh) {
  if (sh == 0) return lo;
  const uint64_t q0 = ((uint64_t)lo.y << 32) | lo.x, q1 = ((uint64_t)lo.w << 32) | lo.z;
  const uint64_t q2 = ((uint64_t)hi.y << 32) | hi.x, q3 = ((uint64_t)hi.w << 32) | hi.z;
  uint64_t w0, w1;
  if (sh < 8) {
    w0 = enc_funnel(q0, q1, 8 * sh);
    w1 = enc_funnel(q1, q2, 8 * sh);
  } else {
    w0 = enc_funnel(q1, q2, 8 * (sh - 8));
    w1 = enc_funnel(q2, q3, 8 * (sh - 8));
  }
  return make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
}

// Wave copy of n bytes: byte head up to 16-byte alignment of dst, then one aligned 16-byte
// store per lane per step whose bytes come from the two aligned 16-byte source blocks that
// cover them (funnel shift by the wave-uniform source misalignment), then a byte tail. The
// second block of the last step lies in the aligned 16 bytes that hold the last source byte,
// so no load leaves the source's pages.
__device__ __forceinline__ void wave_copy(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src, uint64_t n,
                                          uint32_t lane) {
  if (n < 128) {
    for (uint64_t k = lane; k < n; k += 64) dst[k] = src[k];
    return;
  }
  const uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
  if (lane < head) dst[lane] = src[lane];
  dst += head;
  src += head;
  n -= head;
  const uint64_t nb = n >> 4;
  const uint32_t sh = (uint32_t)((uintptr_t)src & 15);
  const uint4 *sa = reinterpret_cast<const uint4 *>(src - sh);
  uint4 *da = reinterpret_cast<uint4 *>(dst);
  uint64_t b = lane;
  for (; b < nb; b += 64) {
    const uint4 lo = enc_ld(sa + b);
    enc_st(da + b, sh == 0 ? lo : enc_shift(lo, enc_ld(sa + b + 1), sh));
  }
  const uint32_t tail = (uint32_t)(n & 15);
  if (lane < tail) dst[(nb << 4) + lane] = src[(nb << 4) + lane];
}

#ifndef DRP_ENC_WAVES
#define DRP_ENC_WAVES 65536  // waves of the write kernel (grid-stride over frames)
#endif

// A varint (or one byte) packed into registers: bytes 0..7 in lo, 8..9 in hi.
struct VSeg {
  uint64_t lo;
  uint32_t hi, n;
};
__device__ __forceinline__ VSeg vseg(uint64_t v) {
  VSeg s{0ull, 0u, 0u};
  for (;;) {
    uint64_t b = v & 0x7F;
    v >>= 7;
    if (v) b |= 0x80;
    if (s.n < 8) s.lo |= b << (8 * s.n);
    else s.hi |= (uint32_t)b << (8 * (s.n - 8));
    s.n++;
    if (!v) return s;
  }
}
__device__ __forceinline__ VSeg vbyte1(uint32_t b, bool present = true) { return VSeg{b, 0u, present ? 1u : 0u}; }
// The concatenated segments, written lane-parallel: lane j stores byte j (segment lengths are
// wave-uniform: every lane holds the same frame). Returns the total length.
template <int N>
__device__ __forceinline__ uint32_t put_segs(uint8_t *o, uint32_t lane, const VSeg (&g)[N]) {
  uint32_t tot = 0, byte = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint32_t k = lane - tot;
    if (lane >= tot && k < g[i].n) byte = (uint32_t)((k < 8 ? g[i].lo >> (8 * k) : (uint64_t)(g[i].hi >> (8 * (k - 8)))) & 0xFF);
    tot += g[i].n;
  }
  if (lane < tot) o[lane] = (uint8_t)byte;
  return tot;
}

#define WAVE_COPY wave_copy
// one wave per frame (grid-stride over frames)
// The bytes of frame i written by one wave (the header and field prefixes lane-parallel, the key /
// subset / value bytes by WAVE_COPY).
__device__ __forceinline__ void write_frame(const EncodeParams &P, uint64_t i, uint32_t lane) {
  const drp_change_src &s = P.src;
  uint8_t *o = P.out + P.frame_off[i];
  const uint32_t fl = s.flags[i];
  const uint64_t pl = payload_len(s, i);
  const bool sub = (fl & DRP_F_SUBSET) != 0, val = (fl & DRP_F_VALUE) != 0;
  uint64_t off;
  {  // header (encode.js:124-137) + subset prefix
    const VSeg g[4] = {vseg(pl + 1), vbyte1(DRP_TYPE_CHANGE), vbyte1(0x0a, sub),
                       sub ? vseg(s.subset_len[i]) : VSeg{0ull, 0u, 0u}};
    off = put_segs(o, lane, g);
  }
  if (sub) {
    WAVE_COPY(o + off, P.heap + s.subset_off[i], s.subset_len[i], lane);
    off += s.subset_len[i];
  }
  {
    const VSeg g[2] = {vbyte1(0x12), vseg(s.key_len[i])};
    off += put_segs(o + off, lane, g);
    WAVE_COPY(o + off, P.heap + s.key_off[i], s.key_len[i], lane);
    off += s.key_len[i];
  }
  {
    const VSeg g[8] = {vbyte1(0x18), vseg(s.change[i]), vbyte1(0x20), vseg(s.from[i]), vbyte1(0x28), vseg(s.to[i]),
                       vbyte1(0x32, val), val ? vseg(s.value_len[i]) : VSeg{0ull, 0u, 0u}};
    off += put_segs(o + off, lane, g);
  }
  if (val) WAVE_COPY(o + off, P.heap + s.value_off[i], s.value_len[i], lane);
}

// one wave per frame (grid-stride over frames): every frame (DRP_ENC_OS=0, A/B)
__global__ __launch_bounds__(256) void enc_write_kernel(EncodeParams P) {
  const uint32_t lane = lane_id();
  const uint64_t wid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  if (P.frame_off[P.n] > P.cap) return;
  for (uint64_t i = wid; i < P.n; i += nw) write_frame(P, i, lane);
}

// ---- output-stationary write ------------------------------------------------------------------
// The output is cut into ENC_BS-byte blocks aligned in memory; a workgroup owns one block and each
// lane fixed 16-byte chunks of it. The workgroup lays out the frames the block touches in LDS (their
// starts, segment ends, heap offsets and prefix bytes), then every lane finds its chunk's frame and
// segment: a chunk inside one key / subset / value copy (nearly all of a 4 KB value) is two aligned
// heap loads, a funnel shift and one aligned 16-byte store, with no per-frame latency chain; a
// chunk that mixes segments is assembled piece by piece. Blocks touching more than ENC_FMAX frames
// (short frames) are left to the per-frame writer (enc_write_dense). 32 KiB blocks and a 16 KB
// LDS layout keep 8 workgroups on a CU, so the descriptor phase's latency (three dependent global
// rounds) is spread over 32 KiB of copies and hidden behind 7 other workgroups.
#ifndef DRP_ENC_OS
#define DRP_ENC_OS 1  // 0: the per-frame writer for every frame (A/B)
#endif
#ifndef DRP_ENC_DPP
#define DRP_ENC_DPP 1  // a lane's second source block from the next lane (wave shift) where it can
#endif                  // (C5 encode 2.02 -> 1.87 ms; 0: two loads per lane, A/B)
#ifndef DRP_ENC_U
#define DRP_ENC_U 4
#endif
#ifndef DRP_ENC_BS
#define DRP_ENC_BS 65536  // output block bytes (a multiple of 16 KiB, at most 1 MiB)
#endif
constexpr uint32_t ENC_BS = DRP_ENC_BS, ENC_CPB = ENC_BS / 16, ENC_OS_T = 256, ENC_FMAX = 128;
constexpr uint32_t ENC_U = DRP_ENC_U, ENC_NB = ENC_CPB / (ENC_OS_T * ENC_U);  // chunks per lane: ENC_NB batches of ENC_U
static_assert(ENC_NB >= 1 && ENC_NB * ENC_U <= 32 && ENC_CPB % (ENC_OS_T * ENC_U) == 0, "ENC_BS");
constexpr uint32_t LIT0 = 0, LIT2 = 24, LIT4 = 32, LITB = 72;  // prefix byte slots per frame
// Mixed chunks (not inside one copy segment) per block: at most 3 + 2 + 4 per frame (the chunks the
// prefix runs L0 <= 24 B, L2 <= 8 B, L4 <= 40 B overlap; a chunk across a copy's end overlaps the
// next prefix run) plus the output's first and last chunk.
constexpr uint32_t ENC_MIXCAP = 9 * ENC_FMAX + 8;
static_assert(ENC_CPB <= 65536, "chunk index in 16 bits");
constexpr uint32_t ENC_F_DENSE_FRAME = 1u << 31;               // (frame bytes that do not fit 31 bits)

// wire offset of output block b's first byte (blocks are aligned in memory; out may not be)
__device__ __forceinline__ int64_t oblk_start(uint64_t b, uint32_t g) { return (int64_t)(b * ENC_BS) - (int64_t)g; }

// oblk_first[b] = the frame holding block b's first wire byte (block 0: byte 0)
__global__ __launch_bounds__(256) void enc_oblk_kernel(EncodeParams P) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= P.n || P.frame_off[P.n] > P.cap) return;
  const uint64_t g = (uintptr_t)P.out & 15;
  const uint64_t lo = P.frame_off[i], hi = P.frame_off[i + 1];
  const uint64_t b0 = i == 0 ? 0 : (lo + g + ENC_BS - 1) / ENC_BS, b1 = (hi + g + ENC_BS - 1) / ENC_BS;
  for (uint64_t b = b0; b < b1 && b < P.nob; b++) P.oblk_first[b] = i;
}

__device__ __forceinline__ uint32_t put_lit(uint8_t *d, const VSeg &v) {
  for (uint32_t k = 0; k < v.n; k++) d[k] = (uint8_t)(k < 8 ? v.lo >> (8 * k) : (uint64_t)(v.hi >> (8 * (k - 8))));
  return v.n;
}

// bytes o .. o + 7 of an LDS byte array (three dword reads; any o)
__device__ __forceinline__ uint64_t enc_lds_u64(const uint8_t *lds, uint32_t o) {
  const uint32_t *q = reinterpret_cast<const uint32_t *>(lds) + (o >> 2);
  const uint32_t sh = (o & 3u) * 8u, a0 = q[0], a1 = q[1], a2 = q[2];
  return (uint64_t)__builtin_amdgcn_alignbit(a1, a0, sh) | ((uint64_t)__builtin_amdgcn_alignbit(a2, a1, sh) << 32);
}

struct EncLds {
  int64_t fst[ENC_FMAX + 1];  // frame starts (wire offsets); [nf] = the last frame's end
  uint32_t e[5][ENC_FMAX];    // segment ends relative to the frame start: L0 | subset | L2 | key | L4 (| value)
  uint64_t src[3][ENC_FMAX];  // heap offsets of subset, key, value
  __attribute__((aligned(4))) uint8_t lit[ENC_FMAX][LITB];
  uint8_t slack[32];  // (16-byte windows read past the last prefix slot)
  uint32_t nmix;
  uint16_t mix[ENC_MIXCAP];  // the block's mixed chunks (chunk index in the block)
};

// One chunk that mixes segments (or the output's first / last chunk), piece by piece (a piece = the
// chunk bytes of one segment of one frame), each piece as one 16-byte window shifted into place and
// masked: two aligned loads for heap bytes, LDS reads for prefix bytes, no byte loops.
__device__ __forceinline__ void enc_mixed_chunk(const EncodeParams &P, const EncLds &S, uint32_t nf,
                                                uint64_t W, int64_t c0) {
  const int64_t p0 = c0 < 0 ? 0 : c0;
  uint32_t j = 0, hi = nf;
  while (hi - j > 1) {
    const uint32_t mid = (j + hi) >> 1;
    if (S.fst[mid] <= p0) j = mid;
    else hi = mid;
  }
  const int64_t ce = c0 + 16 < (int64_t)W ? c0 + 16 : (int64_t)W;
  uint64_t acc0 = 0, acc1 = 0;  // the chunk's bytes 0..7, 8..15
  int64_t w = p0;
  while (w < ce) {
    while (w >= S.fst[j + 1]) j++;
    const int64_t fs = S.fst[j];
    const uint32_t r = (uint32_t)(w - fs);
    const uint32_t ends[6] = {S.e[0][j], S.e[1][j], S.e[2][j], S.e[3][j], S.e[4][j],
                              (uint32_t)(S.fst[j + 1] - fs)};
    uint32_t sg = 0;
#pragma unroll
    for (uint32_t q = 0; q < 5; q++) sg += r >= ends[q] ? 1u : 0u;
    const uint32_t a = sg ? ends[sg - 1] : 0u;
    const int64_t pe = fs + ends[sg] < ce ? fs + ends[sg] : ce;  // this piece: wire bytes [w, pe)
    const uint32_t q0 = (uint32_t)(w - c0), q1 = (uint32_t)(pe - c0);
    uint64_t v0, v1;  // 16 bytes from the piece's first byte on
    if (sg & 1u) {
      const uint8_t *sp = P.heap + S.src[sg >> 1][j] + (r - a);
      const uint32_t sh = (uint32_t)((uintptr_t)sp & 15);
      const uint4 *ab = reinterpret_cast<const uint4 *>(sp - sh);
      const uint4 b0 = ab[0];
      const uint4 b1 = sh + (q1 - q0) > 16u ? ab[1] : b0;  // (only blocks holding piece bytes)
      const uint4 x = enc_shift(b0, b1, sh);
      v0 = ((uint64_t)x.y << 32) | x.x;
      v1 = ((uint64_t)x.w << 32) | x.z;
    } else {
      const uint32_t lo = (uint32_t)(&S.lit[j][sg == 0 ? LIT0 : sg == 2 ? LIT2 : LIT4] - &S.lit[0][0]) + (r - a);
      v0 = enc_lds_u64(&S.lit[0][0], lo);
      v1 = enc_lds_u64(&S.lit[0][0], lo + 8u);
    }
    // shift left by q0 bytes, keep bytes [q0, q1)
    const uint32_t b = 8u * q0;
    uint64_t s0, s1;
    if (b == 0) s0 = v0, s1 = v1;
    else if (b < 64) s0 = v0 << b, s1 = (v1 << b) | (v0 >> (64u - b));
    else s0 = 0, s1 = v0 << (b - 64u);
    const uint32_t e = 8u * q1;
    const uint64_t m0 = (e >= 64 ? ~0ull : (1ull << e) - 1ull) & (b >= 64 ? 0ull : ~0ull << b);
    const uint64_t m1 = (e <= 64 ? 0ull : (e >= 128 ? ~0ull : (1ull << (e - 64u)) - 1ull)) &
                        (b <= 64 ? ~0ull : ~0ull << (b - 64u));
    acc0 |= s0 & m0;
    acc1 |= s1 & m1;
    w = pe;
  }
  if (c0 >= 0 && c0 + 16 <= (int64_t)W) {
    *reinterpret_cast<uint4 *>(P.out + c0) =
        make_uint4((uint32_t)acc0, (uint32_t)(acc0 >> 32), (uint32_t)acc1, (uint32_t)(acc1 >> 32));
  } else {  // the output's first or last chunk: only its own bytes
    for (int64_t x = p0; x < ce; x++) {
      const uint32_t q = (uint32_t)(x - c0);
      P.out[x] = (uint8_t)((q < 8 ? acc0 >> (8 * q) : acc1 >> (8 * (q - 8))) & 0xFF);
    }
  }
}

__global__ __launch_bounds__(ENC_OS_T) void enc_write_os(EncodeParams P) {
  __shared__ EncLds S;
  const uint64_t W = P.frame_off[P.n];
  if (W > P.cap) return;
  const uint32_t g = (uint32_t)((uintptr_t)P.out & 15);
  const uint64_t b = blockIdx.x;
  const int64_t bs = oblk_start(b, g);
  if (bs >= (int64_t)W) return;  // (whole workgroup)
  const int64_t be = bs + (int64_t)ENC_BS;
  const uint64_t f0 = P.oblk_first[b];
  // frames [f0, f1) touch the block (the frame holding the next block's first byte may start at be
  // exactly: laid out, never looked up)
  const uint64_t f1 = be < (int64_t)W ? min(P.oblk_first[b + 1] + 1, P.n) : P.n;
  const uint32_t t = threadIdx.x;
  if (f1 - f0 > ENC_FMAX) {
    if (t == 0) P.dense[atomicAdd(P.dense_n, 1u)] = (uint32_t)b;
    return;
  }
  const uint32_t nf = (uint32_t)(f1 - f0);
  bool big = false;
  if (t < nf) {
    const drp_change_src &s = P.src;
    const uint64_t i = f0 + t;
    const uint32_t fl = s.flags[i];
    const bool sub = (fl & DRP_F_SUBSET) != 0, val = (fl & DRP_F_VALUE) != 0;
    const uint32_t sl = sub ? s.subset_len[i] : 0u, kl = s.key_len[i], vl = val ? s.value_len[i] : 0u;
    const uint64_t pl = payload_len(s, i);
    uint8_t *l = S.lit[t];
    uint32_t x = put_lit(l + LIT0, vseg(pl + 1));
    l[LIT0 + x++] = DRP_TYPE_CHANGE;
    if (sub) {
      l[LIT0 + x++] = 0x0a;
      x += put_lit(l + LIT0 + x, vseg(sl));
    }
    uint32_t y = 0;
    l[LIT2 + y++] = 0x12;
    y += put_lit(l + LIT2 + y, vseg(kl));
    uint32_t z = 0;
    l[LIT4 + z++] = 0x18;
    z += put_lit(l + LIT4 + z, vseg(s.change[i]));
    l[LIT4 + z++] = 0x20;
    z += put_lit(l + LIT4 + z, vseg(s.from[i]));
    l[LIT4 + z++] = 0x28;
    z += put_lit(l + LIT4 + z, vseg(s.to[i]));
    if (val) {
      l[LIT4 + z++] = 0x32;
      z += put_lit(l + LIT4 + z, vseg(vl));
    }
    const uint64_t fs = P.frame_off[i];
    const uint64_t e0 = x, e1 = e0 + sl, e2 = e1 + y, e3 = e2 + kl, e4 = e3 + z, e5 = e4 + vl;
    big = e5 >= ENC_F_DENSE_FRAME;
    S.fst[t] = (int64_t)fs;
    if (t == nf - 1) S.fst[nf] = (int64_t)(fs + e5);
    S.e[0][t] = (uint32_t)e0;
    S.e[1][t] = (uint32_t)e1;
    S.e[2][t] = (uint32_t)e2;
    S.e[3][t] = (uint32_t)e3;
    S.e[4][t] = (uint32_t)e4;
    S.src[0][t] = s.subset_off[i] * (sub ? 1u : 0u);
    S.src[1][t] = s.key_off[i];
    S.src[2][t] = val ? s.value_off[i] : 0ull;
  }
  if (t == 0) S.nmix = 0;
  if (__syncthreads_or(big)) {  // (a frame of 2^31 bytes or more: the per-frame writer)
    if (t == 0) P.dense[atomicAdd(P.dense_n, 1u)] = (uint32_t)b;
    return;
  }
  // ENC_NB batches of ENC_U chunks per lane, strided by the workgroup (each pass of the workgroup
  // stores 4 KiB contiguous). In a batch every chunk's frame and segment are looked up first, then
  // every heap load of the lane's whole-copy chunks is issued, then the stores: a lane keeps up to
  // 2 * ENC_U loads in flight. fm: the lane's chunks written here (the rest: the piece loop below).
  uint32_t fm = 0;
#pragma unroll 1
  for (uint32_t k = 0; k < ENC_NB; k++) {
    const uint4 *sa[ENC_U];
    uint32_t shv[ENC_U];
    bool fast[ENC_U];
#pragma unroll
    for (uint32_t u = 0; u < ENC_U; u++) {
      const int64_t c0 = bs + 16 * (int64_t)(t + (k * ENC_U + u) * ENC_OS_T);
      fast[u] = false;
      sa[u] = nullptr;
      shv[u] = 0;
      if (c0 >= 0 && c0 + 16 <= (int64_t)W) {
        uint32_t lo = 0, hi = nf;  // fst[lo] <= c0 < fst[hi]
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (S.fst[mid] <= c0) lo = mid;
          else hi = mid;
        }
        const uint32_t r = (uint32_t)(c0 - S.fst[lo]);
        const uint32_t fe = (uint32_t)(S.fst[lo + 1] - S.fst[lo]);
        const uint32_t e0 = S.e[0][lo], e1 = S.e[1][lo], e2 = S.e[2][lo], e3 = S.e[3][lo], e4 = S.e[4][lo];
        // a copy segment holding the whole chunk: subset [e0, e1), key [e2, e3), value [e4, end)
        uint32_t a = 0xFFFFFFFFu, seg = 0;
        if (r >= e4 && r + 16 <= fe) a = e4, seg = 2;
        else if (r >= e2 && r + 16 <= e3) a = e2, seg = 1;
        else if (r >= e0 && r + 16 <= e1) a = e0, seg = 0;
        if (a != 0xFFFFFFFFu) {
          const uint8_t *sp = P.heap + S.src[seg][lo] + (r - a);
          shv[u] = (uint32_t)((uintptr_t)sp & 15);
          sa[u] = reinterpret_cast<const uint4 *>(sp - shv[u]);
          fast[u] = true;
        }
      }
    }
    uint4 v0[ENC_U], v1[ENC_U];
#if DRP_ENC_DPP
    // a lane's second block is the next lane's first when that lane copies the next 16 source
    // bytes (one copy segment across the two chunks): taken from it by a wave shift (DPP) instead
    // of loaded again; the lanes at segment ends and lane 63 load it
    bool own1[ENC_U];
#pragma unroll
    for (uint32_t u = 0; u < ENC_U; u++) {
      const uintptr_t a = fast[u] ? (uintptr_t)sa[u] : 0;
      const uint32_t nlo = (uint32_t)__builtin_amdgcn_update_dpp(0u, (uint32_t)a, 0x130, 0xF, 0xF, false);
      const uint32_t nhi = (uint32_t)__builtin_amdgcn_update_dpp(0u, (uint32_t)(a >> 32), 0x130, 0xF, 0xF, false);
      const uintptr_t na = ((uintptr_t)nhi << 32) | nlo;
      own1[u] = fast[u] && shv[u] && na != a + 16;
    }
#pragma unroll
    for (uint32_t u = 0; u < ENC_U; u++) {
      v0[u] = v1[u] = make_uint4(0, 0, 0, 0);
      if (fast[u]) v0[u] = sa[u][0];
      if (own1[u]) v1[u] = sa[u][1];
    }
#pragma unroll
    for (uint32_t u = 0; u < ENC_U; u++) {
      const uint4 n = make_uint4((uint32_t)__builtin_amdgcn_update_dpp(0u, v0[u].x, 0x130, 0xF, 0xF, false),
                                 (uint32_t)__builtin_amdgcn_update_dpp(0u, v0[u].y, 0x130, 0xF, 0xF, false),
                                 (uint32_t)__builtin_amdgcn_update_dpp(0u, v0[u].z, 0x130, 0xF, 0xF, false),
                                 (uint32_t)__builtin_amdgcn_update_dpp(0u, v0[u].w, 0x130, 0xF, 0xF, false));
      if (!own1[u]) v1[u] = n;
    }
#else
#pragma unroll
    for (uint32_t u = 0; u < ENC_U; u++) {
      v0[u] = v1[u] = make_uint4(0, 0, 0, 0);
      if (fast[u]) {
        v0[u] = sa[u][0];
        if (shv[u]) v1[u] = sa[u][1];
      }
    }
#endif
#pragma unroll
    for (uint32_t u = 0; u < ENC_U; u++)
      if (fast[u]) {
        *reinterpret_cast<uint4 *>(P.out + bs + 16 * (int64_t)(t + (k * ENC_U + u) * ENC_OS_T)) =
            shv[u] ? enc_shift(v0[u], v1[u], shv[u]) : v0[u];
        fm |= 1u << (k * ENC_U + u);
      }
  }
  // the mixed chunks, listed in LDS and spread one per lane (a lane's own mixed chunks would run
  // one after another, each a chain of dependent piece loads)
#pragma unroll 1
  for (uint32_t u = 0; u < ENC_NB * ENC_U; u++) {
    const int64_t c0 = bs + 16 * (int64_t)(t + u * ENC_OS_T);
    if (((fm >> u) & 1u) || c0 >= (int64_t)W) continue;
    const uint32_t slot = atomicAdd(&S.nmix, 1u);
    if (slot < ENC_MIXCAP) S.mix[slot] = (uint16_t)(t + u * ENC_OS_T);
    else enc_mixed_chunk(P, S, nf, W, c0);  // (not reached: ENC_MIXCAP bounds the count)
  }
  __syncthreads();
  const uint32_t nm = min(S.nmix, ENC_MIXCAP);
#pragma unroll 1
  for (uint32_t x = t; x < nm; x += ENC_OS_T) enc_mixed_chunk(P, S, nf, W, bs + 16 * (int64_t)S.mix[x]);
}

// The frames of the blocks enc_write_os left (more than ENC_FMAX frames, or a frame of 2^31 bytes
// or more), one wave per frame; a frame shared with a neighbouring block is rewritten with the
// same bytes.
__global__ __launch_bounds__(256) void enc_write_dense(EncodeParams P) {
  const uint64_t W = P.frame_off[P.n];
  if (W > P.cap) return;
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint32_t nd = *P.dense_n;
  const uint32_t g = (uint32_t)((uintptr_t)P.out & 15);
  for (uint32_t d = blockIdx.x; d < nd; d += gridDim.x) {
    const uint64_t b = P.dense[d];
    const int64_t be = oblk_start(b, g) + (int64_t)ENC_BS;
    const uint64_t f0 = P.oblk_first[b];
    uint64_t f1 = P.n;
    if (be < (int64_t)W) {
      const uint64_t nb = P.oblk_first[b + 1];
      f1 = P.frame_off[nb] < (uint64_t)be ? nb + 1 : nb;
    }
    for (uint64_t i = f0 + wv; i < f1; i += 4) write_frame(P, i, lane);
  }
}

// exclusive prefix of stats[i].frames (single block)
__global__ __launch_bounds__(1024) void index_scan_kernel(const drp_stream_stats *stats, uint64_t count,
                                                          uint64_t *base) {
  __shared__ uint64_t part[1024];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t c0 = 0; c0 < count; c0 += 1024) {
    const uint64_t i = c0 + threadIdx.x;
    const uint64_t v0 = i < count ? stats[i].frames : 0;
    part[threadIdx.x] = v0;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
      uint64_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    if (i < count) base[i] = carry + part[threadIdx.x] - v0;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
}

__global__ void stats_kernel(const drp_stream_result *res, const uint64_t *stream_off, uint64_t n,
                             drp_stream_stats *stats) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  drp_stream_stats o;
  o.frames = res[s].frames;
  o.changes = res[s].changes;
  o.blobs = res[s].blobs;
  o.wire_bytes = res[s].consumed;
  (void)stream_off;
  stats[s] = o;
}

}  // namespace drp

using namespace drp;

// output blocks of the write for an output of capacity cap (the grid covers the largest output
// the capacity allows; blocks past the real end exit at once)
extern "C" uint64_t drp_encode_out_blocks(uint64_t cap) { return (cap + 15) / ENC_BS + 2; }

extern "C" void drp_dbg_mark(const char *name, hipStream_t st);  // (drp_api.hip: DRP_WATCHDOG)

extern "C" hipError_t drp_launch_encode(const EncodeParams *Pp, hipStream_t st) {
  EncodeParams P = *Pp;
  if (P.n == 0) return hipSuccess;
  const uint64_t nblk = (P.n + SCAN_BLK - 1) / SCAN_BLK;
  hipLaunchKernelGGL(enc_size_kernel, dim3((uint32_t)nblk), dim3(SCAN_BLK), 0, st, P);
  hipLaunchKernelGGL(enc_blocksum_kernel, dim3(1), dim3(SCAN_BLK), 0, st, P, nblk);
  hipLaunchKernelGGL(enc_addbase_kernel, dim3((uint32_t)nblk), dim3(SCAN_BLK), 0, st, P);
  drp_dbg_mark("enc_size+scan", st);
  if (P.out && DRP_ENC_OS && P.nob && P.nob < (1ull << 31)) {
    hipLaunchKernelGGL(enc_oblk_kernel, dim3((uint32_t)((P.n + 255) / 256)), dim3(256), 0, st, P);
    hipError_t e = hipMemsetAsync(P.dense_n, 0, 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(enc_write_os, dim3((uint32_t)P.nob), dim3(ENC_OS_T), 0, st, P);
    drp_dbg_mark("enc_write_os", st);
    hipLaunchKernelGGL(enc_write_dense, dim3(2048), dim3(256), 0, st, P);
    drp_dbg_mark("enc_write_dense", st);
  } else if (P.out) {
    uint64_t waves = P.n < DRP_ENC_WAVES ? P.n : DRP_ENC_WAVES;  // one frame per wave at a time
    uint32_t grid = (uint32_t)((waves * 64 + 255) / 256);
    hipLaunchKernelGGL(enc_write_kernel, dim3(grid), dim3(256), 0, st, P);
  }
  return hipGetLastError();
}

extern "C" hipError_t drp_launch_index_scan(const drp_stream_stats *stats, uint64_t count, uint64_t *base,
                                            hipStream_t st) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(index_scan_kernel, dim3(1), dim3(1024), 0, st, stats, count, base);
  return hipGetLastError();
}

extern "C" hipError_t drp_launch_stats_from_results(const drp_stream_result *res, const uint64_t *stream_off,
                                                    uint64_t nstreams, drp_stream_stats *stats, hipStream_t st) {
  if (nstreams == 0) return hipSuccess;
  const uint32_t grid = (uint32_t)((nstreams + 255) / 256);
  hipLaunchKernelGGL(stats_kernel, dim3(grid), dim3(256), 0, st, res, stream_off, nstreams, stats);
  return hipGetLastError();
}
