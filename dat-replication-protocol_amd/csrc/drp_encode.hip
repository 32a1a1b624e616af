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

#ifndef DRP_ENC_UNROLL
#define DRP_ENC_UNROLL 1  // 16-byte blocks per lane in flight in the bulk copy
#endif
#ifndef DRP_ENC_NT
#define DRP_ENC_NT 0  // 1: non-temporal heap loads and wire stores in the bulk copy (A/B)
#endif
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 enc_ld(const uint4 *p) {
#if DRP_ENC_NT
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}
__device__ __forceinline__ void enc_st(uint4 *p, uint4 v) {
#if DRP_ENC_NT
  u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(p));
#else
  *p = v;
#endif
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
#ifndef DRP_ENC_PIPE
#define DRP_ENC_PIPE 0  // 1: the next step's loads issued before this step's store (A/B)
#endif
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
#if DRP_ENC_UNROLL > 1
  // DRP_ENC_UNROLL blocks per lane in flight: every load of a step is issued before its stores
  for (; b + 64 * (DRP_ENC_UNROLL - 1) < nb; b += 64 * DRP_ENC_UNROLL) {
    uint4 lo[DRP_ENC_UNROLL], hi[DRP_ENC_UNROLL];
#pragma unroll
    for (int u = 0; u < DRP_ENC_UNROLL; u++) {
      lo[u] = enc_ld(sa + b + 64 * u);
      hi[u] = sh ? enc_ld(sa + b + 64 * u + 1) : lo[u];
    }
#pragma unroll
    for (int u = 0; u < DRP_ENC_UNROLL; u++) enc_st(da + b + 64 * u, enc_shift(lo[u], hi[u], sh));
  }
#endif
#if DRP_ENC_PIPE
  // software-pipelined: step b + 64's two blocks are loaded before step b's store
  if (b < nb) {
    uint4 lo = enc_ld(sa + b), hi = sh ? enc_ld(sa + b + 1) : lo;
    for (; b + 64 < nb; b += 64) {
      const uint4 lo2 = enc_ld(sa + b + 64), hi2 = sh ? enc_ld(sa + b + 65) : lo2;
      enc_st(da + b, enc_shift(lo, hi, sh));
      lo = lo2;
      hi = hi2;
    }
    enc_st(da + b, enc_shift(lo, hi, sh));
    b += 64;
  }
#else
  for (; b < nb; b += 64) {
    const uint4 lo = enc_ld(sa + b);
    enc_st(da + b, sh == 0 ? lo : enc_shift(lo, enc_ld(sa + b + 1), sh));
  }
#endif
  const uint32_t tail = (uint32_t)(n & 15);
  if (lane < tail) dst[(nb << 4) + lane] = src[(nb << 4) + lane];
}

#ifndef DRP_ENC_COPY2
#define DRP_ENC_COPY2 0  // 1: wave_copy2 (measured slower on C5: 4.23 vs 2.92 ms)
#endif
#ifndef DRP_ENC_BATCH
#define DRP_ENC_BATCH 8  // 16-byte blocks per lane loaded before any is stored (wave_copy2)
#endif
// wave_copy2: the same aligned-store copy with up to DRP_ENC_BATCH blocks per lane loaded before
// any is stored (a 4 KB value is one batch: every load of the copy is in flight at once), and
// each source block loaded once: the second block a lane's funnel shift needs is the next lane's
// first (a lane permute), lane 63 taking the first block of the next column. Copies under 64
// bytes are one byte per lane.
__device__ __forceinline__ void wave_copy2(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src, uint64_t n,
                                           uint32_t lane) {
  if (n < 64) {
    if (lane < n) dst[lane] = src[lane];
    return;
  }
  const uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
  if (lane < head) dst[lane] = src[lane];
  dst += head;
  src += head;
  n -= head;
  const uint64_t nb = n >> 4;
  const uint32_t tail = (uint32_t)(n & 15);
  const uint32_t sh = (uint32_t)((uintptr_t)src & 15);
  const uint4 *sa = reinterpret_cast<const uint4 *>(src - sh);
  uint4 *da = reinterpret_cast<uint4 *>(dst);
  // source blocks needed: [0, nb) and, when shifted, block nb (it holds source bytes: the last
  // byte is past 16 nb - sh + 15 whenever sh > 0 and the copy is not empty)
  const uint64_t ns = nb + (sh ? 1 : 0);
  const int nxt = (int)(((lane + 1) & 63u) << 2);
  for (uint64_t b0 = 0; b0 < nb; b0 += 64 * DRP_ENC_BATCH) {
    uint4 v[DRP_ENC_BATCH + 1];
#pragma unroll
    for (int u = 0; u <= DRP_ENC_BATCH; u++) {
      const uint64_t b = b0 + 64u * u + lane;
      v[u] = (u < DRP_ENC_BATCH || lane == 0) && b < ns ? enc_ld(sa + b) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < DRP_ENC_BATCH; u++) {
      const uint64_t b = b0 + 64u * u + lane;
      if (b0 + 64u * u >= nb) break;
      uint4 w = v[u];
      if (sh) {
        const uint4 src_hi = lane == 0 ? v[u + 1] : v[u];  // (lane 63 reads lane 0: the next column)
        uint4 hi;
        hi.x = (uint32_t)__builtin_amdgcn_ds_bpermute(nxt, (int)src_hi.x);
        hi.y = (uint32_t)__builtin_amdgcn_ds_bpermute(nxt, (int)src_hi.y);
        hi.z = (uint32_t)__builtin_amdgcn_ds_bpermute(nxt, (int)src_hi.z);
        hi.w = (uint32_t)__builtin_amdgcn_ds_bpermute(nxt, (int)src_hi.w);
        w = enc_shift(w, hi, sh);
      }
      if (b < nb) enc_st(da + b, w);
    }
  }
  if (lane < tail) dst[(nb << 4) + lane] = src[(nb << 4) + lane];
}

#ifndef DRP_ENC_WAVES
#define DRP_ENC_WAVES 65536  // waves of the write kernel (grid-stride over frames)
#endif
#ifndef DRP_ENC_LANEPREFIX
#define DRP_ENC_LANEPREFIX 1  // 0: lane 0 writes the prefixes byte by byte from private arrays
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

#if DRP_ENC_COPY2
#define WAVE_COPY wave_copy2
#else
#define WAVE_COPY wave_copy
#endif
// one wave per frame (grid-stride over frames)
#ifndef DRP_ENC_MINW
#define DRP_ENC_MINW 0  // > 0: min waves per SIMD for the write kernel (8: 64 VGPRs, a 28-byte spill)
#endif
#if DRP_ENC_MINW
__global__ __launch_bounds__(256, DRP_ENC_MINW) void enc_write_kernel(EncodeParams P) {
#else
__global__ __launch_bounds__(256) void enc_write_kernel(EncodeParams P) {
#endif
  const uint32_t lane = lane_id();
  const uint64_t wid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  if (P.frame_off[P.n] > P.cap) return;
  const drp_change_src &s = P.src;
  for (uint64_t i = wid; i < P.n; i += nw) {
    uint8_t *o = P.out + P.frame_off[i];
    const uint32_t fl = s.flags[i];
    const uint64_t pl = payload_len(s, i);
#if DRP_ENC_LANEPREFIX
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
#else
    // header + subset prefix
    uint8_t pre[32];
    uint32_t h = venc(pl + 1, pre);
    pre[h++] = DRP_TYPE_CHANGE;
    uint64_t off = 0;
    if (lane == 0)
      for (uint32_t k = 0; k < h; k++) o[k] = pre[k];
    off = h;
    if (fl & DRP_F_SUBSET) {
      uint8_t t[12];
      uint32_t m = 0;
      t[m++] = 0x0a;
      m += venc(s.subset_len[i], t + m);
      if (lane == 0)
        for (uint32_t k = 0; k < m; k++) o[off + k] = t[k];
      off += m;
      wave_copy(o + off, P.heap + s.subset_off[i], s.subset_len[i], lane);
      off += s.subset_len[i];
    }
    {
      uint8_t t[12];
      uint32_t m = 0;
      t[m++] = 0x12;
      m += venc(s.key_len[i], t + m);
      if (lane == 0)
        for (uint32_t k = 0; k < m; k++) o[off + k] = t[k];
      off += m;
      wave_copy(o + off, P.heap + s.key_off[i], s.key_len[i], lane);
      off += s.key_len[i];
    }
    {
      uint8_t t[48];  // 3 tags + 3 u64 varints (<= 10 B each) + value tag + u32 length varint = 39 B
      uint32_t m = 0;
      t[m++] = 0x18;
      m += venc(s.change[i], t + m);
      t[m++] = 0x20;
      m += venc(s.from[i], t + m);
      t[m++] = 0x28;
      m += venc(s.to[i], t + m);
      if (fl & DRP_F_VALUE) {
        t[m++] = 0x32;
        m += venc(s.value_len[i], t + m);
      }
      if (lane == 0)
        for (uint32_t k = 0; k < m; k++) o[off + k] = t[k];
      off += m;
    }
    if (fl & DRP_F_VALUE) wave_copy(o + off, P.heap + s.value_off[i], s.value_len[i], lane);
#endif
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

extern "C" hipError_t drp_launch_encode(const EncodeParams *Pp, hipStream_t st) {
  EncodeParams P = *Pp;
  if (P.n == 0) return hipSuccess;
  const uint64_t nblk = (P.n + SCAN_BLK - 1) / SCAN_BLK;
  hipLaunchKernelGGL(enc_size_kernel, dim3((uint32_t)nblk), dim3(SCAN_BLK), 0, st, P);
  hipLaunchKernelGGL(enc_blocksum_kernel, dim3(1), dim3(SCAN_BLK), 0, st, P, nblk);
  hipLaunchKernelGGL(enc_addbase_kernel, dim3((uint32_t)nblk), dim3(SCAN_BLK), 0, st, P);
  if (P.out) {
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
