// drp_keys.hip — on-GPU key post-processing: for every delivered Change frame,
// a 64-bit XXH64 (seed 0) of the key bytes and two flags, DRP_F_KEY_ASCII (every byte < 0x80)
// and DRP_F_KEY_UTF8 (the bytes are well-formed UTF-8, RFC 3629: no overlong forms, no
// surrogates, nothing above U+10FFFF). The reference turns every key into a JS string with
// buf.toString('utf-8') inside messages.Change.decode (decode.js:210-213); with these columns
// a consumer that only needs key bytes or a hash (dat storage) skips that, and the JS layer
// takes the cheaper latin1 path for ASCII keys (same string).
//
// The hash column is optional (DRP_KEY_POST_FLAGS: flags only). One thread per frame, grid-stride; runs after emission over the frames the decode wrote
// (their count is the last tile's base + count), reading the key bytes from the batch in HBM.
#include "drp_device.h"
#include "drp_kernels.h"

namespace drp {
namespace keys {

constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                   P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;

__device__ __forceinline__ uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t round1(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }
__device__ __forceinline__ uint64_t merge(uint64_t acc, uint64_t v) { return (acc ^ round1(0, v)) * P1 + P4; }

// little-endian reads of byte-addressed global memory (keys have any alignment)
__device__ __forceinline__ uint64_t rd64(const uint8_t *p) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}
__device__ __forceinline__ uint32_t rd32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// XXH64, seed 0 (the published algorithm; tests check it against python-xxhash)
__device__ uint64_t xxh64(const uint8_t *p, uint32_t len) {
  const uint8_t *end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    const uint8_t *lim = end - 32;
    do {
      v1 = round1(v1, rd64(p));
      v2 = round1(v2, rd64(p + 8));
      v3 = round1(v3, rd64(p + 16));
      v4 = round1(v4, rd64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = merge(h, v1);
    h = merge(h, v2);
    h = merge(h, v3);
    h = merge(h, v4);
  } else {
    h = P5;
  }
  h += len;
  while (p + 8 <= end) {
    h ^= round1(0, rd64(p));
    h = rotl(h, 27) * P1 + P4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32(p) * P1;
    h = rotl(h, 23) * P2 + P3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * P5;
    h = rotl(h, 11) * P1;
    p++;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

// DRP_F_KEY_ASCII | DRP_F_KEY_UTF8 for the key bytes
__device__ uint32_t key_class(const uint8_t *p, uint32_t len) {
  uint32_t i = 0;
  bool ascii = true;
  while (i < len) {
    const uint32_t b = p[i];
    if (b < 0x80u) {
      i++;
      continue;
    }
    ascii = false;
    uint32_t need, lo = 0x80u, hi = 0xBFu;
    if (b >= 0xC2u && b <= 0xDFu) need = 1;
    else if (b >= 0xE0u && b <= 0xEFu) {
      need = 2;
      if (b == 0xE0u) lo = 0xA0u;        // no overlong 3-byte forms
      else if (b == 0xEDu) hi = 0x9Fu;   // no surrogates
    } else if (b >= 0xF0u && b <= 0xF4u) {
      need = 3;
      if (b == 0xF0u) lo = 0x90u;        // no overlong 4-byte forms
      else if (b == 0xF4u) hi = 0x8Fu;   // nothing above U+10FFFF
    } else {
      return 0;
    }
    if (i + need >= len) return 0;  // truncated sequence
    const uint32_t b1 = p[i + 1];
    if (b1 < lo || b1 > hi) return 0;
    for (uint32_t k = 2; k <= need; k++) {
      const uint32_t bk = p[i + k];
      if (bk < 0x80u || bk > 0xBFu) return 0;
    }
    i += need + 1;
  }
  return (ascii ? DRP_F_KEY_ASCII : 0u) | DRP_F_KEY_UTF8;
}

__global__ __launch_bounds__(256) void key_post_kernel(const uint8_t *bytes, const uint64_t *tile_prefix,
                                                       uint64_t nstreams, const uint64_t *tile_base,
                                                       const uint64_t *tile_count, uint64_t cap,
                                                       const uint64_t *payload_off, const uint8_t *type,
                                                       const uint32_t *key_off, const uint32_t *key_len,
                                                       uint8_t *flags, uint64_t *key_hash,
                                                       const uint32_t *abort_flag, uint32_t abort_mask) {
  if (abort_flag && (*abort_flag & abort_mask)) return;  // (a failed prediction: run again after its repair)
  const uint64_t nt = tile_prefix[nstreams];
  uint64_t total = nt ? tile_base[nt - 1] + tile_count[nt - 1] : 0;
  if (total > cap) total = cap;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total; f += stride) {
    if ((type[f] & 0x3Fu) != DRP_TYPE_CHANGE) continue;
    const uint32_t fl = flags[f];
    if (fl & DRP_F_BAD) {
      if (key_hash) key_hash[f] = 0;
      continue;
    }
    const uint8_t *k = bytes + payload_off[f] + key_off[f];
    const uint32_t n = key_len[f];
    if (key_hash) key_hash[f] = xxh64(k, n);
    flags[f] = (uint8_t)(fl | key_class(k, n));
  }
}

}  // namespace keys
}  // namespace drp

extern "C" hipError_t drp_launch_key_post(const uint8_t *bytes, const uint64_t *tile_prefix, uint64_t nstreams,
                                          const uint64_t *tile_base, const uint64_t *tile_count, uint64_t cap,
                                          const drp_frames *fr, const drp_changes *co, int flags_only,
                                          const uint32_t *abort_flag, uint32_t abort_mask, hipStream_t st) {
  // the hash when the caller gave a column for it; the key flags also without one (flags_only)
  if ((!co->key_hash && !flags_only) || cap == 0) return hipSuccess;
  uint64_t blocks = (cap + 255) / 256;
  if (blocks > 65536) blocks = 65536;  // grid-stride beyond
  hipLaunchKernelGGL(drp::keys::key_post_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, bytes, tile_prefix,
                     nstreams, tile_base, tile_count, cap, fr->payload_off, fr->type, co->key_off, co->key_len,
                     co->flags, co->key_hash, abort_flag, abort_mask);
  return hipGetLastError();
}
