// drp_device.h — device-side building blocks shared by the gfx950 kernels.
//
// Header grammar (README.md:63-71, decode.js:251-262): varint(L) | id | payload[L-1].
// Change grammar (messages/schema.proto:1-8, protocol-buffers@2 generated decoder).
// The policy for inputs the reference leaves undefined is documented in DESIGN.md §policy
// and is identical to oracle/drp_oracle.c.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/drp.h"

namespace drp {

constexpr int WAVE = 64;

// Exit/position encoding used by the frame walkers and the cross-tile look-back.
// Real stream positions are < 2^60. MARK_TERM|p = the chain ends at node p (tail or error).
constexpr uint64_t MARK_TERM = 1ull << 61;
constexpr uint64_t MARK_NONE = 1ull << 62;  // "no speculative exit" (successor must wait)
constexpr uint64_t POS_MASK = (1ull << 60) - 1;

// Header kinds (per candidate frame start).
enum : uint32_t {
  H_VALID = 0,        // complete header, frame ends at or before the stream end
  H_TAIL_HDR = 1,     // header runs past the stream end (not delivered)
  H_TAIL_CHANGE = 2,  // change frame whose payload runs past the stream end (not delivered)
  H_TAIL_BLOB = 3,    // blob frame whose payload runs past the stream end (delivered, partial)
  H_ERR_VARINT = 4,   // > 10 byte length varint or >= 2^64 (policy)
  H_ERR_TYPE = 5,     // id >= 3 (decode.js:159-161)
  H_ERR_LEN = 6,      // L == 0 on id 1/2 (policy)
};

struct Hdr {
  uint64_t succ;  // next frame start (H_VALID only)
  uint64_t L;     // declared length (id byte + payload)
  uint32_t kind;
  uint32_t id;
  uint32_t vlen;  // varint bytes
};

__device__ __forceinline__ bool hdr_delivered(const Hdr &h) {
  return (h.kind == H_VALID && h.id != 0) || h.kind == H_TAIL_BLOB;
}

// 16 bytes starting at LDS byte offset `o` (any alignment). The LDS buffer must have
// >= 24 bytes of slack after the last byte ever addressed.
__device__ __forceinline__ void lds_win16(const uint8_t *lds, uint32_t o, uint64_t &w0,
                                          uint64_t &w1) {
  const uint64_t *q = reinterpret_cast<const uint64_t *>(lds + (o & ~7u));
  uint64_t a = q[0], b = q[1], c = q[2];
  uint32_t sh = (o & 7u) * 8u;
  if (sh) {
    w0 = (a >> sh) | (b << (64 - sh));
    w1 = (b >> sh) | (c << (64 - sh));
  } else {
    w0 = a;
    w1 = b;
  }
}

__device__ __forceinline__ uint32_t win_byte(uint64_t w0, uint64_t w1, uint32_t i) {
  return (uint32_t)(((i < 8) ? (w0 >> (8 * i)) : (w1 >> (8 * (i - 8)))) & 0xFF);
}

// Decode a varint from a 16-byte window starting at byte `i0` (i0 + 10 <= 16 not required:
// bytes past the window read as 0 and the caller bounds-checks with `avail`).
// Returns length (1..10), 0 if it runs past `avail`, -1 if malformed (> 10 bytes / >= 2^64).
__device__ __forceinline__ int win_varint(uint64_t w0, uint64_t w1, uint32_t i0, uint64_t avail,
                                          uint64_t &v) {
  v = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    if ((uint64_t)k >= avail) return 0;
    uint32_t b = win_byte(w0, w1, i0 + k);
    uint64_t bits = b & 0x7F;
    if (k == 9 && bits > 1) return -1;
    v |= bits << (7 * k);
    if (!(b & 0x80)) return k + 1;
  }
  return -1;
}

// Parse the frame header starting at absolute stream position p from the LDS image whose
// byte 0 is absolute position `base`. `se` = stream end.
__device__ __forceinline__ Hdr parse_hdr_lds(const uint8_t *lds, uint64_t base, uint64_t p,
                                             uint64_t se) {
  Hdr h;
  uint64_t w0, w1;
  lds_win16(lds, (uint32_t)(p - base), w0, w1);
  uint64_t avail = se - p;
  uint64_t L;
  int k = win_varint(w0, w1, 0, avail, L);
  h.succ = 0;
  h.L = L;
  h.id = 0;
  h.vlen = (uint32_t)(k > 0 ? k : 0);
  if (k == 0) {
    h.kind = H_TAIL_HDR;
    return h;
  }
  if (k < 0) {
    // a > 10 byte varint that is cut by the stream end is still an incomplete header
    h.kind = (avail < 11) ? H_TAIL_HDR : H_ERR_VARINT;
    return h;
  }
  if ((uint64_t)k >= avail) {  // id byte not yet available
    h.kind = H_TAIL_HDR;
    return h;
  }
  uint32_t id = win_byte(w0, w1, (uint32_t)k);
  h.id = id;
  if (id >= 3) {
    h.kind = H_ERR_TYPE;
    return h;
  }
  if (id == 0) {
    h.kind = H_VALID;
    h.succ = p + (uint64_t)k + 1;
    return h;
  }
  if (L == 0) {
    h.kind = H_ERR_LEN;
    return h;
  }
  // frame = k header bytes + L bytes (id + payload)
  if (L > avail - (uint64_t)k) {
    h.kind = (id == 1) ? H_TAIL_CHANGE : H_TAIL_BLOB;
    return h;
  }
  h.kind = H_VALID;
  h.succ = p + (uint64_t)k + L;
  return h;
}

// Byte readers for the Change decoder.
struct LdsReader {
  static constexpr bool kFast = true;  // two-byte peeks are cheap: decode_change fast path
  const uint8_t *lds;
  uint64_t base;  // absolute position of lds[0]
  uint64_t lim;   // absolute end of valid LDS bytes (exclusive)
  __device__ __forceinline__ bool ok(uint64_t p, uint64_t n) const { return p + n <= lim; }
  __device__ __forceinline__ void win(uint64_t p, uint64_t &w0, uint64_t &w1) const {
    lds_win16(lds, (uint32_t)(p - base), w0, w1);
  }
  // bytes p..p+3 and p+4..p+7 (three aligned dword reads; the buffer is 4-byte aligned and has
  // >= 12 bytes of slack after lim)
  __device__ __forceinline__ void win8(uint64_t p, uint32_t &w, uint32_t &wn) const {
    const uint32_t o = (uint32_t)(p - base), sh = (o & 3u) * 8u;
    const uint32_t *q = reinterpret_cast<const uint32_t *>(lds) + (o >> 2);
    const uint32_t a0 = q[0], a1 = q[1], a2 = q[2];
    w = __builtin_amdgcn_alignbit(a1, a0, sh);
    wn = __builtin_amdgcn_alignbit(a2, a1, sh);
  }
};

struct GlobalReader {
  static constexpr bool kFast = false;
  const uint8_t *g;
  uint64_t lim;  // absolute end of readable bytes
  __device__ __forceinline__ bool ok(uint64_t p, uint64_t n) const { return p + n <= lim; }
  __device__ __forceinline__ void win(uint64_t p, uint64_t &w0, uint64_t &w1) const {
    w0 = 0;
    w1 = 0;
    // byte loads; only used for the rare frame whose fields leave the LDS image
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint64_t b = (p + i < lim) ? (uint64_t)g[p + i] : 0ull;
      if (i < 8)
        w0 |= b << (8 * i);
      else
        w1 |= b << (8 * (i - 8));
    }
  }
};

struct ChangeCols {
  uint32_t key_off, key_len, subset_off, subset_len, value_off, value_len;
  uint64_t change, from, to;
  uint32_t flags;  // DRP_F_*
  uint32_t err;    // DRP_ERR_NONE / DRP_ERR_CHANGE / DRP_ERR_REQUIRED ; 0xFFFF = needs bytes out of reach
};

constexpr uint64_t JS_SAFE = 1ull << 53;
constexpr uint32_t ERR_UNREACHABLE = 0xFFFFu;

// Restatement of the protocol-buffers@2 generated decoder for Change
// (messages/schema.proto:1-8; oracle_change_decode in oracle/drp_oracle.c is the same
// algorithm): switch on tag = ToInt32(prefix) >> 3, wire type unchecked for known tags,
// unknown tags skipped by wire type, last value wins. Only field headers are read: string
// and bytes contents are skipped, so a 4 KB value costs one window load.
template <class R>
__device__ __forceinline__ ChangeCols decode_change(const R &rd, uint64_t pstart, uint64_t len) {
  ChangeCols c;
  c.key_off = c.key_len = c.subset_off = c.subset_len = c.value_off = c.value_len = 0;
  c.change = c.from = c.to = 0;
  c.flags = 0;
  c.err = 0;
  uint32_t found = 0;
  uint64_t off = 0;
  while (off < len) {
    uint64_t avail = len - off;
    if constexpr (R::kFast) if (avail >= 2 && rd.ok(pstart + off, 5)) {
      // fast path: a one-byte field prefix of a known tag and a 1..4-byte varint after it (the
      // shapes the reference's encoder writes for values < 2^28); same results as below
      uint32_t w, wn;
      rd.win8(pstart + off, w, wn);
      const uint32_t b0 = w & 0xFFu, tag = b0 >> 3;
      const uint32_t x = __builtin_amdgcn_alignbit(wn, w, 8);  // bytes 1..4
      const uint32_t tm = ~x & 0x80808080u;
      if (b0 < 0x80u && tag >= 1u && tag <= 6u && tm) {
        const uint32_t k2 = ((uint32_t)__builtin_ctz(tm) >> 3) + 1u;
        if ((uint64_t)k2 > avail - 1) goto bad;  // the varint runs past the field
        const uint32_t v = ((x & 0x7Fu) | ((x >> 1) & 0x3F80u) | ((x >> 2) & 0x1FC000u) | ((x >> 3) & 0xFE00000u)) &
                           ((1u << (7u * k2)) - 1u);
        if (tag == 3u || tag == 4u || tag == 5u) {
          if (tag == 3u) {
            c.change = v;
            found |= 2;
          } else if (tag == 4u) {
            c.from = v;
            found |= 4;
          } else {
            c.to = v;
            found |= 8;
          }
          off += 1u + k2;
        } else {
          const uint64_t o2 = off + 1u + k2;
          if ((uint64_t)v > len - o2) goto bad;
          if (tag == 1u) {
            c.subset_off = (uint32_t)o2;
            c.subset_len = v;
            c.flags |= DRP_F_SUBSET;
          } else if (tag == 2u) {
            c.key_off = (uint32_t)o2;
            c.key_len = v;
            found |= 1;
          } else {
            c.value_off = (uint32_t)o2;
            c.value_len = v;
            c.flags |= DRP_F_VALUE;
          }
          off = o2 + v;
        }
        continue;
      }
    }
    uint64_t need = avail < 16 ? avail : 16;
    if (!rd.ok(pstart + off, need)) {
      c.err = ERR_UNREACHABLE;
      return c;
    }
    uint64_t w0, w1;
    rd.win(pstart + off, w0, w1);
    uint64_t prefix;
    int k = win_varint(w0, w1, 0, avail, prefix);
    if (k <= 0 || prefix >= JS_SAFE) goto bad;
    {
      int32_t tag = ((int32_t)(uint32_t)prefix) >> 3;
      uint32_t wire = (uint32_t)(prefix & 7);
      uint32_t i = (uint32_t)k;  // window index after the prefix
      uint64_t a2 = avail - (uint64_t)k;
      if (k > 6) {  // a second 10-byte varint would not fit the 16-byte window
        uint64_t need2 = a2 < 16 ? a2 : 16;
        if (!rd.ok(pstart + off + (uint64_t)k, need2)) {
          c.err = ERR_UNREACHABLE;
          return c;
        }
        rd.win(pstart + off + (uint64_t)k, w0, w1);
        i = 0;
      }
      uint64_t v;
      int k2;
      if (tag == 1 || tag == 2 || tag == 6) {
        k2 = win_varint(w0, w1, i, a2, v);
        if (k2 <= 0 || v >= JS_SAFE) goto bad;
        uint64_t o2 = off + (uint64_t)k + (uint64_t)k2;
        if (v > len - o2) goto bad;
        if (tag == 1) {
          c.subset_off = (uint32_t)o2;
          c.subset_len = (uint32_t)v;
          c.flags |= DRP_F_SUBSET;
        } else if (tag == 2) {
          c.key_off = (uint32_t)o2;
          c.key_len = (uint32_t)v;
          found |= 1;
        } else {
          c.value_off = (uint32_t)o2;
          c.value_len = (uint32_t)v;
          c.flags |= DRP_F_VALUE;
        }
        off = o2 + v;
      } else if (tag == 3 || tag == 4 || tag == 5) {
        k2 = win_varint(w0, w1, i, a2, v);
        if (k2 <= 0) goto bad;
        if (tag == 3) {
          c.change = v;
          found |= 2;
        } else if (tag == 4) {
          c.from = v;
          found |= 4;
        } else {
          c.to = v;
          found |= 8;
        }
        off += (uint64_t)k + (uint64_t)k2;
      } else if (wire == 0) {
        k2 = win_varint(w0, w1, i, a2, v);
        if (k2 <= 0) goto bad;
        off += (uint64_t)k + (uint64_t)k2;
      } else if (wire == 1) {
        if (a2 < 8) goto bad;
        off += (uint64_t)k + 8;
      } else if (wire == 2) {
        k2 = win_varint(w0, w1, i, a2, v);
        if (k2 <= 0 || v >= JS_SAFE) goto bad;
        uint64_t o2 = off + (uint64_t)k + (uint64_t)k2;
        if (v > len - o2) goto bad;
        off = o2 + v;
      } else if (wire == 5) {
        if (a2 < 4) goto bad;
        off += (uint64_t)k + 4;
      } else {
        goto bad;
      }
    }
  }
  if (found != 15) {
    c.err = DRP_ERR_REQUIRED;
    c.flags |= DRP_F_BAD;
  }
  return c;
bad:
  c.err = DRP_ERR_CHANGE;
  c.flags |= DRP_F_BAD;
  return c;
}

// decode_change restricted to the shapes encoders write (a one-byte field prefix of a known tag
// and a 1..5-byte varint: every Change field up to 2^35), 32-bit offsets: true with the same
// columns decode_change gives, or false for anything else (the caller then runs decode_change;
// emit_tiles defers such tiles to a second kernel so the general decoder's registers stay out
// of its main one).
template <class R>
__device__ __forceinline__ bool decode_change_fast(const R &rd, uint64_t pstart, uint64_t len, ChangeCols &c) {
  c.key_off = c.key_len = c.subset_off = c.subset_len = c.value_off = c.value_len = 0;
  c.change = c.from = c.to = 0;
  c.flags = 0;
  c.err = 0;
  if (len > 0xFFFFFFFFull) return false;
  const uint32_t n = (uint32_t)len;
  uint32_t found = 0, off = 0;
  while (off < n) {
    const uint32_t avail = n - off;
    if (avail < 2 || !rd.ok(pstart + off, 2)) return false;
    uint32_t w, wn;
    rd.win8(pstart + off, w, wn);
    const uint32_t b0 = w & 0xFFu, tag = b0 >> 3;
    const uint64_t x = ((((uint64_t)wn) << 32) | w) >> 8;  // bytes 1..7
    const uint64_t tm = ~x & 0x8080808080ull;               // terminators among bytes 1..5
    if (b0 >= 0x80u || tag < 1u || tag > 6u || !tm) return false;
    const uint32_t k2 = ((uint32_t)__builtin_ctzll(tm) >> 3) + 1u;
    if (k2 > avail - 1 || !rd.ok(pstart + off, 1 + k2)) return false;
    const uint64_t v = ((x & 0x7Full) | ((x >> 1) & 0x3F80ull) | ((x >> 2) & 0x1FC000ull) | ((x >> 3) & 0xFE00000ull) |
                        ((x >> 4) & 0x7F0000000ull)) &
                       ((1ull << (7u * k2)) - 1ull);
    if (tag == 3u || tag == 4u || tag == 5u) {
      if (tag == 3u) {
        c.change = v;
        found |= 2;
      } else if (tag == 4u) {
        c.from = v;
        found |= 4;
      } else {
        c.to = v;
        found |= 8;
      }
      off += 1u + k2;
    } else {
      const uint32_t o2 = off + 1u + k2;
      if (v > (uint64_t)(n - o2)) return false;
      const uint32_t v32 = (uint32_t)v;
      if (tag == 1u) {
        c.subset_off = o2;
        c.subset_len = v32;
        c.flags |= DRP_F_SUBSET;
      } else if (tag == 2u) {
        c.key_off = o2;
        c.key_len = v32;
        found |= 1;
      } else {
        c.value_off = o2;
        c.value_len = v32;
        c.flags |= DRP_F_VALUE;
      }
      off = o2 + v32;
    }
  }
  if (found != 15) {
    c.err = DRP_ERR_REQUIRED;
    c.flags |= DRP_F_BAD;
  }
  return true;
}

// ---- byte-class bit masks (live-position scan) ------------------------------------
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
// bit k of the result = MSB of byte k of x
__device__ __forceinline__ uint32_t msb4(uint32_t x) {
  return (((x >> 7) & 0x01010101u) * 0x01020408u) >> 24;
}
// MSB of each byte set iff that byte <= 2
__device__ __forceinline__ uint32_t le2(uint32_t x) {
  return ~(((x & 0x7F7F7F7Fu) + 0x7D7D7D7Du) | x) & 0x80808080u;
}
__device__ __forceinline__ void gather16(const uint4 v, uint32_t &m16, uint32_t &s16) {
  m16 = msb4(v.x) | (msb4(v.y) << 4) | (msb4(v.z) << 8) | (msb4(v.w) << 12);
  s16 = msb4(le2(v.x)) | (msb4(le2(v.y)) << 4) | (msb4(le2(v.z)) << 8) | (msb4(le2(v.w)) << 12);
}

// ---- wave helpers -------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t readlane32(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
  uint32_t lo = readlane32((uint32_t)v, l), hi = readlane32((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t uniform32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  uint32_t lo = uniform32((uint32_t)v), hi = uniform32((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t shfl_up32(uint32_t v, uint32_t d) {
  return (uint32_t)__shfl_up((int)v, d, WAVE);
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, uint32_t d) {
  uint32_t lo = shfl_up32((uint32_t)v, d), hi = shfl_up32((uint32_t)(v >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t shfl_xor32(uint32_t v, uint32_t m) {
  return (uint32_t)__shfl_xor((int)v, m, WAVE);
}
// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v) {
  uint32_t lane = lane_id();
#pragma unroll
  for (uint32_t d = 1; d < WAVE; d <<= 1) {
    uint32_t t = shfl_up32(v, d);
    if (lane >= d) v += t;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (uint32_t m = 1; m < WAVE; m <<= 1) {
    uint32_t lo = shfl_xor32((uint32_t)v, m), hi = shfl_xor32((uint32_t)(v >> 32), m);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
  for (uint32_t m = 1; m < WAVE; m <<= 1) v += shfl_xor32(v, m);
  return v;
}

// Agent-scope relaxed atomics on 8-byte granules (the value IS the flag: guide §6 G16 R2).
__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace drp
