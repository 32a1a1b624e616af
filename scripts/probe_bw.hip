// Measurement probe (not product code): HBM rates of the access shapes the C2 emission uses.
//   read16     streaming 16-B-per-lane read of R bytes (sum kept live)
//   write16    streaming 16-B-per-lane write of W bytes
//   cols       100M rows x the 13 output columns (62 B per row), one row per thread, u64/u32/u8 stores
//   cols_rd    the same plus 24 B per row of SoA record reads (the record emission's traffic)
// Build: hipcc -O3 --offload-arch=gfx950 scripts/probe_bw.hip -o /tmp/probe_bw ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void read16(const uint4 *p, uint64_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void write16(uint4 *p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
struct Cols {
  uint64_t *poff; uint32_t *plen; uint8_t *type; uint32_t *ko, *kl, *so, *sl, *vo, *vl; uint64_t *ch, *fr, *to; uint8_t *fl;
  const uint32_t *rec;  // 6 words per row, word-major per 128-row tile (null: no reads)
};
__global__ void cols(Cols c, uint64_t n, uint32_t shift) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x + shift;  // (shift: rows not 64-aligned per wave)
  if (i >= n) return;
  uint32_t w[6] = {(uint32_t)i, 84, 10u | (22u << 16), 7, 8, 9};
  if (c.rec) {
    const uint32_t *r = c.rec + (i / 128) * 768 + (i % 128);
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = r[k * 128];
  }
  c.poff[i] = i * 86 + (w[0] & 0x3FFF);
  c.plen[i] = w[1];
  c.type[i] = 1;
  c.ko[i] = 2;
  c.kl[i] = w[2] & 0xFFFF;
  c.so[i] = 0;
  c.sl[i] = 0;
  c.vo[i] = w[2] >> 16;
  c.vl[i] = w[1] - (w[2] >> 16);
  c.ch[i] = w[3];
  c.fr[i] = w[4];
  c.to[i] = w[5];
  c.fl[i] = 2;
}

int main() {
  const uint64_t R = 8600000000ull, N = 100000000ull;
  void *a;
  CK(hipMalloc(&a, R));
  CK(hipMemset(a, 1, R));
  uint32_t *sink;
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;
  auto timeit = [&](const char *name, double bytes, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("%-10s %8.3f ms  %7.2f TB/s (%.2f GB)\n", name, best, bytes / best / 1e9, bytes / 1e9);
    return 0;
  };
  const uint32_t G = 256 * 64;
  timeit("read16", (double)R, [&] { hipLaunchKernelGGL(read16, dim3(G), dim3(256), 0, 0, (const uint4 *)a, R / 16, sink); });
  timeit("write16", 6.2e9, [&] { hipLaunchKernelGGL(write16, dim3(G), dim3(256), 0, 0, (uint4 *)a, (uint64_t)6200000000ull / 16); });
  // columns: 62 B per row
  uint8_t *cb;
  CK(hipMalloc((void **)&cb, N * 62 + 4096));
  Cols c;
  uint8_t *q = cb;
  auto take = [&](uint64_t bytes) { uint8_t *r = q; q += (bytes + 255) & ~255ull; return r; };
  c.poff = (uint64_t *)take(N * 8); c.plen = (uint32_t *)take(N * 4); c.type = take(N);
  c.ko = (uint32_t *)take(N * 4); c.kl = (uint32_t *)take(N * 4); c.so = (uint32_t *)take(N * 4);
  c.sl = (uint32_t *)take(N * 4); c.vo = (uint32_t *)take(N * 4); c.vl = (uint32_t *)take(N * 4);
  c.ch = (uint64_t *)take(N * 8); c.fr = (uint64_t *)take(N * 8); c.to = (uint64_t *)take(N * 8); c.fl = take(N);
  c.rec = nullptr;
  timeit("cols", N * 62.0, [&] { hipLaunchKernelGGL(cols, dim3((uint32_t)(N / 256)), dim3(256), 0, 0, c, N, 0u); });
  timeit("cols_mis", N * 62.0, [&] { hipLaunchKernelGGL(cols, dim3((uint32_t)(N / 256) - 1), dim3(256), 0, 0, c, N, 37u); });
  c.rec = (const uint32_t *)a;
  timeit("cols_rd", N * 86.0, [&] { hipLaunchKernelGGL(cols, dim3((uint32_t)(N / 256)), dim3(256), 0, 0, c, N, 0u); });
  timeit("cols_rd_mis", N * 86.0, [&] { hipLaunchKernelGGL(cols, dim3((uint32_t)(N / 256) - 1), dim3(256), 0, 0, c, N, 37u); });
  return 0;
}
