// drp_api.hip — the extern "C" boundary of libdrp (include/drp.h).
//
// Owns one HIP stream + scratch per device context and launches the decode / encode
// kernels. A decode is one pass: the kernel resolves every tile's entry exactly
// (DESIGN.md §decode), so there is no host-side repair loop.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <algorithm>
#include <chrono>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../../include/drp.h"
#include "drp_kernels.h"

using drp::DecodeParams;
using drp::EncodeParams;

namespace {

bool trace_on() {
  static int v = -1;
  if (v < 0) v = getenv("DRP_TRACE") ? 1 : 0;
  return v == 1;
}
#define TRACE(...)                                \
  do {                                            \
    if (trace_on()) {                             \
      fprintf(stderr, "[drp] " __VA_ARGS__);      \
      fputc('\n', stderr);                        \
      fflush(stderr);                             \
    }                                             \
  } while (0)

// Hang finding (DRP_WATCHDOG=<seconds>, off by default): the speculative decode's launches record
// named events (drp_dbg_mark), and a host wait that runs past the limit prints which of them have
// completed, then ends the process (a measurement aid: the default path records nothing).
struct DbgMarks {
  int on = -1;
  double limit_s = 0;
  hipEvent_t ev[64] = {};
  const char *name[64] = {};
  int n = 0;
};
DbgMarks g_dbg;
bool dbg_on() {
  if (g_dbg.on < 0) {
    const char *w = getenv("DRP_WATCHDOG");
    g_dbg.limit_s = w ? atof(w) : 0;
    g_dbg.on = g_dbg.limit_s > 0 ? 1 : 0;
    if (g_dbg.on)
      for (auto &e : g_dbg.ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  }
  return g_dbg.on == 1;
}
// a stream synchronisation that, under DRP_WATCHDOG, gives up after the limit and names the
// first marked launch that has not completed
hipError_t sync_watch(hipStream_t st, const char *where) {
  if (!dbg_on()) return hipStreamSynchronize(st);
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e;
  while ((e = hipStreamQuery(st)) == hipErrorNotReady) {
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (s > g_dbg.limit_s) {
      fprintf(stderr, "[drp] watchdog: %s still running after %.1f s; marks:", where, s);
      for (int k = g_dbg.n > 64 ? g_dbg.n - 64 : 0; k < g_dbg.n; k++)  // (a ring of the last 64)
        fprintf(stderr, " %s=%s", g_dbg.name[k % 64], hipEventQuery(g_dbg.ev[k % 64]) == hipSuccess ? "done" : "PENDING");
      fputc('\n', stderr);
      fflush(stderr);
      _exit(3);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  g_dbg.n = 0;
  return e;
}

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  bool ensure(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = n + n / 4 + 4096;
    if (hipMalloc(&p, want) != hipSuccess) {
      p = nullptr;
      (void)hipGetLastError();  // (the failure is reported by the caller, not by a later launch)
      return false;
    }
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *at(size_t off) const {
    return reinterpret_cast<T *>(static_cast<char *>(p) + off);
  }
};

// Page-locked host memory that only grows (the gather buffer of chunked host batches).
struct PinBuf {
  void *p = nullptr;
  size_t cap = 0;
  bool ensure(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = n + n / 4 + 4096;
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      (void)hipGetLastError();
      return false;
    }
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// A host batch: one buffer, or the caller's chunks laid end to end (drp_decode_stage_v).
struct HostSrc {
  const uint8_t *flat = nullptr;
  const drp_chunk *ch = nullptr;
  std::vector<uint64_t> start;  // chunk k's first batch offset (chunks only)
  uint64_t n = 0;
};

bool is_device_ptr(const void *p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// page-locked host memory (the DMA engine reads it directly, without a staging copy)
bool is_pinned_host(const void *p) {
  hipPointerAttribute_t a;
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

double now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

}  // namespace

struct drp_ctx {
  int device = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev[4] = {};
  hipEvent_t hev[2] = {};  // a staged piece's H2D
  // pipelined staging (stage_pieces): the copy stream and one event per chunk (created on first use)
  hipStream_t cst = nullptr;
  hipEvent_t pev[32] = {};
  // their early fetches: a fetch stream, the event behind a piece's last row writes, and a pinned
  // bounce buffer the rows land in before a worker thread copies them into the caller's columns
  hipStream_t fst = nullptr;
  hipEvent_t fev = nullptr;
  PinBuf fbounce;
  uint64_t pipe_chunk = 128ull << 20;  // DRP_PIPE_CHUNK (MiB; 0: no pipelining)
  uint32_t B = 128;
  int strict = 0;
  int exact = 0;  // 1: always the exact kernel (decode_tiles), never the speculative one
  int key_post = 0;  // DRP_KEY_POST_*: key hashes and/or key flags on every decode
  // claims_fast's structural check of long frames: on after a decode whose frames average
  // >= 512 bytes (or none yet); DRP_CHANGE_CHECKS=0/1 forces it (A/B, tests)
  int change_checks = 1, change_checks_env = -1;
  int cus = 256;
  uint32_t waves_per_cu = 16;
  // test / measurement knobs, read once by drp_open (never on a decode): DRP_KSTRONG_HBM weakens
  // predictions, DRP_DIRTY_CAP caps the repair dirty lists, DRP_STATS / DRP_TRACE_FILE collect
  // kernel counters and per-tile traces into dstats (allocated here when asked for)
  uint32_t kstrong_hbm = 0;
  uint32_t cascade_min = 4096;  // DRP_CASCADE_MIN (tests: small cascades)
  int64_t jump_min = -1;        // DRP_JUMP_MIN (-1: max(64, tiles / 512))
  // claims kernel: the region walkers (drp_walk.hip) for batches of at least walk_min tiles,
  // claims_fast below; DRP_CLAIMS=walk / fast forces one (A/B, tests)
  uint64_t walk_min = 32768;
  int claims_mode = 0;  // 0 auto, 2 fast, 3 hop
  int crec = 1;         // claims_fast's per-frame records and the record emission (DRP_CREC=0: off)
  DevBuf recbuf;
  uint64_t dirty_cap = ~0ull;
  bool stats = false;
  const char *trace_file = nullptr;
  unsigned long long *dstats = nullptr;
  uint32_t *ctile = nullptr;  // segmented repair: per-tile candidate positions (grown on demand)
  uint64_t ctile_cap = 0;
  DevBuf scratch, in_stage, out_stage, aux;
  PinBuf gather;  // chunked host batches: the staged ranges, gathered (drp_decode_stage_v)
  DevBuf dec_cols;  // device columns of the staged host-batch decode (drp_decode_stage)
  DevBuf fetch_tmp; // drp_decode_fetch_block: the caller's block layout, packed on the device
  DevBuf keybuf;    // drp_decode_fetch_keys: per-row key lengths and positions
  DevBuf keytext;   // drp_decode_fetch_keys: the key text
  double frames_per_byte = 0;  // density of the last staged batch (sizes the next one's columns)
  int blob_skip = DRP_BLOB_SKIP_AUTO;
  bool blob_heavy = false;     // the last host batch was mostly blob payload (AUTO: stage in pieces)
  uint64_t blob_run = 0;       // bytes from a piece's start to its blob's payload, last seen
  uint64_t piece_span = 0;     // batch bytes one blob-skipping piece covered on average, last seen
  drp_timing timing = {};
  // drp_decode_batch's host columns while it stages (pipelined pieces fetch their rows into them
  // during the copy; dfetched: rows already there)
  const drp_frames *dfr = nullptr;
  const drp_changes *dco = nullptr;
  uint64_t dcap = 0, dfetched = 0;
  std::vector<uint64_t> host_tmp;
  // the staged host-batch decode: row 0 is a host-built blob continuation when nf0 == 1; GPU
  // rows follow, each piece's payload_off relative to the batch offset where that piece was
  // staged (pieces: {first GPU row, batch offset}; one piece unless blobs were skipped)
  struct Staged {
    uint64_t rows = 0, nf0 = 0, cap = 0;
    std::vector<std::pair<uint64_t, uint64_t>> pieces;
    const uint8_t *dev = nullptr;  // the last piece's bytes on the device (a one-piece batch: all of it)
    uint64_t off0 = 0;
    uint32_t len0 = 0;
    uint8_t ty0 = 0;
    drp_frames fr = {};
    drp_changes co = {};
  } staged;
};

#define CHK(x)                                                                     \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      if (getenv("DRP_DEBUG")) fprintf(stderr, "drp: %s -> %s\n", #x, hipGetErrorString(e_)); \
      return DRP_E_HIP;                                                            \
    }                                                                              \
  } while (0)

extern "C" {

int drp_abi_version(void) { return DRP_ABI_VERSION; }

int drp_device_count(int *n) {
  if (!n) return DRP_E_INVAL;
  *n = 0;
  int k = 0;
  if (hipGetDeviceCount(&k) != hipSuccess) {
    (void)hipGetLastError();
    return DRP_OK;  // no runtime / no device: zero devices
  }
  *n = k;
  return DRP_OK;
}

int drp_open(int device, drp_ctx **out) {
  if (!out) return DRP_E_INVAL;
  *out = nullptr;
  int n = 0;
  const hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= device || device < 0) {
    if (getenv("DRP_DEBUG"))
      fprintf(stderr, "drp_open(%d): hipGetDeviceCount -> %s, %d devices\n", device, hipGetErrorString(e), n);
    return DRP_E_NODEV;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return DRP_E_NODEV;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return DRP_E_NODEV;
  drp_ctx *c = new drp_ctx();
  c->device = device;
  c->cus = prop.multiProcessorCount;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return DRP_E_HIP;
  }
  for (auto &e : c->ev) (void)hipEventCreate(&e);
  for (auto &e : c->hev) (void)hipEventCreate(&e);
  if (hipStreamCreateWithFlags(&c->cst, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->fst, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->fev, hipEventDisableTiming) != hipSuccess) {
    if (c->cst) (void)hipStreamDestroy(c->cst);
    if (c->fst) (void)hipStreamDestroy(c->fst);
    (void)hipStreamDestroy(c->st);
    delete c;
    return DRP_E_HIP;
  }
  if (const char *t = getenv("DRP_TILE")) {
    uint32_t tb = (uint32_t)atoi(t);
    if (tb == 4096 || tb == 8192) c->B = tb / 64;
  }
  if (const char *d = getenv("DRP_DECODE")) c->exact = strcmp(d, "exact") == 0;
  if (const char *d = getenv("DRP_CHANGE_CHECKS")) c->change_checks = c->change_checks_env = atoi(d) ? 1 : 0;
  if (const char *w = getenv("DRP_WAVES_PER_CU")) {
    int v = atoi(w);
    if (v > 0 && v <= 32) c->waves_per_cu = (uint32_t)v;
  }
  if (const char *e = getenv("DRP_KSTRONG_HBM")) c->kstrong_hbm = (uint32_t)atoi(e);
  if (const char *e = getenv("DRP_CASCADE_MIN")) c->cascade_min = (uint32_t)strtoul(e, nullptr, 10);
  if (const char *e = getenv("DRP_JUMP_MIN")) c->jump_min = strtoll(e, nullptr, 10);
  if (const char *e = getenv("DRP_WALK_MIN")) c->walk_min = strtoull(e, nullptr, 10);
  if (const char *e = getenv("DRP_PIPE_CHUNK")) c->pipe_chunk = strtoull(e, nullptr, 10) << 20;
  if (const char *e = getenv("DRP_CREC")) c->crec = atoi(e);
  if (const char *e = getenv("DRP_CLAIMS")) c->claims_mode = strcmp(e, "fast") == 0 ? 2 : strcmp(e, "hop") == 0 ? 3 : 0;
  if (const char *e = getenv("DRP_DIRTY_CAP")) c->dirty_cap = strtoull(e, nullptr, 10);
  c->trace_file = getenv("DRP_TRACE_FILE");
  if (getenv("DRP_STATS") && hipMalloc((void **)&c->dstats, 64 * 8) == hipSuccess) c->stats = true;
  *out = c;
  return DRP_OK;
}

void drp_close(drp_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->st);
  c->scratch.release();
  c->in_stage.release();
  c->gather.release();
  c->out_stage.release();
  c->aux.release();
  c->dec_cols.release();
  c->recbuf.release();
  c->fetch_tmp.release();
  c->keybuf.release();
  c->keytext.release();
  if (c->dstats) (void)hipFree(c->dstats);
  if (c->ctile) (void)hipFree(c->ctile);
  for (auto &e : c->ev) (void)hipEventDestroy(e);
  for (auto &e : c->hev) (void)hipEventDestroy(e);
  for (auto &e : c->pev)
    if (e) (void)hipEventDestroy(e);
  (void)hipStreamSynchronize(c->cst);
  (void)hipStreamDestroy(c->cst);
  (void)hipStreamSynchronize(c->fst);
  (void)hipStreamDestroy(c->fst);
  (void)hipEventDestroy(c->fev);
  c->fbounce.release();
  (void)hipStreamDestroy(c->st);
  delete c;
}

void *drp_stream(drp_ctx *c) { return c ? (void *)c->st : nullptr; }

int drp_device(drp_ctx *c) { return c ? c->device : DRP_E_INVAL; }

int drp_synchronize(drp_ctx *c) {
  if (!c) return DRP_E_INVAL;
  CHK(hipStreamSynchronize(c->st));
  return DRP_OK;
}

int drp_last_timing(drp_ctx *c, drp_timing *out) {
  if (!c || !out) return DRP_E_INVAL;
  *out = c->timing;
  return DRP_OK;
}

int drp_set_tile(drp_ctx *c, uint32_t tile_bytes) {
  if (!c) return DRP_E_INVAL;
  if (tile_bytes == 0) tile_bytes = 8192;
  if (tile_bytes != 4096 && tile_bytes != 8192) return DRP_E_INVAL;
  c->B = tile_bytes / 64;
  return DRP_OK;
}

int drp_set_exact(drp_ctx *c, int exact) {
  if (!c) return DRP_E_INVAL;
  c->exact = exact ? 1 : 0;
  return DRP_OK;
}

int drp_set_key_post(drp_ctx *c, int mode) {
  if (!c || mode < DRP_KEY_POST_OFF || mode > DRP_KEY_POST_FLAGS) return DRP_E_INVAL;
  c->key_post = mode;
  return DRP_OK;
}

int drp_set_strict(drp_ctx *c, int strict) {
  if (!c) return DRP_E_INVAL;
  c->strict = strict ? 1 : 0;
  return DRP_OK;
}

int drp_set_blob_skip(drp_ctx *c, int mode) {
  if (!c || mode < DRP_BLOB_SKIP_OFF || mode > DRP_BLOB_SKIP_ALWAYS) return DRP_E_INVAL;
  c->blob_skip = mode;
  return DRP_OK;
}

// scratch layout for a decode of `nbytes` over `ns` streams
struct DecLayout {
  uint64_t ntiles_max;
  size_t tile_prefix, rec, sgrp, tiles, perr, scount, ctrl, tstream, ent, tk, tsp, fmiss, segw, scan_tmp, walk, went, wdense, trec, trok, total;
  uint64_t nsg;
};
static DecLayout dec_layout(uint32_t B, uint64_t nbytes, uint64_t ns) {
  DecLayout L;
  const uint64_t tile = 64ull * B;
  L.ntiles_max = nbytes / tile + 2 * ns + 2;
  size_t o = 0;
  L.tile_prefix = o; o += al((ns + 1) * 8);
  L.rec = o; o += al(6 * L.ntiles_max * 8);    // ywd, aggv, aggn, inclx, aggc, inclc (zeroed per call)
  L.nsg = L.ntiles_max / 64 + 2;
  L.sgrp = o; o += al(L.nsg * 32);             // sgc_agg+sgc_cnt (u32 x2), sagg, saggn, scnt (zeroed)
  L.tiles = o; o += al(5 * L.ntiles_max * 8);  // exit, base, count, changes, changes prefix
  L.perr = o; o += al(ns * 8);
  L.scount = o; o += al(2 * ns * 8);
  L.ctrl = o; o += 256;
  L.tstream = o; o += al(L.ntiles_max * 4);    // tile -> stream (speculative kernel)
  L.ent = o; o += al(L.ntiles_max * 128 * 3);  // per-thread entries + counts (speculative kernel)
  L.tk = o; o += al(L.ntiles_max);             // first entry thread per tile (verify_lite)
  L.tsp = o; o += al(L.ntiles_max);            // sparse-tile marks (verify_lite -> emit_sparse)
  L.fmiss = o; o += al(ns * 8);                  // first missed tile per stream (verify)
  L.segw = o; o += al((2 * 64 * 8192 + 8194) * 8 + 65 * 8192);  // segmented repair: candidates, entries,
                                                                // next-candidate tables, lanes (SEG_NMAX)
  L.scan_tmp = o; o += al((L.ntiles_max / 4096 + 2) * 8);  // tile scans: block sums
  L.walk = o; o += al((ns + 2) * 8);                         // region walkers: per-stream region prefix
  L.went = o; o += al((L.ntiles_max + ns + 2) * 8);          // region walkers: entries
  L.wdense = o; o += 64;                                     // region walkers: density sample
  L.trec = o; o += al(L.ntiles_max * 4);                     // first record per tile (region walkers)
  L.trok = o; o += al(L.ntiles_max);                         // record emission marks (verify_lite)
  L.total = o;
  return L;
}

int drp_host_alloc(uint64_t bytes, void **out) {
  if (!out || !bytes) return DRP_E_INVAL;
  *out = nullptr;
  if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return DRP_E_NOMEM;
  }
  return DRP_OK;
}

void drp_host_free(void *p) {
  if (p) (void)hipHostFree(p);
}

uint64_t drp_decode_scratch_bytes(drp_ctx *c, uint64_t n, uint64_t nstreams) {
  return dec_layout(c ? c->B : 128, n, nstreams).total;
}

}  // extern "C"

namespace {

constexpr int kWaitExpired = -100;  // internal: a bounded look-back spin gave up (retryable)

int run_decode_exact_once(drp_ctx *c, const uint8_t *bytes, uint64_t nbytes, const uint64_t *stream_off,
                          const uint64_t *entry, uint64_t ns, const drp_frames *fr, const drp_changes *co,
                          uint64_t cap, drp_stream_result *res) {
  if (ns == 0) return DRP_OK;
  if (((uintptr_t)bytes & 15) != 0) return DRP_E_INVAL;
  const DecLayout L = dec_layout(c->B, nbytes, ns);
  if (!c->scratch.ensure(L.total)) return DRP_E_NOMEM;
  const uint64_t NT = L.ntiles_max;
  uint64_t *tile_prefix = c->scratch.at<uint64_t>(L.tile_prefix);
  uint64_t *rec = c->scratch.at<uint64_t>(L.rec);
  uint64_t *tiles = c->scratch.at<uint64_t>(L.tiles);
  uint64_t *perr = c->scratch.at<uint64_t>(L.perr);
  uint64_t *scount = c->scratch.at<uint64_t>(L.scount);
  uint32_t *ctrl = c->scratch.at<uint32_t>(L.ctrl);  // [0] tile counter [1] overflow flags

  hipStream_t st = c->st;
  CHK(hipEventRecord(c->ev[0], st));
  CHK(hipMemsetAsync(rec, 0, 6 * NT * 8, st));
  uint8_t *sgrp = c->scratch.at<uint8_t>(L.sgrp);
  CHK(hipMemsetAsync(sgrp, 0, L.nsg * 32, st));
  CHK(hipMemsetAsync(perr, 0xFF, ns * 8, st));
  CHK(hipMemsetAsync(scount, 0, 2 * ns * 8, st));
  CHK(hipMemsetAsync(ctrl, 0, 16, st));
  CHK(drp_launch_tile_prefix(c->B, stream_off, ns, tile_prefix, st));

  DecodeParams P;
  memset(&P, 0, sizeof(P));
  P.bytes = bytes;
  P.nbytes = nbytes;
  P.stream_off = stream_off;
  P.entry = entry;
  P.nstreams = ns;
  P.tile_prefix = tile_prefix;
  P.payload_off = fr->payload_off;
  P.payload_len = fr->payload_len;
  P.type = fr->type;
  P.key_off = co->key_off;
  P.key_len = co->key_len;
  P.subset_off = co->subset_off;
  P.subset_len = co->subset_len;
  P.value_off = co->value_off;
  P.value_len = co->value_len;
  P.change = co->change;
  P.from = co->from;
  P.to = co->to;
  P.flags = co->flags;
  P.cap = cap;
  P.ywd = rec;
  P.aggv = rec + NT;
  P.inclx = rec + 2 * NT;
  P.aggc = rec + 3 * NT;
  P.inclc = rec + 4 * NT;
  P.aggn = rec + 5 * NT;
  P.sgc_agg = reinterpret_cast<uint32_t *>(sgrp);
  P.sgc_cnt = P.sgc_agg + L.nsg;
  P.sagg = reinterpret_cast<uint64_t *>(sgrp + L.nsg * 8);
  P.saggn = P.sagg + L.nsg;
  P.scnt = P.saggn + L.nsg;
  P.tile_exit = tiles;
  P.tile_base = tiles + NT;
  P.tile_count = tiles + 2 * NT;
  P.payload_err = perr;
  P.scount = scount;
  P.counter = ctrl;
  P.overflow = ctrl + 1;
  P.strict = (uint32_t)c->strict;
  unsigned long long *dstats = c->stats ? c->dstats : nullptr;
  if (dstats) {
    CHK(hipMemsetAsync(dstats, 0, 64 * 8, st));
    P.stats = dstats;
  }
  unsigned long long *dtrace = nullptr;
  if (dstats && c->trace_file) {
    CHK(hipMalloc((void **)&dtrace, NT * 64));
    CHK(hipMemsetAsync(dtrace, 0, NT * 64, st));
    P.trace = dtrace;
  }

  // persistent grid: single-wave blocks, several per CU; tiles are handed out in stream
  // order by an atomic counter, so a tile only ever waits on tiles already taken.
  const uint32_t tile = 64u * c->B;
  const uint32_t wpg = drp_decode_waves_per_group();
  const uint64_t groups_needed = (nbytes / tile + ns + 1 + wpg - 1) / wpg;
  uint32_t grid = (uint32_t)(c->cus * ((c->waves_per_cu + wpg - 1) / wpg));
  if (groups_needed < grid) grid = (uint32_t)groups_needed;
  if (grid == 0) grid = 1;
  TRACE("decode: nbytes=%llu ns=%llu B=%u grid=%u NT=%llu", (unsigned long long)nbytes,
        (unsigned long long)ns, c->B, grid, (unsigned long long)NT);
  CHK(hipEventRecord(c->ev[1], st));
  P.tile_nch = tiles + 3 * NT;
  P.tile_nch_base = tiles + 4 * NT;
  CHK(drp_launch_decode(c->B, &P, grid, st));
  CHK(drp_launch_tile_scan(P.tile_nch, tile_prefix, ns, NT, c->scratch.at<uint64_t>(L.scan_tmp), P.tile_nch_base,
                           ~0ull, P.overflow, st));
  CHK(drp_launch_stream_counts(tile_prefix, ns, P.tile_count, P.tile_base, P.tile_nch, P.tile_nch_base, scount, st));
  CHK(hipEventRecord(c->ev[2], st));
  CHK(drp_launch_finalize(bytes, stream_off, ns, tile_prefix, P.tile_exit, P.tile_base, P.tile_count, perr,
                          scount, fr->type, co->flags, cap, res, nullptr, 0, st));
  CHK(drp_launch_key_post(bytes, tile_prefix, ns, P.tile_base, P.tile_count, cap, fr, co,
                          c->key_post == DRP_KEY_POST_FLAGS, nullptr, 0, st));
  CHK(hipEventRecord(c->ev[3], st));
  uint32_t h[2];
  CHK(hipMemcpyAsync(h, ctrl, 8, hipMemcpyDeviceToHost, st));
  CHK(hipStreamSynchronize(st));
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[1], c->ev[2]);
  c->timing.decode_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[3]);
  c->timing.total_ms = ms;
  c->timing.finalize_ms = 0;
  c->timing.spec_repairs = 0;
  c->timing.strict_reruns = 0;
  c->timing.verify_relisted = 0;
  c->timing.seg_repairs = 0;
  TRACE("decode done: tiles=%u flags=%u", h[0], h[1]);
  if (dstats) {
    unsigned long long hs[40];
    CHK(hipMemcpy(hs, dstats, sizeof(hs), hipMemcpyDeviceToHost));
    static const char *nm[] = {"lb_iters", "lb_noincl", "lb_noagg", "lb_keymiss", "lb_vunk", "lb_ok0", "lb_okn",
                               "y_spins", "serial", "cnt_spins", "y_count", "agg_unk", "tiles", "pass", "ovf_pos",
                               "t_grab", "t_stage", "t_dp", "t_y", "t_lb", "t_path", "t_cnt", "t_emit",
                               "ev_tiles", "ev_sg", "skips", "phaseA", "rt_cyc", "drain_cyc", "dp_live", "dp_trips",
                               "t_dploop", "emit_frames", "emit_trips", "t_dpparse"};
    fprintf(stderr, "[drp-stats]");
    for (int i = 0; i < 35; i++) fprintf(stderr, " %s=%llu", nm[i], hs[i]);
    fprintf(stderr, " decode_ms=%.3f\n", c->timing.decode_ms);
  }
  if (dtrace) {
    std::vector<unsigned long long> ht(NT * 8);
    CHK(hipMemcpy(ht.data(), dtrace, NT * 64, hipMemcpyDeviceToHost));
    if (FILE *f = fopen(c->trace_file, "wb")) {
      fwrite(ht.data(), 8, ht.size(), f);
      fclose(f);
    }
    (void)hipFree(dtrace);
  }
  if (h[1] & ~1u) return kWaitExpired;  // bounded wait expired / inconsistent walk inside the kernel
  if (h[1]) return DRP_E_CAPACITY;
  return DRP_OK;
}

// A bounded spin that expires (a preempted or slow predecessor wave) is not an input error:
// the kernel's scratch is reset on entry, so the call is re-run once before reporting it.
int run_decode_exact(drp_ctx *c, const uint8_t *bytes, uint64_t nbytes, const uint64_t *stream_off,
                     const uint64_t *entry, uint64_t ns, const drp_frames *fr, const drp_changes *co,
                     uint64_t cap, drp_stream_result *res) {
  int r = run_decode_exact_once(c, bytes, nbytes, stream_off, entry, ns, fr, co, cap, res);
  uint32_t retries = 0;
  if (r == kWaitExpired) {
    const float ms = c->timing.decode_ms, tot = c->timing.total_ms;
    TRACE("decode_exact: bounded wait expired, re-running once");
    r = run_decode_exact_once(c, bytes, nbytes, stream_off, entry, ns, fr, co, cap, res);
    c->timing.decode_ms += ms;
    c->timing.total_ms += tot;
    retries = 1;
  }
  c->timing.exact_retries = retries;
  return r == kWaitExpired ? DRP_E_HIP : r;
}

// The default decode: speculate-and-verify kernel (drp_decode_spec.hip). Returns DRP_E_RETRY
// when a prediction failed (or a bounded wait expired): the caller then runs the exact kernel.
constexpr int kSpecRepairPasses = 16;
constexpr int kChain = 3;  // dirty-list repair passes queued per host read
constexpr int kSegRepairAfter = 3;  // verify passes before the segmented repair of the streams still missing

// A repair pass's clears in one launch (six fills cost ~50 us of launch gaps per pass): the entry
// words, the flag word, the first-miss words, the verify list's count and this pass's dirty-list
// count and overflow word.
__global__ __launch_bounds__(256) void pass_clear_kernel(uint64_t *incl_e, uint64_t nt, uint64_t *first_miss,
                                                         uint64_t ns, uint32_t *overflow, uint32_t *vlist_n,
                                                         uint32_t *dl_n, uint32_t *dl_ovf) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u, i0 = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  for (uint64_t i = i0; i < nt; i += stride) incl_e[i] = 0;
  for (uint64_t i = i0; i < ns; i += stride) first_miss[i] = ~0ull;
  if (i0 == 0) {
    *overflow = 0;
    *vlist_n = 0;
    *dl_n = 0;
    *dl_ovf = 0;
  }
}

int run_decode_spec(drp_ctx *c, const uint8_t *bytes, uint64_t nbytes, const uint64_t *stream_off,
                    const uint64_t *entry, uint64_t ns, const drp_frames *fr, const drp_changes *co,
                    uint64_t cap, drp_stream_result *res) {
  if (((uintptr_t)bytes & 15) != 0) return DRP_E_INVAL;
  const uint32_t B = drp_spec_tile_bytes() / 64;
  const DecLayout L = dec_layout(B, nbytes, ns);
  if (!c->scratch.ensure(L.total)) return DRP_E_NOMEM;
  const uint64_t NT = L.ntiles_max;
  uint64_t *tile_prefix = c->scratch.at<uint64_t>(L.tile_prefix);
  uint64_t *rec = c->scratch.at<uint64_t>(L.rec);
  uint64_t *tiles = c->scratch.at<uint64_t>(L.tiles);
  uint64_t *perr = c->scratch.at<uint64_t>(L.perr);
  uint64_t *scount = c->scratch.at<uint64_t>(L.scount);
  uint32_t *ctrl = c->scratch.at<uint32_t>(L.ctrl);
  uint32_t *tstream = c->scratch.at<uint32_t>(L.tstream);
  uint64_t *sgscan = c->scratch.at<uint64_t>(L.scan_tmp);
  hipStream_t st = c->st;
  CHK(hipEventRecord(c->ev[0], st));
  DecodeParams P;
  memset(&P, 0, sizeof(P));
  P.bytes = bytes;
  P.nbytes = nbytes;
  P.stream_off = stream_off;
  P.entry = entry;
  P.nstreams = ns;
  P.tile_prefix = tile_prefix;
  P.payload_off = fr->payload_off;
  P.payload_len = fr->payload_len;
  P.type = fr->type;
  P.key_off = co->key_off;
  P.key_len = co->key_len;
  P.subset_off = co->subset_off;
  P.subset_len = co->subset_len;
  P.value_off = co->value_off;
  P.value_len = co->value_len;
  P.change = co->change;
  P.from = co->from;
  P.to = co->to;
  P.flags = co->flags;
  P.cap = cap;
  P.claim = rec;
  P.incl_e = rec + NT;
  P.work = reinterpret_cast<uint32_t *>(rec + 2 * NT);
  P.work_n = ctrl + 2;
  P.tile_exit = tiles;
  P.tile_base = tiles + NT;
  P.tile_count = tiles + 2 * NT;
  P.payload_err = perr;
  P.scount = scount;
  P.counter = ctrl;
  P.overflow = ctrl + 1;
  P.ent = c->scratch.at<uint8_t>(L.ent);
  P.ent_n = P.ent + NT * 128;
  P.ent_c = P.ent_n + NT * 128;
  P.tile_nch = tiles + 3 * NT;
  P.tile_nch_base = tiles + 4 * NT;
  P.vlist = reinterpret_cast<uint32_t *>(rec + 2 * NT) + NT;  // (after the dense work list)
  P.vlist_n = ctrl + 5;
  P.tile_k = c->scratch.at<uint8_t>(L.tk);
  P.tile_sparse = c->scratch.at<uint8_t>(L.tsp);
  P.first_miss = c->scratch.at<uint64_t>(L.fmiss);
  // dirty lists (ping-pong, after the work list and vlist in rec): the tiles each verify pass's
  // repairs handed to the next pass; counts at ctrl[8 + k], overflow words at ctrl[10 + k]
  uint32_t *dl[2] = {reinterpret_cast<uint32_t *>(rec + 3 * NT), reinterpret_cast<uint32_t *>(rec + 3 * NT) + NT};
  P.dlist = dl[0];
  P.dlist_n = ctrl + 8;
  P.dlist_cap = NT;
  P.dstamp = reinterpret_cast<uint32_t *>(rec + 4 * NT);  // (after the dirty lists)
  P.pass_id = 1;
  P.change_checks = (uint32_t)c->change_checks;
  P.kstrong_hbm = c->kstrong_hbm;  // (tests: weaker predictions)
  P.cascade_min = c->cascade_min;
  P.jump_min = c->jump_min >= 0 ? (uint32_t)c->jump_min : (uint32_t)std::max<uint64_t>(64, NT / 512);
  P.dlist_cap = std::min<uint64_t>(NT, c->dirty_cap);  // (tests: DRP_DIRTY_CAP)
  if (c->claims_mode == 3 || (c->claims_mode == 0 && NT >= c->walk_min)) {
    P.walk_rp = c->scratch.at<uint64_t>(L.walk);
    P.walk_entry = c->scratch.at<uint64_t>(L.went);
    P.walk_dense = c->scratch.at<unsigned long long>(L.wdense);
    P.walk_hop = c->claims_mode == 3 ? 1u : 2u;  // 2: by the density sample
    P.walk_tpr = drp_walk_tiles_per_region(NT, (int)P.walk_hop);
  }
  // claims_fast's per-frame records (fast_records, 24 B per frame slot): emit_lean expands them into
  // columns without reading the wire again (DRP_CREC=0: off; a buffer that cannot be had: off)
  const uint64_t rec_bytes = (NT * drp_spec_rec_words() * 4ull + 255) & ~255ull;
  if (c->crec && c->recbuf.ensure(rec_bytes + (cap / 64 + 2) * 4)) {
    P.rec = c->recbuf.at<uint32_t>(0);
    P.chunk_tile = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(c->recbuf.p) + rec_bytes);
    P.tile_rec = c->scratch.at<uint32_t>(L.trec);
    P.tile_recok = c->scratch.at<uint8_t>(L.trok);
  }
  unsigned long long *dstats = c->stats ? c->dstats : nullptr;
  if (dstats) P.stats = dstats;
  {  // tile_prefix and every per-decode clear in one launch
    ClearSet cs = {};
    hipError_t ce = hipSuccess;
    auto add = [&](void *p, uint64_t bytes, uint32_t v) {
      if (cs.n == ClearSet::CAP) {  // (not reached: CAP covers every fill of a decode)
        if (ce == hipSuccess) ce = hipMemsetAsync(p, (int)(v & 0xFF), bytes, st);
        return;
      }
      cs.ptr[cs.n] = p;
      cs.bytes[cs.n] = bytes;
      cs.value[cs.n++] = v;
    };
    add(rec + NT, NT * 8, 0);  // incl_e (every claim is written by the claims kernels)
    add(perr, ns * 8, 0xFF);
    add(scount, 2 * ns * 8, 0);
    add(ctrl, 64, 0);
    add(P.dstamp, NT * 4, 0);
    add(P.first_miss, ns * 8, 0xFF);
    if (P.tile_rec) add(P.tile_rec, NT * 4, 0xFF);
    if (P.walk_dense) add(P.walk_dense, 16, 0);
    if (dstats) add(dstats, 64 * 8, 0);
    CHK(ce);
    CHK(drp_launch_prologue(B, stream_off, ns, tile_prefix, &cs, st));
  }
  c->timing.seg_repairs = 0;
  CHK(hipEventRecord(c->ev[1], st));
  // claims + verification, then the prediction check on the host (one flag word) before any
  // output is written: a failed prediction is repaired in place first. Verify patched the
  // missed tiles' claims, so verify runs again (each pass fixes at least the first missed tile,
  // whose entry is exact) until a pass has no miss. Only when that does not settle within a
  // few passes (e.g. a protocol error on the exact chain) does the caller run the exact kernel.
  uint32_t h[16];
  const uint32_t miss = drp_spec_miss_bit();
  CHK(drp_launch_spec_head(&P, NT, ns, tstream, st));  // (verify_counts keeps the relisted count in ctrl[14])
  // Emission, the output bases and the per-stream results go right behind verification, with no
  // host read in between: the emit, finalize and key kernels read the flag word and do nothing
  // after a failed prediction, which is repaired below before they run again. A decode whose
  // prediction holds makes one host round trip.
  const uint32_t *abort_flag = P.overflow;
  auto launch_tail = [&]() -> int {
    CHK(drp_launch_spec_tail(&P, NT, ns, tstream, sgscan, st));
    CHK(hipEventRecord(c->ev[2], st));
    CHK(drp_launch_finalize(bytes, stream_off, ns, tile_prefix, P.tile_exit, P.tile_base, P.tile_count, perr,
                            scount, fr->type, co->flags, cap, res, abort_flag, drp_spec_retry_mask(), st));
    CHK(drp_launch_key_post(bytes, tile_prefix, ns, P.tile_base, P.tile_count, cap, fr, co,
                            c->key_post == DRP_KEY_POST_FLAGS, abort_flag, drp_spec_retry_mask(), st));
    CHK(hipEventRecord(c->ev[3], st));
    CHK(hipMemcpyAsync(h, ctrl, 64, hipMemcpyDeviceToHost, st));
    CHK(sync_watch(st, "decode (claims .. key_post)"));
    return DRP_OK;
  };
  if (const int rt = launch_tail()) return rt;
  const uint32_t relisted = h[14];
  int pass = 0;
  bool seg_done = false;
  if ((h[1] & drp_spec_retry_mask()) == miss) {
    // the next pass verifies the dirty list the last one wrote (k: its index), or every tile
    uint32_t k = 0;
    bool full = h[10] != 0 || h[8] > P.dlist_cap;
    for (; pass < kSpecRepairPasses && (h[1] & miss); pass++) {
      // a dirty list this long after a repair pass is a cascade already (C5's first list is ~300
      // tiles). Not after the head's pass: independent misses (C3: a blob tile whose random bytes
      // held a far candidate that landed on the next unit's chain, ~1.5% of the blob tiles) each
      // list the identity tiles behind them, and one repair pass fixes them all; taken for a
      // cascade, they cost a segmented repair (~100 ms per 0.34 GB)
      const uint64_t seg_early = std::max<uint64_t>(1024, NT / 256);
      if ((pass >= kSegRepairAfter || (pass > 0 && h[8 + k] > seg_early) || (h[1] & drp_spec_cascade_bit())) &&
          !seg_done) {
        // the misses keep coming one tile per pass (wrong predictions that agree with each
        // other): recompute the claims of each stream from its first missed tile by exact
        // chain walks (drp_decode_spec.hip, segmented repair), then verify them
        seg_done = true;
        std::vector<uint64_t> fm(ns), tp(ns + 1);
        CHK(hipMemcpyAsync(fm.data(), P.first_miss, ns * 8, hipMemcpyDeviceToHost, st));
        CHK(hipMemcpyAsync(tp.data(), tile_prefix, (ns + 1) * 8, hipMemcpyDeviceToHost, st));
        CHK(hipStreamSynchronize(st));
        for (uint64_t s = 0; s < ns; s++)
          if (fm[s] != ~0ull) {
            TRACE("decode_spec: segmented repair of stream %llu from tile %llu to %llu", (unsigned long long)s,
                  (unsigned long long)fm[s], (unsigned long long)tp[s + 1]);
            // the parallel seg_claims' per-tile candidate positions (256 B per tile of the range),
            // allocated on the first segmented repair that needs more
            const uint64_t need = std::min<uint64_t>(tp[s + 1] - fm[s], 8192ull * 1024) * 64;
            if (need > c->ctile_cap) {
              if (c->ctile) (void)hipFree(c->ctile);
              c->ctile = nullptr;
              c->ctile_cap = 0;
              if (hipMalloc((void **)&c->ctile, need * 4) == hipSuccess) c->ctile_cap = need;
              else (void)hipGetLastError();
            }
            CHK(drp_launch_seg_repair(&P, s, fm[s], tp[s + 1], c->scratch.at<uint64_t>(L.segw), c->ctile, c->ctile_cap,
                                      st));
            c->timing.seg_repairs++;
            full = true;  // (claims rewritten over a range)
          }
      }
      // a full pass alone; dirty-list passes kChain at a time with one host read at the end
      // (a pass whose input list is empty launches nothing but the memsets)
      const int chain = full ? 1 : std::min(kChain, kSpecRepairPasses - pass);
      for (int cp = 0; cp < chain; cp++) {
        const uint32_t kn = k ^ 1u;  // this pass's dirty list
        const uint32_t cg = (uint32_t)std::min<uint64_t>(1024, (std::max<uint64_t>(NT, ns) + 255) / 256);
        hipLaunchKernelGGL(pass_clear_kernel, dim3(cg), dim3(256), 0, st, P.incl_e, NT, P.first_miss, ns, P.overflow,
                           P.vlist_n, ctrl + 8 + kn, ctrl + 10 + kn);
        CHK(hipGetLastError());
        DecodeParams V = P;
        V.dlist = dl[kn];
        V.dlist_n = ctrl + 8 + kn;
        V.pass_id = (uint32_t)(pass + cp + 2);
        if (full) {
          CHK(drp_launch_spec_verify(&V, NT, ns, tstream, st));
        } else {
          V.vlist = dl[k];
          V.vlist_n = ctrl + 8 + k;
          V.vlist_ovf = ctrl + 10 + k;
          CHK(drp_launch_spec_verify_list(&V, cp == 0 ? h[8 + k] : ~0ull, ns, tstream, st));
        }
        k = kn;
      }
      CHK(hipMemcpyAsync(h, ctrl, 64, hipMemcpyDeviceToHost, st));
      CHK(sync_watch(st, "repair passes"));
      TRACE("decode_spec: passes %d-%d over %s, %u listed next", pass + 1, pass + chain,
            full ? "every tile" : "dirty lists", h[8 + k]);
      pass += chain - 1;
      full = h[10 + k] != 0 || h[8 + k] > P.dlist_cap;
      if (trace_on()) {
        uint64_t f0 = 0;
        CHK(hipMemcpy(&f0, P.first_miss, 8, hipMemcpyDeviceToHost));
        TRACE("decode_spec: pass %d flags=%#x first miss (stream 0) %lld", pass + 1, h[1], (long long)f0);
      }
    }
    TRACE("decode_spec: %d repair pass(es), flags=%#x", pass, h[1]);
    if (!(h[1] & drp_spec_retry_mask()))  // repaired: emission and results again
      if (const int rt = launch_tail()) return rt;
  }
  const bool retry = (h[1] & drp_spec_retry_mask()) != 0;
  if (retry && pass) {  // (the timings then cover the repair passes too, not just the first tail)
    CHK(hipEventRecord(c->ev[2], st));
    CHK(hipEventRecord(c->ev[3], st));
    CHK(hipStreamSynchronize(st));
  }
  if (!retry && c->change_checks_env < 0)  // (h[3]: the call's frames, from stream_counts)
    c->change_checks = h[3] == 0 || nbytes / h[3] >= 512 ? 1 : 0;
  if (retry) h[1] |= miss;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[1], c->ev[2]);
  c->timing.decode_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[3]);
  c->timing.total_ms = ms;
  c->timing.finalize_ms = 0;
  c->timing.strict_reruns = 0;
  c->timing.exact_retries = 0;
  c->timing.spec_repairs = (uint32_t)pass;
  c->timing.verify_relisted = relisted;
  TRACE("decode_spec done: tiles=%u flags=%#x", h[0], h[1]);
  if (dstats) {
    unsigned long long hs[64];
    CHK(hipMemcpy(hs, dstats, sizeof(hs), hipMemcpyDeviceToHost));
    fprintf(stderr, "[drp-spec] misses=%llu", hs[0]);
    for (unsigned k = 0; k < 5 && k < hs[0]; k++)
      fprintf(stderr, " | t=%llu e=%#llx claim=%#llx exit=%#llx", hs[1 + 6 * k], hs[2 + 6 * k], hs[3 + 6 * k],
              hs[4 + 6 * k]);
    fprintf(stderr, " walk: synced regions=%llu deaths=%llu first death at %#llx lds=%#llx hbm=%#llx w|lane|o=%#llx", hs[31], hs[32],
            hs[36], hs[37], hs[38], hs[39]);
    fprintf(stderr, " sync (lane sums): shape_cyc=%llu rest_cyc=%llu all_cyc=%llu shape_steps=%llu shaped_checks=%llu"
            " merge_live=%llu merge_chains=%llu general=%llu", hs[33], hs[34], hs[35], hs[40], hs[41], hs[42], hs[43], hs[44]);
    fprintf(stderr, " repairs=%d (avg cycles per tile) link_rounds=%llu max=%llu tiles_over8=%llu restart_tiles=%llu"
            " jump_tiles=%llu seg_claims: walk_cycles=%llu frames=%llu tiles=%llu wg_cycles=%llu\n", pass, hs[56],
            hs[57], hs[58], hs[59], hs[60], hs[61], hs[62], hs[63], hs[55]);
  }
  if (h[1] & drp_spec_retry_mask()) return DRP_E_RETRY;
  if (h[1]) return DRP_E_CAPACITY;
  return DRP_OK;
}

int run_decode(drp_ctx *c, const uint8_t *bytes, uint64_t nbytes, const uint64_t *stream_off,
               const uint64_t *entry, uint64_t ns, const drp_frames *fr, const drp_changes *co,
               uint64_t cap, drp_stream_result *res) {
  if (ns == 0) return DRP_OK;
  float spec_ms = 0, spec_total = 0;
  if (!c->exact && !c->strict) {
    const int r = run_decode_spec(c, bytes, nbytes, stream_off, entry, ns, fr, co, cap, res);
    if (r != DRP_E_RETRY) return r;
    spec_ms = c->timing.decode_ms;
    spec_total = c->timing.total_ms;
    TRACE("decode_spec: prediction failed, exact re-run");
  }
  const int r = run_decode_exact(c, bytes, nbytes, stream_off, entry, ns, fr, co, cap, res);
  if (spec_total > 0) {  // report the whole cost of the call
    c->timing.decode_ms += spec_ms;
    c->timing.total_ms += spec_total;
    c->timing.strict_reruns = 1;
  }
  return r;
}

// carve SoA outputs for `cap` frames out of a device buffer
void carve(DevBuf &b, uint64_t cap, drp_frames &fr, drp_changes &co) {
  size_t o = 0;
  auto take = [&](size_t bytes) { void *p = b.at<char>(o); o += al(bytes); return p; };
  fr.payload_off = (uint64_t *)take(cap * 8);
  fr.payload_len = (uint32_t *)take(cap * 4);
  fr.type = (uint8_t *)take(cap);
  co.key_off = (uint32_t *)take(cap * 4);
  co.key_len = (uint32_t *)take(cap * 4);
  co.subset_off = (uint32_t *)take(cap * 4);
  co.subset_len = (uint32_t *)take(cap * 4);
  co.value_off = (uint32_t *)take(cap * 4);
  co.value_len = (uint32_t *)take(cap * 4);
  co.change = (uint64_t *)take(cap * 8);
  co.from = (uint64_t *)take(cap * 8);
  co.to = (uint64_t *)take(cap * 8);
  co.flags = (uint8_t *)take(cap);
  co.key_hash = (uint64_t *)take(cap * 8);
}
size_t carve_bytes(uint64_t cap) { return 14 * 256 + cap * 70; }

}  // namespace

extern "C" {

int drp_decode_device(drp_ctx *c, const uint8_t *bytes, uint64_t nbytes, const uint64_t *stream_off,
                      const uint64_t *entry, uint64_t nstreams, const drp_frames *frames,
                      const drp_changes *cols, uint64_t cap, drp_stream_result *results) {
  if (!c || !stream_off || !frames || !cols || !results || (!bytes && nbytes)) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  return run_decode(c, bytes, nbytes, stream_off, entry, nstreams, frames, cols, cap, results);
}

// drp_decode_batch into caller-owned DEVICE columns: the whole batch is staged and decoded in place.
static int decode_batch_device_out(drp_ctx *c, const uint8_t *bytes, uint64_t n, drp_carry *carry,
                                   const drp_frames *frames, const drp_changes *cols, uint64_t cap,
                                   uint64_t *n_frames, uint64_t *err_frame, uint32_t *err_code,
                                   uint32_t *err_detail) {
  const bool out_dev = true;
  carry->frame_bytes = 0;
  c->staged.rows = 0;
  hipStream_t st = c->st;
  *err_frame = ~0ull;
  *err_code = DRP_ERR_NONE;
  *err_detail = 0;
  uint64_t nf0 = 0;
  const uint64_t brem = carry->blob_remaining;
  // A blob continuation (decode.js _id == 2 with _missing > 0 across _write calls) is frame 0.
  if (brem) {
    if (cap < 1) return DRP_E_CAPACITY;
    uint64_t off0 = 0;
    uint32_t len0 = brem > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)brem;
    uint8_t ty0 = DRP_TYPE_BLOB | DRP_FRAME_CONT | (brem > n ? DRP_FRAME_PARTIAL : 0);
    if (out_dev) {
      CHK(hipMemcpyAsync(frames->payload_off, &off0, 8, hipMemcpyHostToDevice, st));
      CHK(hipMemcpyAsync(frames->payload_len, &len0, 4, hipMemcpyHostToDevice, st));
      CHK(hipMemcpyAsync(frames->type, &ty0, 1, hipMemcpyHostToDevice, st));
      CHK(hipStreamSynchronize(st));
    } else {
      frames->payload_off[0] = off0;
      frames->payload_len[0] = len0;
      frames->type[0] = ty0;
    }
    nf0 = 1;
    if (brem >= n) {
      carry->blob_remaining = brem - n;
      carry->consumed = n;
      carry->tail_kind = carry->blob_remaining ? DRP_TAIL_BLOB : DRP_TAIL_NONE;
      *n_frames = 1;
      return DRP_OK;
    }
  }
  const uint64_t entry0 = brem;
  // input: device & aligned, or staged
  const uint8_t *dbytes = bytes;
  const size_t stage_meta = 256;
  if (!c->aux.ensure(stage_meta + sizeof(drp_stream_result) + 64)) return DRP_E_NOMEM;
  uint64_t *soff = c->aux.at<uint64_t>(0);
  uint64_t *ent = c->aux.at<uint64_t>(16);
  drp_stream_result *dres = c->aux.at<drp_stream_result>(stage_meta);
  if (!is_device_ptr(bytes) || ((uintptr_t)bytes & 15)) {
    if (!c->in_stage.ensure(n + 64)) return DRP_E_NOMEM;
    if (n) CHK(hipMemcpyAsync(c->in_stage.p, bytes, n, hipMemcpyDefault, st));
    dbytes = (const uint8_t *)c->in_stage.p;
  }
  uint64_t hv[3] = {0, n, entry0};
  CHK(hipMemcpyAsync(soff, hv, 16, hipMemcpyHostToDevice, st));
  CHK(hipMemcpyAsync(ent, hv + 2, 8, hipMemcpyHostToDevice, st));
  const uint64_t cap_rest = cap - nf0;
  drp_frames dfr;
  drp_changes dco;
  if (out_dev) {
    dfr.payload_off = frames->payload_off + nf0;
    dfr.payload_len = frames->payload_len + nf0;
    dfr.type = frames->type + nf0;
    dco.key_off = cols->key_off + nf0;
    dco.key_len = cols->key_len + nf0;
    dco.subset_off = cols->subset_off + nf0;
    dco.subset_len = cols->subset_len + nf0;
    dco.value_off = cols->value_off + nf0;
    dco.value_len = cols->value_len + nf0;
    dco.change = cols->change + nf0;
    dco.from = cols->from + nf0;
    dco.to = cols->to + nf0;
    dco.flags = cols->flags + nf0;
    dco.key_hash = cols->key_hash ? cols->key_hash + nf0 : nullptr;
  } else {
    if (!c->out_stage.ensure(carve_bytes(cap_rest))) return DRP_E_NOMEM;
    carve(c->out_stage, cap_rest, dfr, dco);
  }
  int rc = run_decode(c, dbytes, n, soff, ent, 1, &dfr, &dco, cap_rest, dres);
  if (rc != DRP_OK && rc != DRP_E_CAPACITY) return rc;
  drp_stream_result r;
  CHK(hipMemcpyAsync(&r, dres, sizeof(r), hipMemcpyDeviceToHost, st));
  CHK(hipStreamSynchronize(st));
  const uint64_t nf = r.frames;
  // keep the failing Change in the table (its flags say why)
  uint64_t ncopy = nf + ((r.err_code == DRP_ERR_CHANGE || r.err_code == DRP_ERR_REQUIRED) ? 1 : 0);
  if (ncopy > cap_rest) ncopy = cap_rest;
  if (!out_dev && ncopy) {
    auto cp = [&](void *dst, const void *src, size_t bytes) {
      return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
    };
    CHK(cp(frames->payload_off + nf0, dfr.payload_off, ncopy * 8));
    CHK(cp(frames->payload_len + nf0, dfr.payload_len, ncopy * 4));
    CHK(cp(frames->type + nf0, dfr.type, ncopy));
    CHK(cp(cols->key_off + nf0, dco.key_off, ncopy * 4));
    CHK(cp(cols->key_len + nf0, dco.key_len, ncopy * 4));
    CHK(cp(cols->subset_off + nf0, dco.subset_off, ncopy * 4));
    CHK(cp(cols->subset_len + nf0, dco.subset_len, ncopy * 4));
    CHK(cp(cols->value_off + nf0, dco.value_off, ncopy * 4));
    CHK(cp(cols->value_len + nf0, dco.value_len, ncopy * 4));
    CHK(cp(cols->change + nf0, dco.change, ncopy * 8));
    CHK(cp(cols->from + nf0, dco.from, ncopy * 8));
    CHK(cp(cols->to + nf0, dco.to, ncopy * 8));
    CHK(cp(cols->flags + nf0, dco.flags, ncopy));
    CHK(hipStreamSynchronize(st));
  }
  *n_frames = nf0 + nf;
  if (r.err_code) {
    *err_frame = nf0 + r.err_frame;
    *err_code = r.err_code;
    *err_detail = r.err_detail;
  }
  carry->blob_remaining = r.blob_remaining;
  carry->consumed = r.consumed;
  carry->tail_kind = r.tail_kind;
  carry->frame_bytes = r.tail_kind == DRP_TAIL_CHANGE ? r.tail_frame_bytes : 0;
  return rc;
}


constexpr uint64_t kPieceMin = 64 << 10;     // bytes of a blob-skipping piece, at least
constexpr uint64_t kPieceMargin = 64 << 10;  // past the predicted next blob header
constexpr uint64_t kPiecesMin = 1 << 20;     // batches below this are staged whole
// A piece costs ~150 us of host time (its launch sequence and two waits) however small it is, and
// a flat batch (one buffer the DMA engine reads directly) stages at the full PCIe rate, so when the
// blobs are dense (C3: a 1 MiB blob per 86 KB of Changes, ~950 pieces per GiB: 132 ms) the rest of
// a flat batch goes in one more piece as soon as more than kPieceBudget pieces are still expected
// (~20 ms per GiB by DMA). Chunked batches keep their pieces: staging them whole would copy every
// blob payload on the host into the pinned gather buffer.
constexpr uint64_t kPieceBudget = 8;
constexpr uint64_t kPieceProbe = 4;  // pieces of a batch before its own span is trusted
// A flat batch in page-locked memory that is staged whole (or its rest, above) is decoded as it
// lands: the DMA engine copies it in chunks of at least drp_ctx::pipe_chunk (128 MiB; 64 and 256
// measured 0.3 and 0.2 ms slower on C3) on the ctx's copy stream while the compute stream decodes a
// piece per chunk (each piece waits for its chunk's event) and fetches its rows into
// drp_decode_batch's host columns, so only the last chunk's decode and fetch follow the copy (C3:
// 19 ms of PCIe per GiB, 2.8 ms of decode and 1.3 ms of fetch).
constexpr uint64_t kPipeEvents = 32;  // chunks at most (drp_ctx::pev)

// payload offsets of a pipelined piece's rows: piece-relative -> relative to the pipelined range
__global__ void piece_shift_kernel(uint64_t *payload_off, uint64_t n, uint64_t d) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
    payload_off[i] += d;
}

// The staged rows' capacity for m bytes: from the density of the ctx's previous batch (a
// stream's batches are alike), 1/32 per byte at first.
static uint64_t stage_cap(const drp_ctx *c, uint64_t m) {
  const double dens = c->frames_per_byte > 0 ? c->frames_per_byte * 1.25 : 1.0 / 32;
  return (uint64_t)((double)m * dens) + 1024;
}

// Batch bytes [a, a + len) into device memory at dst (asynchronously on st). A chunked batch's
// range is gathered into the ctx's page-locked buffer first (*copied counts those host bytes),
// so the copy into HBM runs by DMA and only the staged ranges are ever copied on the host.
static int h2d_range(drp_ctx *c, const HostSrc &H, uint64_t a, uint64_t len, void *dst, hipStream_t st,
                     uint64_t *copied) {
  if (!len) return DRP_OK;
  if (H.flat) {
    CHK(hipMemcpyAsync(dst, H.flat + a, len, hipMemcpyDefault, st));
    return DRP_OK;
  }
  if (!c->gather.ensure(len)) return DRP_E_NOMEM;
  CHK(hipStreamSynchronize(st));  // (the buffer's previous range has left)
  uint8_t *g = static_cast<uint8_t *>(c->gather.p);
  uint64_t k = (uint64_t)(std::upper_bound(H.start.begin(), H.start.end(), a) - H.start.begin()) - 1;
  for (uint64_t at = a, end = a + len; at < end; k++) {
    const uint64_t s0 = H.start[k], take = std::min(end, s0 + H.ch[k].n) - at;
    memcpy(g + (at - a), H.ch[k].bytes + (at - s0), take);
    at += take;
  }
  *copied += len;
  CHK(hipMemcpyAsync(dst, g, len, hipMemcpyHostToDevice, st));
  return DRP_OK;
}

// Pass-through of in-batch blob payloads (drp_set_blob_skip): bytes [pos, n) of a host batch are
// staged and decoded piece by piece. A piece ends kPieceMargin past where the next blob header
// is expected (the distance from a piece's start to its blob header, learned); when the
// decode of a piece ends inside a blob, the next piece starts after that blob, so the blob's
// remaining payload is never copied. A piece that ends inside a header or a Change frame is
// resumed at that frame. The rows of all pieces are consecutive, as a whole-batch decode
// writes them (a blob the batch holds whole loses the PARTIAL mark its piece gave it).
// DRP_E_RETRY: the capacity guess was short; the caller stages the batch whole.
// a piece's stream bounds and entry (no host buffer to keep alive: the values travel as arguments)
__global__ void piece_meta_kernel(uint64_t *soff, uint64_t *ent, uint64_t n, uint64_t e) {
  soff[0] = 0;
  soff[1] = n;
  ent[0] = e;
}

// the payload offset of a piece's last row (a cut blob's), next to its stream result
__global__ void piece_tail_kernel(const drp_stream_result *r, const uint64_t *payload_off, uint64_t *boff) {
  *boff = r->frames ? payload_off[r->frames - 1] : 0;
}

static int fetch_staged(drp_ctx *c, const drp_frames *frames, const drp_changes *cols, uint64_t first,
                        uint64_t rows);

// staged rows [first, first + rows) into host columns from their row `first` on (fetch_staged
// writes from row 0)
static int fetch_staged_at(drp_ctx *c, const drp_frames *frames, const drp_changes *cols, uint64_t first,
                           uint64_t rows) {
  drp_frames f = *frames;
  drp_changes o = *cols;
  f.payload_off += first;
  f.payload_len += first;
  f.type += first;
  o.key_off += first;
  o.key_len += first;
  o.subset_off += first;
  o.subset_len += first;
  o.value_off += first;
  o.value_len += first;
  o.change += first;
  o.from += first;
  o.to += first;
  o.flags += first;
  if (o.key_hash) o.key_hash += first;
  return fetch_staged(c, &f, &o, first, rows);
}

// An early fetch of pipelined pieces (worker thread): staged GPU rows [g0, g0 + ng) into the host
// columns from row `dst` on, by DMA into the pinned bounce buffer on the fetch stream (behind
// c->fev, recorded after the rows' last writes) and a host copy from there; payload offsets made
// batch offsets per piece as fetch_staged does. The caller sized c->fbounce (fetch_bounce_bytes).
struct FetchCol {
  const void *src;
  void *dst;
  uint32_t w;
};
static int fetch_cols(const drp_ctx *c, const drp_frames *F, const drp_changes *O, FetchCol *col) {
  const auto &S = c->staged;
  const void *src[14] = {S.fr.payload_off, S.fr.payload_len, S.fr.type, S.co.key_off, S.co.key_len,
                         S.co.subset_off, S.co.subset_len, S.co.value_off, S.co.value_len, S.co.change,
                         S.co.from, S.co.to, S.co.flags, S.co.key_hash};
  void *dst[14] = {F->payload_off, F->payload_len, F->type, O->key_off, O->key_len, O->subset_off, O->subset_len,
                   O->value_off, O->value_len, O->change, O->from, O->to, O->flags, O->key_hash};
  static const uint32_t W[14] = {8, 4, 1, 4, 4, 4, 4, 4, 4, 8, 8, 8, 1, 8};
  int n = 0;
  for (int k = 0; k < 14; k++)
    if (src[k] && dst[k]) col[n++] = {src[k], dst[k], W[k]};
  return n;
}
constexpr uint64_t kBounceRows = 1 << 20;  // rows per bounce round (14 columns: <= 112 MiB pinned)
static uint64_t fetch_bounce_bytes(uint64_t ng) { return 14 * al(std::min(ng, kBounceRows) * 8); }
static int fetch_bounce(drp_ctx *c, uint64_t dst, uint64_t g0, uint64_t ng) {
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  FetchCol col[14];
  const int n = fetch_cols(c, c->dfr, c->dco, col);
  uint8_t *b = static_cast<uint8_t *>(c->fbounce.p);
  CHK(hipStreamWaitEvent(c->fst, c->fev, 0));
  for (uint64_t r = 0; r < ng; r += kBounceRows) {
    const uint64_t m = std::min(kBounceRows, ng - r);
    uint64_t o = 0;
    for (int k = 0; k < n; o += al(m * col[k].w), k++)
      CHK(hipMemcpyAsync(b + o, static_cast<const uint8_t *>(col[k].src) + (g0 + r) * col[k].w, m * col[k].w,
                         hipMemcpyDeviceToHost, c->fst));
    CHK(hipStreamSynchronize(c->fst));
    o = 0;
    for (int k = 0; k < n; o += al(m * col[k].w), k++)
      memcpy(static_cast<uint8_t *>(col[k].dst) + (dst + r) * col[k].w, b + o, m * col[k].w);
  }
  const auto &S = c->staged;
  for (size_t k = 0; k < S.pieces.size(); k++) {
    const uint64_t r0 = S.pieces[k].first, r1 = k + 1 < S.pieces.size() ? S.pieces[k + 1].first : ~0ull;
    const uint64_t sh = S.pieces[k].second, lo = std::max(r0, g0), hi = std::min(r1, g0 + ng);
    if (sh)
      for (uint64_t g = lo; g < hi; g++) c->dfr->payload_off[dst + (g - g0)] += sh;
  }
  return DRP_OK;
}

static int stage_pieces(drp_ctx *c, const HostSrc &H, uint64_t pos, bool pipe, drp_carry *carry,
                        uint64_t *n_frames, uint64_t *err_frame, uint32_t *err_code, uint32_t *err_detail) {
  hipStream_t st = c->st;
  // pipelined (pipe): [pbase, n) goes to in_stage (offset 0) by DMA on c->cst, chunk k ending at
  // pend[k] and signalled by c->pev[k]; each piece ends at a chunk's end. The copy stream is
  // drained on every way out (its DMAs write into in_stage).
  uint64_t pbase = 0, jumped = 0;
  double tf = 0, tw = 0, tb = now_ms();  // (DRP_TRACE: early-fetch and piece-wait host time)
  int nfetch = 0;
  // the early fetches (pipe, drp_decode_batch's host columns): one worker thread at a time
  std::thread fetcher;
  int fetch_rc = DRP_OK;
  struct Join {
    std::thread &t;
    ~Join() {
      if (t.joinable()) t.join();
    }
  } join{fetcher};
  std::vector<uint64_t> pend;
  size_t pk = 0;
  struct Drain {
    drp_ctx *c;
    const std::vector<uint64_t> &pend;
    ~Drain() {
      if (!pend.empty()) (void)hipStreamSynchronize(c->cst);
    }
  } drain{c, pend};
  auto &S = c->staged;
  const size_t stage_meta = 256;
  if (!c->aux.ensure(stage_meta + sizeof(drp_stream_result) + 64)) return DRP_E_NOMEM;
  uint64_t *soff = c->aux.at<uint64_t>(0);
  uint64_t *ent = c->aux.at<uint64_t>(16);
  drp_stream_result *dres = c->aux.at<drp_stream_result>(stage_meta);
  uint64_t *dboff = c->aux.at<uint64_t>(stage_meta + sizeof(drp_stream_result));
  const uint64_t n = H.n;
  uint64_t copied = 0;
  const uint64_t cap = stage_cap(c, n - pos);
  if (!c->dec_cols.ensure(carve_bytes(cap))) return DRP_E_NOMEM;
  carve(c->dec_cols, cap, S.fr, S.co);
  if (c->key_post != DRP_KEY_POST_HASH) S.co.key_hash = nullptr;
  S.cap = cap;
  S.pieces.clear();
  uint64_t rows = 0, staged = 0, skipped = 0;
  // the next piece: kPieceMargin past where the last blob seen suggests the next blob header is;
  // doubled within this batch after each piece that met no blob
  uint64_t want = std::max(kPieceMin, c->blob_run + kPieceMargin);
  const uint64_t pos0 = pos;
  uint64_t npieces = 0, span_now = 0;  // (span_now: batch bytes per piece so far)
  float h2d_ms = 0;
  drp_timing sum = {};
  // (per piece, one wait for the decode's verification and one for its result: the H2D, the
  // piece's bounds and the blob row's type are queued on the stream)
  struct {
    drp_stream_result r;
    uint64_t boff;  // the cut blob's payload offset in the piece (tail BLOB)
  } hr;
  drp_stream_result &r = hr.r;
  for (;;) {
    if (!pipe && H.flat && c->blob_skip == DRP_BLOB_SKIP_AUTO) {  // dense blobs in a flat batch: the rest in one piece
      const uint64_t span = npieces >= kPieceProbe ? span_now : c->piece_span;
      if (span && (n - pos) / span > kPieceBudget) {
        want = n - pos;
        pipe = c->pipe_chunk && n - pos >= 2 * c->pipe_chunk && is_pinned_host(H.flat);
      }
    }
    if (pipe && pend.empty()) {  // (the compute stream is idle here: every piece ends in a wait)
      pbase = pos & ~15ull;
      const uint64_t m = n - pbase;
      if (!c->in_stage.ensure(m + 64)) return DRP_E_NOMEM;
      // uniform chunks, then a half and a quarter chunk: the decode and fetch left after the copy
      // are a quarter chunk's (each piece's decode hides behind the next, shorter copy)
      const uint64_t chunk =
          (std::max(c->pipe_chunk, (m + kPipeEvents - 3) / (kPipeEvents - 2)) + 0xFFFF) & ~0xFFFFull;
      const uint64_t t2 = (n - chunk / 4) & ~0xFFFFull, t1 = (n - 3 * chunk / 4) & ~0xFFFFull;
      for (uint64_t e = pbase + chunk; e < t1; e += chunk) pend.push_back(e);
      if (t1 > pbase) pend.push_back(t1);
      if (t2 > t1) pend.push_back(t2);
      pend.push_back(n);
      CHK(hipEventRecord(c->hev[0], c->cst));
      for (size_t k = 0; k < pend.size(); k++) {
        if (!c->pev[k]) CHK(hipEventCreateWithFlags(&c->pev[k], hipEventDisableTiming));
        const uint64_t lo = k ? pend[k - 1] : pbase;
        CHK(hipMemcpyAsync(c->in_stage.at<uint8_t>(lo - pbase), H.flat + lo, pend[k] - lo, hipMemcpyHostToDevice,
                           c->cst));
        CHK(hipEventRecord(c->pev[k], c->cst));
      }
      CHK(hipEventRecord(c->hev[1], c->cst));
      TRACE("stage: pipelined from %llu in %zu chunks of %llu B", (unsigned long long)pbase, pend.size(),
            (unsigned long long)chunk);
      staged += m;
      S.pieces.emplace_back(rows, pbase);
    }
    uint64_t pe, ps, mp;
    const uint8_t *dp;
    if (pipe) {  // to the end of the first chunk past pos (and past the last piece's end)
      while (pk < pend.size() && pend[pk] <= pos) pk++;
      if (pk == pend.size()) return DRP_E_HIP;  // (unreachable: pos < n)
      pe = pend[pk];
      ps = pos & ~15ull;
      mp = pe - ps;
      dp = c->in_stage.at<uint8_t>(ps - pbase);
      CHK(hipStreamWaitEvent(st, c->pev[pk], 0));
      pk++;
      hipLaunchKernelGGL(piece_meta_kernel, dim3(1), dim3(1), 0, st, soff, ent, mp, pos - ps);
      CHK(hipGetLastError());
    } else {
      pe = std::min(n, pos + want);
      ps = pos & ~15ull;
      mp = pe - ps;
      if (!c->in_stage.ensure(mp + 64)) return DRP_E_NOMEM;
      dp = static_cast<const uint8_t *>(c->in_stage.p);
      CHK(hipEventRecord(c->hev[0], st));
      if (const int rc = h2d_range(c, H, ps, mp, c->in_stage.p, st, &copied)) return rc;
      hipLaunchKernelGGL(piece_meta_kernel, dim3(1), dim3(1), 0, st, soff, ent, mp, pos - ps);
      CHK(hipGetLastError());
      CHK(hipEventRecord(c->hev[1], st));
      staged += mp;
    }
    npieces++;
    drp_frames fr;
    drp_changes co;
    fr.payload_off = S.fr.payload_off + rows;
    fr.payload_len = S.fr.payload_len + rows;
    fr.type = S.fr.type + rows;
    co.key_off = S.co.key_off + rows;
    co.key_len = S.co.key_len + rows;
    co.subset_off = S.co.subset_off + rows;
    co.subset_len = S.co.subset_len + rows;
    co.value_off = S.co.value_off + rows;
    co.value_len = S.co.value_len + rows;
    co.change = S.co.change + rows;
    co.from = S.co.from + rows;
    co.to = S.co.to + rows;
    co.flags = S.co.flags + rows;
    co.key_hash = S.co.key_hash ? S.co.key_hash + rows : nullptr;
    const int rc = run_decode(c, dp, mp, soff, ent, 1, &fr, &co, cap - rows, dres);
    if (rc == DRP_E_CAPACITY) return DRP_E_RETRY;
    if (rc != DRP_OK) return rc;
    // (run_decode describes one launch sequence: the call's timing is the sum over its pieces)
    sum.decode_ms += c->timing.decode_ms;
    sum.total_ms += c->timing.total_ms;
    sum.strict_reruns += c->timing.strict_reruns;
    sum.spec_repairs += c->timing.spec_repairs;
    sum.exact_retries += c->timing.exact_retries;
    sum.verify_relisted += c->timing.verify_relisted;
    sum.seg_repairs += c->timing.seg_repairs;
    hipLaunchKernelGGL(piece_tail_kernel, dim3(1), dim3(1), 0, st, dres, fr.payload_off, dboff);
    CHK(hipGetLastError());
    CHK(hipMemcpyAsync(&hr, dres, sizeof(hr), hipMemcpyDeviceToHost, st));
    {
      const double t0 = now_ms();
      CHK(hipStreamSynchronize(st));
      tw += now_ms() - t0;
    }
    const uint64_t boff = hr.boff;
    if (pipe) {  // the pipelined range is one piece: its rows' payload offsets from pbase
      const uint64_t nr = r.frames + ((r.err_code == DRP_ERR_CHANGE || r.err_code == DRP_ERR_REQUIRED) ? 1 : 0);
      if (nr && ps > pbase) {
        const uint32_t g = (uint32_t)std::min<uint64_t>((nr + 255) / 256, 1024);
        hipLaunchKernelGGL(piece_shift_kernel, dim3(g), dim3(256), 0, st, fr.payload_off, nr, ps - pbase);
        CHK(hipGetLastError());
      }
      S.dev = static_cast<const uint8_t *>(c->in_stage.p);
    } else {
      float ms = 0;
      if (hipEventElapsedTime(&ms, c->hev[0], c->hev[1]) == hipSuccess) h2d_ms += ms;
      S.pieces.emplace_back(rows, ps);
      S.dev = static_cast<const uint8_t *>(c->in_stage.p);
    }
    const uint64_t bad = (r.err_code == DRP_ERR_CHANGE || r.err_code == DRP_ERR_REQUIRED) ? 1 : 0;
    if (r.err_code || pe == n) {  // the batch's end or its error: this piece's tail is the batch's
      if (r.err_code) {
        *err_frame = S.nf0 + rows + r.err_frame;
        *err_code = r.err_code;
        *err_detail = r.err_detail;
      }
      rows += r.frames + bad;
      carry->blob_remaining = r.blob_remaining;
      carry->consumed = r.err_code ? n : r.consumed + ps;  // (an error ends the stream: nothing carried)
      carry->tail_kind = r.tail_kind;
      carry->frame_bytes = r.tail_kind == DRP_TAIL_CHANGE ? r.tail_frame_bytes : 0;
      break;
    }
    rows += r.frames;
    if (r.tail_kind == DRP_TAIL_BLOB) {
      const uint64_t bend = pe + r.blob_remaining;  // the blob's end in the batch
      c->blob_run = ps + boff - pos;                // (where this piece's blob payload began)
      want = std::max(kPieceMin, c->blob_run + kPieceMargin);
      if (bend <= n) {  // the batch holds the whole blob: its row is not partial
        CHK(hipMemsetAsync(S.fr.type + rows - 1, DRP_TYPE_BLOB, 1, st));
        (pipe ? jumped : skipped) += bend - pe;
        pos = bend;
        span_now = (pos - pos0) / npieces;
        if (pos == n) {
          carry->blob_remaining = 0;
          carry->consumed = n;
          carry->tail_kind = DRP_TAIL_NONE;
          break;
        }
      } else {  // the blob continues past the batch: the carry says how far
        (pipe ? jumped : skipped) += n - pe;
        carry->blob_remaining = bend - n;
        carry->consumed = n;
        carry->tail_kind = DRP_TAIL_BLOB;
        break;
      }
    } else {
      // no blob reached: resume at the frame the piece cut (or its end), with a longer piece
      const uint64_t np = r.tail_kind == DRP_TAIL_NONE ? pe : ps + r.consumed;
      want *= 2;
      if (np > pos) pos = np;
      span_now = (pos - pos0) / npieces;
    }
    if (pipe && c->dfr) {  // the rows so far into drp_decode_batch's host columns, while the copy runs
      const uint64_t upto = std::min(S.nf0 + rows, c->dcap);
      if (upto > c->dfetched) {
        const double t0 = now_ms();
        if (fetcher.joinable()) fetcher.join();
        tf += now_ms() - t0;
        if (fetch_rc) return fetch_rc;
        uint64_t a = c->dfetched;
        if (a == 0 && S.nf0) {  // (the carried blob's row, built on the host)
          c->dfr->payload_off[0] = S.off0;
          c->dfr->payload_len[0] = S.len0;
          c->dfr->type[0] = S.ty0;
          a = 1;
        }
        if (upto > a) {
          const uint64_t g0 = a - S.nf0, ng = upto - a;
          if (c->fbounce.ensure(fetch_bounce_bytes(ng))) {
            CHK(hipEventRecord(c->fev, st));
            fetcher = std::thread([c, a, g0, ng, &fetch_rc] { fetch_rc = fetch_bounce(c, a, g0, ng); });
          } else {  // (no pinned bounce buffer: a direct fetch here)
            S.rows = S.nf0 + rows;
            if (const int rc = fetch_staged_at(c, c->dfr, c->dco, a, ng)) return rc;
          }
          nfetch++;
        }
        c->dfetched = upto;
      }
    }
  }
  if (fetcher.joinable()) {
    const double t0 = now_ms();
    fetcher.join();
    tf += now_ms() - t0;
  }
  if (fetch_rc) return fetch_rc;
  c->timing = sum;
  if (span_now) c->piece_span = span_now;
  if (!pend.empty()) {
    CHK(hipStreamSynchronize(c->cst));
    float ms = 0;
    if (hipEventElapsedTime(&ms, c->hev[0], c->hev[1]) == hipSuccess) h2d_ms += ms;
  }
  c->timing.h2d_ms = h2d_ms;
  TRACE("stage: %llu pieces in %.2f ms (h2d %.2f): %d early fetches (%.2f ms waited for), result waits %.2f ms",
        (unsigned long long)npieces, now_ms() - tb, h2d_ms, nfetch, tf, tw);
  c->timing.h2d_bytes = staged;
  c->timing.h2d_skipped = skipped;
  c->timing.host_copied = copied;
  c->blob_heavy = (skipped + jumped) * 4 >= n;  // (AUTO: keep skipping while it pays)
  c->frames_per_byte = (double)rows / (double)(n - S.pieces[0].second);
  S.rows = S.nf0 + rows;
  *n_frames = S.nf0 + rows - ((*err_code == DRP_ERR_CHANGE || *err_code == DRP_ERR_REQUIRED) ? 1 : 0);
  return DRP_OK;
}

// Decode a host batch (bytes [a, n), a = the 16-byte-aligned start of the bytes after a leading
// blob continuation) into the ctx's device columns. The frame capacity starts at a guess and is
// grown to the exact count when the first launch overflows it (the count is exact either way).
static int stage_decode(drp_ctx *c, const HostSrc &H, drp_carry *carry, uint64_t *n_frames,
                        uint64_t *err_frame, uint32_t *err_code, uint32_t *err_detail) {
  hipStream_t st = c->st;
  const uint64_t n = H.n;
  const uint8_t *bytes = H.flat;
  auto &S = c->staged;
  S.rows = S.nf0 = 0;
  S.pieces.clear();
  *err_frame = ~0ull;
  *err_code = DRP_ERR_NONE;
  *err_detail = 0;
  carry->frame_bytes = 0;
  c->timing.h2d_bytes = 0;
  c->timing.h2d_skipped = 0;
  c->timing.host_copied = 0;
  const uint64_t brem = carry->blob_remaining;
  // A blob continuation (decode.js _id == 2 with _missing > 0 across _write calls) is row 0.
  if (brem) {
    S.nf0 = 1;
    S.off0 = 0;
    S.len0 = brem > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)brem;
    S.ty0 = DRP_TYPE_BLOB | DRP_FRAME_CONT | (brem > n ? DRP_FRAME_PARTIAL : 0);
    if (brem >= n) {
      carry->blob_remaining = brem - n;
      carry->consumed = n;
      carry->tail_kind = carry->blob_remaining ? DRP_TAIL_BLOB : DRP_TAIL_NONE;
      *n_frames = 1;
      S.rows = 1;
      return DRP_OK;
    }
  }
  const bool host_in = !bytes || !is_device_ptr(bytes) || ((uintptr_t)bytes & 15);
  const bool pieces = host_in && n - brem >= kPiecesMin &&
                      (c->blob_skip == DRP_BLOB_SKIP_ALWAYS ||
                       (c->blob_skip == DRP_BLOB_SKIP_AUTO && (c->blob_heavy || c->frames_per_byte == 0)));
  // a large flat batch in page-locked memory staged whole: decoded as it lands (pipe_chunk)
  const bool pipe =
      !pieces && host_in && H.flat && c->pipe_chunk && n - brem >= 2 * c->pipe_chunk && is_pinned_host(H.flat);
  TRACE("stage: %llu B, host %d flat %d pinned %d pieces %d pipe %d", (unsigned long long)n, (int)host_in,
        H.flat != nullptr, (int)(H.flat && is_pinned_host(H.flat)), (int)pieces, (int)pipe);
  if (pieces || pipe) {
    // (AUTO: a ctx's first batch probes in pieces too; pieces grow geometrically while no blob
    // is met, so a batch without blobs costs a few more launches once)
    const drp_carry in = *carry;
    const int rc = stage_pieces(c, H, brem, pipe, carry, n_frames, err_frame, err_code, err_detail);
    if (rc != DRP_E_RETRY) return rc;
    c->dfetched = 0;
    *carry = in;  // (capacity: staged whole below)
    *err_frame = ~0ull;
    *err_code = DRP_ERR_NONE;
    *err_detail = 0;
    S.pieces.clear();
  }
  // the continuation's payload bytes are pass-through: only [a, n) goes to the device
  const uint64_t a = brem & ~15ull, m = n - a;
  const uint8_t *dbytes = bytes ? bytes + a : nullptr;
  float h2d_ms = 0;
  uint64_t copied = 0;
  if (host_in) {
    if (!c->in_stage.ensure(m + 64)) return DRP_E_NOMEM;
    const double t0 = now_ms();
    if (m) {
      if (const int rc = h2d_range(c, H, a, m, c->in_stage.p, st, &copied)) return rc;
      CHK(hipStreamSynchronize(st));
    }
    h2d_ms = (float)(now_ms() - t0);
    dbytes = (const uint8_t *)c->in_stage.p;
  }
  const size_t stage_meta = 256;
  if (!c->aux.ensure(stage_meta + sizeof(drp_stream_result) + 64)) return DRP_E_NOMEM;
  uint64_t *soff = c->aux.at<uint64_t>(0);
  uint64_t *ent = c->aux.at<uint64_t>(16);
  uint64_t *bsum = c->aux.at<uint64_t>(24);
  drp_stream_result *dres = c->aux.at<drp_stream_result>(stage_meta);
  uint64_t hv[3] = {0, m, brem - a};
  CHK(hipMemcpyAsync(soff, hv, 16, hipMemcpyHostToDevice, st));
  CHK(hipMemcpyAsync(ent, hv + 2, 8, hipMemcpyHostToDevice, st));
  uint64_t cap = stage_cap(c, m);
  drp_stream_result r;
  int rc = DRP_OK;
  for (int attempt = 0; attempt < 2; attempt++) {
    if (!c->dec_cols.ensure(carve_bytes(cap))) return DRP_E_NOMEM;
    carve(c->dec_cols, cap, S.fr, S.co);
    if (c->key_post != DRP_KEY_POST_HASH) S.co.key_hash = nullptr;
    S.cap = cap;
    rc = run_decode(c, dbytes, m, soff, ent, 1, &S.fr, &S.co, cap, dres);
    if (rc != DRP_OK && rc != DRP_E_CAPACITY) return rc;
    CHK(hipMemcpyAsync(&r, dres, sizeof(r), hipMemcpyDeviceToHost, st));
    CHK(hipStreamSynchronize(st));
    if (rc == DRP_OK) break;
    // The chain held more frames than the guess. Rows needed: the delivered frames plus a
    // malformed Change. When they fit, the result is complete (a malformed Change inside the
    // capacity was seen, so nothing before it was missed; the frames after it are not
    // delivered). Otherwise r.frames is the exact chain count or a malformed Change past the
    // capacity ends the stream earlier: retry at that bound.
    const uint64_t need = r.frames + ((r.err_code == DRP_ERR_CHANGE || r.err_code == DRP_ERR_REQUIRED) ? 1 : 0);
    if (need <= cap) {
      rc = DRP_OK;
      break;
    }
    cap = need + 1;
  }
  if (rc != DRP_OK) return rc;
  if (host_in && c->blob_skip == DRP_BLOB_SKIP_AUTO && r.blobs) {
    // the batch's blob payload bytes: mostly blobs -> the next batches are staged in pieces
    uint64_t bb = 0;
    CHK(hipMemsetAsync(bsum, 0, 8, st));
    CHK(drp_launch_blob_bytes(S.fr.type, S.fr.payload_len, r.frames, bsum, st));
    CHK(hipMemcpyAsync(&bb, bsum, 8, hipMemcpyDeviceToHost, st));
    CHK(hipStreamSynchronize(st));
    c->blob_heavy = bb * 2 >= m;
  } else if (host_in) {
    c->blob_heavy = false;
  }
  c->timing.h2d_ms = h2d_ms;
  c->timing.h2d_bytes = host_in ? m : 0;
  c->timing.host_copied = copied;
  c->frames_per_byte = m ? (double)r.frames / (double)m : 0.0;
  const uint64_t bad = (r.err_code == DRP_ERR_CHANGE || r.err_code == DRP_ERR_REQUIRED) ? 1 : 0;
  S.pieces.emplace_back(0, a);
  S.dev = dbytes;
  S.rows = S.nf0 + r.frames + bad;
  *n_frames = S.nf0 + r.frames;
  if (r.err_code) {
    *err_frame = S.nf0 + r.err_frame;
    *err_code = r.err_code;
    *err_detail = r.err_detail;
  }
  carry->blob_remaining = r.blob_remaining;
  carry->consumed = r.consumed + a;
  carry->tail_kind = r.tail_kind;
  carry->frame_bytes = r.tail_kind == DRP_TAIL_CHANGE ? r.tail_frame_bytes : 0;
  return DRP_OK;
}

// Copy staged rows [first, first + rows) into host columns.
static int fetch_staged(drp_ctx *c, const drp_frames *frames, const drp_changes *cols, uint64_t first,
                        uint64_t rows) {
  auto &S = c->staged;
  if (first > S.rows || rows > S.rows - first) return DRP_E_INVAL;
  if (!rows) return DRP_OK;
  hipStream_t st = c->st;
  uint64_t dst = 0;  // destination row
  if (first == 0 && S.nf0) {
    frames->payload_off[0] = S.off0;
    frames->payload_len[0] = S.len0;
    frames->type[0] = S.ty0;
    dst = 1;
  }
  const uint64_t g0 = first + dst - S.nf0;  // first GPU row
  const uint64_t ng = rows - dst;
  const double t0 = now_ms();
  if (ng) {
    auto cp = [&](void *d, const void *s_, size_t w) {
      return hipMemcpyAsync(static_cast<char *>(d) + dst * w, static_cast<const char *>(s_) + g0 * w, ng * w,
                            hipMemcpyDeviceToHost, st);
    };
    CHK(cp(frames->payload_off, S.fr.payload_off, 8));
    CHK(cp(frames->payload_len, S.fr.payload_len, 4));
    CHK(cp(frames->type, S.fr.type, 1));
    CHK(cp(cols->key_off, S.co.key_off, 4));
    CHK(cp(cols->key_len, S.co.key_len, 4));
    CHK(cp(cols->subset_off, S.co.subset_off, 4));
    CHK(cp(cols->subset_len, S.co.subset_len, 4));
    CHK(cp(cols->value_off, S.co.value_off, 4));
    CHK(cp(cols->value_len, S.co.value_len, 4));
    CHK(cp(cols->change, S.co.change, 8));
    CHK(cp(cols->from, S.co.from, 8));
    CHK(cp(cols->to, S.co.to, 8));
    CHK(cp(cols->flags, S.co.flags, 1));
    if (cols->key_hash) {
      if (!S.co.key_hash) return DRP_E_INVAL;  // not computed: drp_set_key_post(ctx, 1) first
      CHK(cp(cols->key_hash, S.co.key_hash, 8));
    }
    CHK(hipStreamSynchronize(st));
    // payload offsets relative to each piece's staging offset -> batch offsets
    for (size_t k = 0; k < S.pieces.size(); k++) {
      const uint64_t r0 = S.pieces[k].first, r1 = k + 1 < S.pieces.size() ? S.pieces[k + 1].first : ~0ull;
      const uint64_t sh = S.pieces[k].second, lo = std::max(r0, g0), hi = std::min(r1, g0 + ng);
      if (sh)
        for (uint64_t g = lo; g < hi; g++) frames->payload_off[dst + (g - g0)] += sh;
    }
  }
  c->timing.d2h_ms = (float)(now_ms() - t0);
  return DRP_OK;
}

// drp_decode_fetch_block: the staged columns' rows packed into the caller's block layout on the
// device (one launch), then one D2H of the block
struct PackSegs {
  const uint8_t *src[DRP_FETCH_COLS];
  uint64_t dst[DRP_FETCH_COLS];
  uint64_t bytes[DRP_FETCH_COLS];
  uint32_t n;
};
__global__ __launch_bounds__(256) void pack_cols_kernel(PackSegs S, uint8_t *out) {
  // bytes [i, i + 16) of the segments' concatenation (they may span several short segments)
  const uint64_t i = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 16u, e = i + 16u;
  uint64_t base = 0;
  for (uint32_t k = 0; k < S.n && base < e; k++) {
    const uint64_t end = base + S.bytes[k], lo = i > base ? i : base, hi = e < end ? e : end;
    for (uint64_t x = lo; x < hi; x++) out[S.dst[k] + (x - base)] = S.src[k][x - base];
    base = end;
  }
}

// u64 -> double in place of a column copy (DRP_FETCH_F64): dst[i] = (double)src[i]
__global__ __launch_bounds__(256) void u64_f64_kernel(const uint64_t *src, double *dst, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
    dst[i] = (double)src[i];
}

int drp_decode_fetch_block(drp_ctx *c, void *block, uint64_t block_bytes, const uint64_t *col_off, uint64_t first,
                           uint64_t rows) {
  return drp_decode_fetch_block_ex(c, block, block_bytes, col_off, first, rows, 0);
}

int drp_decode_fetch_block_ex(drp_ctx *c, void *block, uint64_t block_bytes, const uint64_t *col_off, uint64_t first,
                              uint64_t rows, uint32_t flags) {
  if (!c || (!block && block_bytes) || !col_off || (flags & ~DRP_FETCH_F64)) return DRP_E_INVAL;
  const bool f64 = flags & DRP_FETCH_F64;
  static const uint32_t W[DRP_FETCH_COLS] = {8, 4, 1, 4, 4, 4, 4, 4, 4, 8, 8, 8, 1, 8};
  const bool kh = col_off[13] != ~0ull;
  for (int k = 0; k < DRP_FETCH_COLS - (kh ? 0 : 1); k++)
    if (col_off[k] > block_bytes || rows * W[k] > block_bytes - col_off[k]) return DRP_E_INVAL;
  if (rows && is_device_ptr(block)) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  auto &S = c->staged;
  if (first > S.rows || rows > S.rows - first) return DRP_E_INVAL;
  if (kh && !S.co.key_hash) return DRP_E_INVAL;  // not computed: drp_set_key_post(ctx, 1) first
  if (!rows) return DRP_OK;
  uint8_t *B = static_cast<uint8_t *>(block);
  const double t0 = now_ms();
  const uint64_t dst = first == 0 && S.nf0 ? 1 : 0;  // (a carried blob row: set on the host below)
  const uint64_t g0 = first + dst - S.nf0, ng = rows - dst;
  if (ng) {
    if (!c->fetch_tmp.ensure(block_bytes)) return DRP_E_NOMEM;
    const void *src[DRP_FETCH_COLS] = {S.fr.payload_off, S.fr.payload_len, S.fr.type, S.co.key_off, S.co.key_len,
                                       S.co.subset_off, S.co.subset_len, S.co.value_off, S.co.value_len,
                                       S.co.change, S.co.from, S.co.to, S.co.flags, S.co.key_hash};
    if (f64) {  // the four u64 columns as doubles, converted into the space after the packed block
      if (!c->fetch_tmp.ensure(block_bytes + 4 * ng * 8 + 256)) return DRP_E_NOMEM;
      double *cv = reinterpret_cast<double *>(static_cast<uint8_t *>(c->fetch_tmp.p) + ((block_bytes + 255) & ~255ull));
      const int ks[4] = {0, 9, 10, 11};
      const uint32_t grid = (uint32_t)std::min<uint64_t>((ng + 255) / 256, 4096);
      for (int q = 0; q < 4; q++) {
        hipLaunchKernelGGL(u64_f64_kernel, dim3(grid), dim3(256), 0, c->st,
                           static_cast<const uint64_t *>(src[ks[q]]) + g0, cv + q * ng, ng);
        src[ks[q]] = cv + q * ng - g0;  // (the packing below adds g0 rows)
      }
    }
    PackSegs P = {};
    uint64_t total = 0;
    for (int k = 0; k < DRP_FETCH_COLS - (kh ? 0 : 1); k++) {
      P.src[P.n] = static_cast<const uint8_t *>(src[k]) + g0 * W[k];
      P.dst[P.n] = col_off[k] + dst * W[k];
      P.bytes[P.n] = ng * W[k];
      total += ng * W[k];
      P.n++;
    }
    const uint64_t threads = (total + 15) / 16;
    hipLaunchKernelGGL(pack_cols_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, c->st, P,
                       static_cast<uint8_t *>(c->fetch_tmp.p));
    CHK(hipGetLastError());
    CHK(hipMemcpyAsync(B, c->fetch_tmp.p, block_bytes, hipMemcpyDeviceToHost, c->st));
    CHK(hipStreamSynchronize(c->st));
    uint64_t *poff = reinterpret_cast<uint64_t *>(B + col_off[0]);
    double *poffd = reinterpret_cast<double *>(B + col_off[0]);
    for (size_t k = 0; k < S.pieces.size(); k++) {  // (as fetch_staged: piece offsets -> batch offsets)
      const uint64_t r0 = S.pieces[k].first, r1 = k + 1 < S.pieces.size() ? S.pieces[k + 1].first : ~0ull;
      const uint64_t sh = S.pieces[k].second, lo = std::max(r0, g0), hi = std::min(r1, g0 + ng);
      if (sh && f64)
        for (uint64_t g = lo; g < hi; g++) poffd[dst + (g - g0)] += (double)sh;  // (exact below 2^53)
      else if (sh)
        for (uint64_t g = lo; g < hi; g++) poff[dst + (g - g0)] += sh;
    }
  }
  if (dst) {  // (the other columns of that row are zero)
    for (int k = 3; k < DRP_FETCH_COLS - (kh ? 0 : 1); k++) memset(B + col_off[k], 0, W[k]);
    if (f64) reinterpret_cast<double *>(B + col_off[0])[0] = (double)S.off0;
    else reinterpret_cast<uint64_t *>(B + col_off[0])[0] = S.off0;
    reinterpret_cast<uint32_t *>(B + col_off[1])[0] = S.len0;
    B[col_off[2]] = S.ty0;
  }
  c->timing.d2h_ms = (float)(now_ms() - t0);
  return DRP_OK;
}

// drp_decode_fetch_keys: per row the length of its ASCII key (0 for every other row), an
// exclusive scan of those (drp_launch_tile_scan over rows: one "tile" per row), then every key
// copied from the staged bytes to its position and the positions narrowed to u32
__global__ __launch_bounds__(256) void key_len_kernel(const uint8_t *type, const uint8_t *flags, const uint32_t *kl,
                                                      uint64_t n, uint64_t *len, uint64_t *prefix) {
  const uint64_t g = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (g == 0) {
    prefix[0] = 0;
    prefix[1] = n;
  }
  if (g >= n) return;
  const bool on = (type[g] & 0x3f) == DRP_TYPE_CHANGE && (flags[g] & (DRP_F_KEY_ASCII | DRP_F_BAD)) == DRP_F_KEY_ASCII;
  len[g] = on ? kl[g] : 0u;
}
__global__ __launch_bounds__(256) void key_copy_kernel(const uint8_t *bytes, const uint64_t *poff, const uint32_t *ko,
                                                       const uint64_t *len, const uint64_t *pos, uint64_t n,
                                                       uint32_t *kp, uint8_t *text) {
  const uint64_t g = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (g >= n) return;
  const uint64_t p = pos[g], m = len[g];
  kp[g] = (uint32_t)p;  // (the text's length is checked against 256 MiB by the caller)
  const uint8_t *src = bytes + poff[g] + ko[g];
  for (uint64_t x = 0; x < m; x++) text[p + x] = src[x];
}

int drp_decode_fetch_keys(drp_ctx *c, uint64_t first, uint64_t rows, uint32_t *kp, char *text, uint64_t text_cap,
                          uint64_t *text_len) {
  if (!c || !kp || !text_len || (!text && text_cap)) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  auto &S = c->staged;
  if (first > S.rows || rows > S.rows - first) return DRP_E_INVAL;
  if (S.pieces.size() != 1 || !S.dev || c->key_post == DRP_KEY_POST_OFF) return DRP_E_INVAL;
  *text_len = 0;
  if (!rows) return DRP_OK;
  const uint64_t dst = first == 0 && S.nf0 ? 1 : 0;  // (a carried blob row: no key)
  const uint64_t g0 = first + dst - S.nf0, ng = rows - dst;
  if (dst) kp[0] = 0;
  if (!ng) return DRP_OK;
  hipStream_t st = c->st;
  // scratch: lengths, positions, the scan's tile bounds and block sums, u32 positions
  const uint64_t nb = (ng + 4095) / 4096 + 2;
  const size_t o_len = 0, o_pos = o_len + ng * 8, o_pre = o_pos + ng * 8, o_tmp = o_pre + 16, o_kp = o_tmp + nb * 8,
               o_end = o_kp + ng * 4 + 16;
  if (!c->keybuf.ensure(o_end)) return DRP_E_NOMEM;
  uint8_t *K = static_cast<uint8_t *>(c->keybuf.p);
  uint64_t *len = reinterpret_cast<uint64_t *>(K + o_len), *pos = reinterpret_cast<uint64_t *>(K + o_pos);
  uint64_t *pre = reinterpret_cast<uint64_t *>(K + o_pre), *tmp = reinterpret_cast<uint64_t *>(K + o_tmp);
  uint32_t *dkp = reinterpret_cast<uint32_t *>(K + o_kp);
  const uint32_t grid = (uint32_t)((ng + 255) / 256);
  hipLaunchKernelGGL(key_len_kernel, dim3(grid), dim3(256), 0, st, S.fr.type + g0, S.co.flags + g0, S.co.key_len + g0,
                     ng, len, pre);
  CHK(hipGetLastError());
  CHK(drp_launch_tile_scan(len, pre, 1, ng, tmp, pos, ~0ull, nullptr, st));
  // the total first (the text's size), then the text
  uint64_t total = 0;
  {
    uint64_t lastp = 0, lastl = 0;
    CHK(hipMemcpyAsync(&lastp, pos + ng - 1, 8, hipMemcpyDeviceToHost, st));
    CHK(hipMemcpyAsync(&lastl, len + ng - 1, 8, hipMemcpyDeviceToHost, st));
    CHK(hipStreamSynchronize(st));
    total = lastp + lastl;
  }
  if (!c->keytext.ensure(total + 64)) return DRP_E_NOMEM;
  uint8_t *T = static_cast<uint8_t *>(c->keytext.p);
  hipLaunchKernelGGL(key_copy_kernel, dim3(grid), dim3(256), 0, st, S.dev, S.fr.payload_off + g0, S.co.key_off + g0, len,
                     pos, ng, dkp, T);
  CHK(hipGetLastError());
  CHK(hipMemcpyAsync(kp + dst, dkp, ng * 4, hipMemcpyDeviceToHost, st));
  if (text && total && total <= text_cap) CHK(hipMemcpyAsync(text, T, total, hipMemcpyDeviceToHost, st));
  CHK(hipStreamSynchronize(st));
  *text_len = total;
  return total > text_cap && text ? DRP_E_CAPACITY : DRP_OK;
}

int drp_decode_stage(drp_ctx *c, const uint8_t *bytes, uint64_t n, drp_carry *carry, uint64_t *n_frames,
                     uint64_t *err_frame, uint32_t *err_code, uint32_t *err_detail) {
  if (!c || !carry || !n_frames || !err_frame || !err_code || !err_detail || (!bytes && n)) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  HostSrc H;
  H.flat = bytes;
  H.n = n;
  return stage_decode(c, H, carry, n_frames, err_frame, err_code, err_detail);
}

int drp_decode_stage_v(drp_ctx *c, const drp_chunk *chunks, uint64_t nchunks, drp_carry *carry, uint64_t *n_frames,
                       uint64_t *err_frame, uint32_t *err_code, uint32_t *err_detail) {
  if (!c || !carry || !n_frames || !err_frame || !err_code || !err_detail || (!chunks && nchunks)) return DRP_E_INVAL;
  HostSrc H;
  H.ch = chunks;
  H.start.resize(nchunks);
  for (uint64_t k = 0; k < nchunks; k++) {
    if (!chunks[k].bytes && chunks[k].n) return DRP_E_INVAL;
    H.start[k] = H.n;
    H.n += chunks[k].n;
  }
  if (nchunks == 1) {  // (one chunk: the flat form)
    H.flat = chunks[0].bytes;
    H.ch = nullptr;
  }
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  if (!H.n) {
    HostSrc E;
    return stage_decode(c, E, carry, n_frames, err_frame, err_code, err_detail);
  }
  return stage_decode(c, H, carry, n_frames, err_frame, err_code, err_detail);
}

int drp_decode_fetch(drp_ctx *c, const drp_frames *frames, const drp_changes *cols, uint64_t first, uint64_t rows) {
  if (!c || !frames || !cols) return DRP_E_INVAL;
  if (rows && (is_device_ptr(frames->payload_off) || is_device_ptr(cols->key_off))) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  return fetch_staged(c, frames, cols, first, rows);
}

int drp_decode_batch(drp_ctx *c, const uint8_t *bytes, uint64_t n, drp_carry *carry, const drp_frames *frames,
                     const drp_changes *cols, uint64_t cap, uint64_t *n_frames, uint64_t *err_frame,
                     uint32_t *err_code, uint32_t *err_detail) {
  if (!c || !carry || !frames || !cols || !n_frames || !err_frame || !err_code || !err_detail) return DRP_E_INVAL;
  if (!bytes && n) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  if (is_device_ptr(frames->payload_off)) return decode_batch_device_out(c, bytes, n, carry, frames, cols, cap,
                                                                         n_frames, err_frame, err_code, err_detail);
  const int key_post = c->key_post;
  if (cols->key_hash) c->key_post = DRP_KEY_POST_HASH;  // key hashes when the caller asks for them
  else if (key_post == DRP_KEY_POST_HASH) c->key_post = DRP_KEY_POST_OFF;
  HostSrc H;
  H.flat = bytes;
  H.n = n;
  c->dfr = frames;
  c->dco = cols;
  c->dcap = cap;
  c->dfetched = 0;
  int rc = stage_decode(c, H, carry, n_frames, err_frame, err_code, err_detail);
  c->dfr = nullptr;
  c->dco = nullptr;
  c->key_post = key_post;
  if (rc != DRP_OK) return rc;
  const uint64_t rows = c->staged.rows, upto = rows < cap ? rows : cap;
  rc = fetch_staged_at(c, frames, cols, c->dfetched, upto > c->dfetched ? upto - c->dfetched : 0);
  if (rc != DRP_OK) return rc;
  return rows > cap ? DRP_E_CAPACITY : DRP_OK;
}

int drp_encode_device(drp_ctx *c, const drp_change_src *src, const uint8_t *heap, uint64_t heap_bytes,
                      uint64_t n, uint64_t *frame_off, uint8_t *out, uint64_t cap) {
  if (!c || !src || !frame_off) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  const uint64_t nblk = (n + 1023) / 1024;
  const uint64_t nob = out ? drp_encode_out_blocks(cap) : 0;
  const size_t ob = al(4096 + nblk * 8 + 64), dn = al(ob + nob * 8);
  if (!c->aux.ensure(dn + nob * 4 + 64)) return DRP_E_NOMEM;
  EncodeParams P;
  P.src = *src;
  P.heap = heap;
  P.heap_bytes = heap_bytes;
  P.n = n;
  P.frame_off = frame_off;
  P.out = out;
  P.cap = cap;
  P.block_sum = c->aux.at<uint64_t>(4096);
  P.overflow = c->aux.at<uint32_t>(1024);
  P.dense_n = c->aux.at<uint32_t>(1028);
  P.oblk_first = c->aux.at<uint64_t>(ob);
  P.dense = c->aux.at<uint32_t>(dn);
  P.nob = nob;
  CHK(hipMemsetAsync(P.overflow, 0, 4, c->st));
  if (n == 0) {
    CHK(hipMemsetAsync(frame_off, 0, 8, c->st));
    return DRP_OK;
  }
  CHK(drp_launch_encode(&P, c->st));
  return DRP_OK;
}

// stage src columns (+heap) to the device if needed; returns device-side src
static int stage_src(drp_ctx *c, const drp_change_src *src, const uint8_t *heap, uint64_t heap_bytes, uint64_t n,
                     drp_change_src &dsrc, const uint8_t *&dheap) {
  if (is_device_ptr(src->key_off)) {
    dsrc = *src;
    dheap = heap;
    if (!is_device_ptr(heap) && heap_bytes) {
      if (!c->in_stage.ensure(heap_bytes)) return DRP_E_NOMEM;
      CHK(hipMemcpyAsync(c->in_stage.p, heap, heap_bytes, hipMemcpyDefault, c->st));
      dheap = (const uint8_t *)c->in_stage.p;
    }
    return DRP_OK;
  }
  const size_t need = al(heap_bytes + 16) + 10 * al(n * 8 + 8);
  if (!c->in_stage.ensure(need)) return DRP_E_NOMEM;
  size_t o = 0;
  hipError_t copy_err = hipSuccess;  // first failed staging copy, returned below
  auto put = [&](const void *h, size_t bytes) -> void * {
    void *d = c->in_stage.at<char>(o);
    o += al(bytes + 8);
    if (bytes) {
      const hipError_t e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->st);
      if (copy_err == hipSuccess) copy_err = e;
    }
    return d;
  };
  dheap = (const uint8_t *)put(heap, heap_bytes);
  dsrc.key_off = (const uint64_t *)put(src->key_off, n * 8);
  dsrc.key_len = (const uint32_t *)put(src->key_len, n * 4);
  dsrc.subset_off = (const uint64_t *)put(src->subset_off, n * 8);
  dsrc.subset_len = (const uint32_t *)put(src->subset_len, n * 4);
  dsrc.value_off = (const uint64_t *)put(src->value_off, n * 8);
  dsrc.value_len = (const uint32_t *)put(src->value_len, n * 4);
  dsrc.change = (const uint64_t *)put(src->change, n * 8);
  dsrc.from = (const uint64_t *)put(src->from, n * 8);
  dsrc.to = (const uint64_t *)put(src->to, n * 8);
  dsrc.flags = (const uint8_t *)put(src->flags, n);
  CHK(copy_err);
  CHK(hipGetLastError());
  return DRP_OK;
}

int drp_encode_size(drp_ctx *c, const drp_change_src *src, uint64_t n, uint64_t *wire_bytes) {
  if (!c || !src || !wire_bytes) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  drp_change_src dsrc;
  const uint8_t *dheap;
  int rc = stage_src(c, src, nullptr, 0, n, dsrc, dheap);
  if (rc) return rc;
  if (!c->out_stage.ensure((n + 1) * 8)) return DRP_E_NOMEM;
  uint64_t *foff = c->out_stage.at<uint64_t>(0);
  rc = drp_encode_device(c, &dsrc, dheap, ~0ull, n, foff, nullptr, ~0ull);  // sizes only: no heap read
  if (rc) return rc;
  CHK(hipMemcpyAsync(wire_bytes, foff + n, 8, hipMemcpyDeviceToHost, c->st));
  CHK(hipStreamSynchronize(c->st));
  return DRP_OK;
}

int drp_encode_batch(drp_ctx *c, const drp_change_src *src, const uint8_t *heap, uint64_t heap_bytes, uint64_t n,
                     uint8_t *out, uint64_t cap, uint64_t *written) {
  if (!c || !src || !written || (!out && cap)) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  drp_change_src dsrc;
  const uint8_t *dheap;
  int rc = stage_src(c, src, heap, heap_bytes, n, dsrc, dheap);
  if (rc) return rc;
  const bool odev = is_device_ptr(out);
  const size_t fo_bytes = al((n + 1) * 8);
  if (!c->out_stage.ensure(fo_bytes + (odev ? 0 : cap + 64))) return DRP_E_NOMEM;
  uint64_t *foff = c->out_stage.at<uint64_t>(0);
  uint8_t *dout = odev ? out : c->out_stage.at<uint8_t>(fo_bytes);
  rc = drp_encode_device(c, &dsrc, dheap, heap_bytes, n, foff, dout, cap);
  if (rc) return rc;
  uint64_t total = 0;
  CHK(hipMemcpyAsync(&total, foff + n, 8, hipMemcpyDeviceToHost, c->st));
  CHK(hipStreamSynchronize(c->st));
  if (total == ~0ull) {  // a row's key/subset/value range is outside the heap
    *written = 0;
    return DRP_E_INVAL;
  }
  *written = total;
  if (total > cap) return DRP_E_CAPACITY;
  if (!odev && total) {
    CHK(hipMemcpyAsync(out, dout, total, hipMemcpyDeviceToHost, c->st));
    CHK(hipStreamSynchronize(c->st));
  }
  return DRP_OK;
}

int drp_index_scan(drp_ctx *c, const drp_stream_stats *stats, uint64_t count, uint64_t *base) {
  if (!c || (!stats && count) || (!base && count)) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  CHK(drp_launch_index_scan(stats, count, base, c->st));
  return DRP_OK;
}

int drp_stream_stats_from_results(drp_ctx *c, const drp_stream_result *results, const uint64_t *stream_off,
                                  uint64_t nstreams, drp_stream_stats *stats) {
  if (!c || (!results && nstreams) || (!stats && nstreams)) return DRP_E_INVAL;
  if (hipSetDevice(c->device) != hipSuccess) return DRP_E_HIP;
  CHK(drp_launch_stats_from_results(results, stream_off, nstreams, stats, c->st));
  return DRP_OK;
}

}  // extern "C"

extern "C" void drp_dbg_mark(const char *name, hipStream_t st) {
  if (!dbg_on()) return;
  g_dbg.name[g_dbg.n % 64] = name;
  (void)hipEventRecord(g_dbg.ev[g_dbg.n++ % 64], st);
}
