/*
 * drp_napi.c — thin N-API addon over libdrp's C ABI (include/drp.h).
 *
 * This is the binding a maintainer adds under the reference's streaming API: the JS
 * Decoder (decode.js in this package) hands coalesced writes to decode(), which runs the
 * gfx950 frame split + Change decode and returns the frame table and Change columns; the JS
 * Encoder hands batches of Change rows to encode(). No CPU decode path exists: if libdrp or
 * the GPU is unavailable the calls fail.
 *
 * Threading: the GPU work of decode()/encode() runs on a libuv worker thread
 * (napi_async_work); the result is delivered to the callback on the JS thread, where the JS
 * layer replays the reference's callbacks. A context may be shared by several streams: its
 * calls are serialised by a mutex (one HIP stream and one scratch set per device context).
 *
 *   open(device)                                 -> ctx (external)
 *   decode(ctx, buf, blobRemaining, cb[, keyPost])
 *                                                -> cb(err, {n, errFrame, errCode, errDetail,
 *                                                   consumed, tailKind, blobRemaining, frameBytes,
 *                                                   off, len, type, ko, kl, so, sl, vo, vl,
 *                                                   change, from, to, flags[, keyHash]})
 *                                                   keyPost: also keyHash (BigUint64Array, XXH64
 *                                                   of each key) and the key flags 0x10 / 0x20
 *   decodeSync(ctx, buf, blobRemaining[, keyPost]) -> the same object (blocks the JS thread)
 *   encode(ctx, heap, n, 10 column arrays, cb)   -> cb(err, Buffer of wire bytes)
 *   deviceCount()                                -> HIP devices visible to the process
 *   indexAllgather(ctxs[], stats[])              -> {table, base}: the global frame index of
 *                                                   streams sharded over this process's devices
 *
 * Host columns are sized from the decoded frame count (drp_decode_stage, then
 * drp_decode_fetch), and handed to JS as external ArrayBuffers (no second copy).
 */
#include <node_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/drp.h"

#define NAPI_CALL(env, call)                                        \
  do {                                                              \
    if ((call) != napi_ok) {                                        \
      napi_throw_error((env), NULL, "drp addon: N-API call failed"); \
      return NULL;                                                  \
    }                                                               \
  } while (0)

typedef struct {
  drp_ctx *c;
  pthread_mutex_t mu;
} ctx_box;

static void ctx_finalize(napi_env env, void *data, void *hint) {
  (void)env;
  (void)hint;
  ctx_box *b = (ctx_box *)data;
  drp_close(b->c);
  pthread_mutex_destroy(&b->mu);
  free(b);
}

static napi_value throw_rc(napi_env env, const char *what, int rc) {
  char msg[128];
  snprintf(msg, sizeof msg, "libdrp %s failed (%d)", what, rc);
  napi_throw_error(env, NULL, msg);
  return NULL;
}

static napi_value make_error(napi_env env, const char *what, int rc) {
  char msg[128];
  snprintf(msg, sizeof msg, "libdrp %s failed (%d)", what, rc);
  napi_value m, e;
  napi_create_string_utf8(env, msg, NAPI_AUTO_LENGTH, &m);
  napi_create_error(env, NULL, m, &e);
  return e;
}

static napi_value js_open(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int32_t dev = 0;
  if (argc > 0) napi_get_value_int32(env, argv[0], &dev);
  drp_ctx *c = NULL;
  int rc = drp_open(dev, &c);
  if (rc != DRP_OK) return throw_rc(env, "open", rc);
  ctx_box *b = (ctx_box *)calloc(1, sizeof *b);
  if (!b) {
    drp_close(c);
    napi_throw_error(env, NULL, "drp addon: out of memory");
    return NULL;
  }
  b->c = c;
  pthread_mutex_init(&b->mu, NULL);
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, b, ctx_finalize, NULL, &ext));
  return ext;
}

/* ---- per-environment state ------------------------------------------------------------
 * Each Node environment (the main thread and every worker_thread) has its own pool of pinned
 * column blocks and its own communicator cache (napi_set_instance_data): nothing mutable is
 * shared between environments, so a worker's teardown cannot free what another thread uses. The
 * state lives until the environment is torn down AND every column block it handed out has been
 * released (an ArrayBuffer's finalizer may run after the environment's own), counted in `refs`. */
#define COL_KEEP 4 /* idle column blocks kept for reuse; the rest go back to the driver */

typedef struct {
  pthread_mutex_t mu; /* (decode workers take blocks off the JS thread) */
  int refs;           /* 1 for the live environment + one per block handed out */
  int closing;        /* the environment is gone: released blocks are freed, not kept */
  struct colblock *idle[COL_KEEP];
  int nidle;
  int comm_ng;
  int comm_dev[64];
  drp_comm *comm[64];
} env_state;

static void env_unref(env_state *st) {
  pthread_mutex_lock(&st->mu);
  const int last = --st->refs == 0;
  pthread_mutex_unlock(&st->mu);
  if (last) {
    pthread_mutex_destroy(&st->mu);
    free(st);
  }
}

static env_state *env_get(napi_env env) {
  void *p = NULL;
  if (napi_get_instance_data(env, &p) != napi_ok) return NULL;
  return (env_state *)p;
}

/* ---- pinned column blocks ----------------------------------------------------------------
 * The decoded columns of a batch are copied from HBM into one page-locked block (drp_host_alloc:
 * DMA at the PCIe rate, not the runtime's pageable bounce buffer) and handed to JS as external
 * ArrayBuffers over it. The block goes back to its environment's pool when the last of those
 * ArrayBuffers is collected; a batch takes the smallest idle block that fits, else a new one
 * (sized to a power of two). */
typedef struct colblock {
  env_state *st;
  void *p;
  size_t cap;
  int refs; /* (1 while a Buffer holds it) */
} colblock;

static colblock *col_get(env_state *st, size_t need) {
  colblock *b = NULL;
  pthread_mutex_lock(&st->mu);
  int best = -1;
  for (int i = 0; i < st->nidle; i++)
    if (st->idle[i]->cap >= need && (best < 0 || st->idle[i]->cap < st->idle[best]->cap)) best = i;
  if (best >= 0) {
    b = st->idle[best];
    st->idle[best] = st->idle[--st->nidle];
  }
  st->refs++; /* (the block is out) */
  pthread_mutex_unlock(&st->mu);
  if (!b) {
    size_t cap = (size_t)1 << 20;
    while (cap < need) cap <<= 1;
    void *p = NULL;
    b = (colblock *)calloc(1, sizeof *b);
    if (!b || drp_host_alloc(cap, &p) != DRP_OK) {
      free(b);
      env_unref(st);
      return NULL;
    }
    b->st = st;
    b->p = p;
    b->cap = cap;
  }
  b->refs = 0;
  return b;
}

static void col_put(colblock *b) {
  env_state *st = b->st;
  pthread_mutex_lock(&st->mu);
  colblock *drop = b;
  if (!st->closing) {
    if (st->nidle < COL_KEEP) {
      st->idle[st->nidle++] = b;
      drop = NULL;
    } else { /* (keep the larger blocks) */
      int small = 0;
      for (int i = 1; i < st->nidle; i++)
        if (st->idle[i]->cap < st->idle[small]->cap) small = i;
      if (st->idle[small]->cap < b->cap) {
        drop = st->idle[small];
        st->idle[small] = b;
      }
    }
  }
  pthread_mutex_unlock(&st->mu);
  if (drop) {
    drp_host_free(drop->p);
    free(drop);
  }
  env_unref(st);
}

/* finalizer of a batch's column Buffer (JS thread) */
static void col_finalize(napi_env env, void *data, void *hint) {
  (void)data;
  colblock *b = (colblock *)hint;
  int64_t adj;
  if (!b->st->closing) napi_adjust_external_memory(env, -(int64_t)b->cap, &adj);
  col_put(b);
}

static void comm_cache_clear(env_state *st) {
  for (int g = 0; g < st->comm_ng; g++) drp_comm_destroy(st->comm[g]);
  st->comm_ng = 0;
}

static void env_finalize(napi_env env, void *data, void *hint) {
  (void)env;
  (void)hint;
  env_state *st = (env_state *)data;
  comm_cache_clear(st);
  pthread_mutex_lock(&st->mu);
  st->closing = 1;
  while (st->nidle) {
    colblock *b = st->idle[--st->nidle];
    drp_host_free(b->p);
    free(b);
  }
  pthread_mutex_unlock(&st->mu);
  env_unref(st);
}

/* ---- decode ---------------------------------------------------------------------------- */

enum { C_OFF, C_LEN, C_TYPE, C_KO, C_KL, C_SO, C_SL, C_VO, C_VL, C_CH, C_FR, C_TO, C_FL, NCOL };
static const char *const COL_NAME[NCOL] = {"off", "len", "type", "ko", "kl", "so", "sl",
                                           "vo", "vl", "change", "from", "to", "flags"};
static const int COL_W[NCOL] = {8, 4, 1, 4, 4, 4, 4, 4, 4, 8, 8, 8, 1};
static const napi_typedarray_type COL_T[NCOL] = {
    napi_float64_array, napi_uint32_array, napi_uint8_array,   napi_uint32_array, napi_uint32_array,
    napi_uint32_array,  napi_uint32_array, napi_uint32_array,  napi_uint32_array, napi_float64_array,
    napi_float64_array, napi_float64_array, napi_uint8_array};

typedef struct {
  napi_async_work work;
  napi_ref buf_ref, cb_ref;
  ctx_box *box;
  env_state *st;
  drp_chunk *chunks; /* the batch: the written chunks end to end (one: the buffer itself) */
  uint64_t nchunks;
  drp_chunk one;
  int rc;
  uint64_t nf, ef, rows;
  uint32_t ec, ed;
  drp_carry carry;
  colblock *blk;  /* the pinned block the columns live in (NULL: the malloc'd block `mem`) */
  void *mem;
  size_t bytes;   /* the columns' block: all columns at 64-byte aligned offsets */
  void *col[NCOL];
  int key_post;   /* also the key hash column (drp_set_key_post; the key flags are always on) */
  void *khash;
  uint32_t *kp;   /* each row's key position in `keys` (rows with an ASCII key) */
  char *keys;     /* the batch's ASCII keys end to end (malloc'd; a latin1 string on the JS thread) */
  colblock *kblk; /* or those keys built on the device (drp_decode_fetch_keys) in a pinned block */
  uint64_t nkeys; /* its length; ~0: too long for one string (the JS layer decodes keys one by one) */
  int keys_done;  /* the key text (or its absence) is settled: the device built it */
  double t_h2d, t_gpu, t_d2h, t_convert; /* ms: batch to HBM, decode kernels, columns back,
                                            u64 -> Number + the key text */
  double h2d_bytes, h2d_skipped, host_copied; /* bytes staged into HBM / blob payload bytes left in host
                                                 memory / bytes gathered from the chunks on the host */
} dec_job;

static void free_cols(dec_job *j) {
  if (j->blk) col_put(j->blk); /* (never handed to JS) */
  if (j->kblk) col_put(j->kblk);
  j->kblk = NULL;
  free(j->mem);
  free(j->keys);
  j->blk = NULL;
  j->mem = NULL;
  j->keys = NULL;
  for (int i = 0; i < NCOL; i++) j->col[i] = NULL;
  j->khash = NULL;
  j->kp = NULL;
}

static void free_job(dec_job *j) {
  free_cols(j);
  if (j->chunks != &j->one) free(j->chunks);
  if (j->st) env_unref(j->st); /* (the job's reference: dec_args) */
  free(j);
}

/* the GPU part: decode, size the host columns from the frame count, fetch (worker thread) */
static double now_ms(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

static size_t al64(size_t x) { return (x + 63) & ~(size_t)63; }

/* host columns for j->rows rows in one block: pinned (the fetch then runs by DMA), else malloc */
static int alloc_cols(dec_job *j) {
  size_t need = 0;
  for (int i = 0; i < NCOL; i++) need += al64(j->rows * COL_W[i] + 8);
  need += al64(j->rows * 4 + 8);
  if (j->key_post) need += al64(j->rows * 8 + 8);
  j->bytes = need;
  j->blk = j->st ? col_get(j->st, need) : NULL;
  char *p = j->blk ? (char *)j->blk->p : (char *)(j->mem = malloc(need));
  if (!p) return DRP_E_NOMEM;
  for (int i = 0; i < NCOL; i++) {
    j->col[i] = p;
    p += al64(j->rows * COL_W[i] + 8);
  }
  j->kp = (uint32_t *)p;
  p += al64(j->rows * 4 + 8);
  if (j->key_post) j->khash = p;
  return DRP_OK;
}

/* The ASCII keys of the batch's Change rows end to end, copied from the written chunks, and
   each row's position in them: the JS thread makes one latin1 string of them and cuts every such
   key as a substring (a string per key from the chunk, toString('utf8'), costs a UTF-8 decode and
   a native call per frame; a string of the whole batch copies every byte, values included) */
#define KEYS_MAX ((uint64_t)256 << 20) /* (well below V8's string length limit) */

static int key_text(dec_job *j) {
  const double *off = (const double *)j->col[C_OFF]; /* (converted: DRP_FETCH_F64) */
  const uint32_t *ko = (const uint32_t *)j->col[C_KO], *kl = (const uint32_t *)j->col[C_KL];
  const uint8_t *ty = (const uint8_t *)j->col[C_TYPE], *fl = (const uint8_t *)j->col[C_FL];
  uint32_t *kp = j->kp;
  uint64_t tot = 0;
  for (uint64_t r = 0; r < j->rows; r++) {
    const int on = (ty[r] & 0x3f) == DRP_TYPE_CHANGE && (fl[r] & (DRP_F_KEY_ASCII | DRP_F_BAD)) == DRP_F_KEY_ASCII;
    kp[r] = (uint32_t)tot;
    tot += on ? kl[r] : 0;
    if (tot > KEYS_MAX) {
      j->nkeys = ~(uint64_t)0;
      return DRP_OK;
    }
  }
  j->nkeys = tot;
  j->keys = (char *)malloc(tot ? tot : 1);
  if (!j->keys) return DRP_E_NOMEM;
  uint64_t k = 0, s0 = 0; /* the chunk holding batch offset a, and its start */
  for (uint64_t r = 0; r < j->rows; r++) {
    if (!((ty[r] & 0x3f) == DRP_TYPE_CHANGE && (fl[r] & (DRP_F_KEY_ASCII | DRP_F_BAD)) == DRP_F_KEY_ASCII)) continue;
    uint64_t a = (uint64_t)off[r] + ko[r], n = kl[r];
    char *d = j->keys + kp[r];
    while (n) {
      while (k + 1 < j->nchunks && s0 + j->chunks[k].n <= a) s0 += j->chunks[k++].n;
      const uint64_t take = n < s0 + j->chunks[k].n - a ? n : s0 + j->chunks[k].n - a;
      memcpy(d, j->chunks[k].bytes + (a - s0), take);
      d += take;
      a += take;
      n -= take;
    }
  }
  return DRP_OK;
}

static void dec_run(dec_job *j) {
  pthread_mutex_lock(&j->box->mu);
  /* the key flags always (the JS layer cuts ASCII keys from one latin1 string of the batch),
     the key hash column when asked */
  drp_set_key_post(j->box->c, j->key_post ? DRP_KEY_POST_HASH : DRP_KEY_POST_FLAGS);
  j->rc = drp_decode_stage_v(j->box->c, j->chunks, j->nchunks, &j->carry, &j->nf, &j->ef, &j->ec, &j->ed);
  if (j->rc == DRP_OK) {
    /* rows to expose: delivered frames plus a malformed Change (its flags say why) */
    j->rows = j->nf + ((j->ec == DRP_ERR_CHANGE || j->ec == DRP_ERR_REQUIRED) ? 1 : 0);
    j->rc = alloc_cols(j);
    if (j->rc == DRP_OK) {  /* the columns' block in one transfer (its layout: alloc_cols) */
      char *base = j->blk ? (char *)j->blk->p : (char *)j->mem;
      uint64_t off[DRP_FETCH_COLS];
      for (int i = 0; i < NCOL; i++) off[i] = (uint64_t)((char *)j->col[i] - base);
      off[13] = j->khash ? (uint64_t)((char *)j->khash - base) : ~(uint64_t)0;
      /* payload_off, change, from, to as doubles (JS Numbers), converted on the device */
      j->rc = drp_decode_fetch_block_ex(j->box->c, base, j->bytes, off, 0, j->rows, DRP_FETCH_F64);
    }
    /* the key text on the device, into a pinned block (a batch staged in blob-skipping pieces has
       its earlier pieces off the device: DRP_E_INVAL, the host builds it below) */
    if (j->rc == DRP_OK && j->st && j->rows) {
      const double tk = now_ms();
      uint64_t tl = 0;
      j->kblk = col_get(j->st, (size_t)j->rows * 40 + 4096);
      int r = j->kblk ? drp_decode_fetch_keys(j->box->c, 0, j->rows, j->kp, (char *)j->kblk->p, j->kblk->cap, &tl)
                      : DRP_E_NOMEM;
      if (r == DRP_E_CAPACITY && tl <= KEYS_MAX) { /* (keys longer than the guess: once more) */
        col_put(j->kblk);
        j->kblk = col_get(j->st, (size_t)tl + 64);
        r = j->kblk ? drp_decode_fetch_keys(j->box->c, 0, j->rows, j->kp, (char *)j->kblk->p, j->kblk->cap, &tl)
                    : DRP_E_NOMEM;
      }
      if (r == DRP_OK || (r == DRP_E_CAPACITY && tl > KEYS_MAX)) {
        j->nkeys = tl > KEYS_MAX ? ~(uint64_t)0 : tl; /* (too long for one string: keys one by one) */
        if (j->nkeys == ~(uint64_t)0 && j->kblk) {
          col_put(j->kblk);
          j->kblk = NULL;
        }
        j->keys_done = 1;
      } else if (j->kblk) {
        col_put(j->kblk);
        j->kblk = NULL;
      }
      j->t_convert = now_ms() - tk;
    }
  }
  drp_timing tm;
  if (drp_last_timing(j->box->c, &tm) == DRP_OK) {
    j->t_h2d = tm.h2d_ms;
    j->h2d_bytes = (double)tm.h2d_bytes;
    j->h2d_skipped = (double)tm.h2d_skipped;
    j->host_copied = (double)tm.host_copied;
    j->t_gpu = tm.total_ms;
    j->t_d2h = tm.d2h_ms;
  }
  pthread_mutex_unlock(&j->box->mu);
  if (j->rc != DRP_OK) {
    free_cols(j);
    return;
  }
  if (j->keys_done) return; /* (the key text came from the device) */
  const double t0 = now_ms();
  if ((j->rc = key_text(j)) != DRP_OK) {
    free_cols(j);
    return;
  }
  if (j->keys) j->host_copied += (double)j->nkeys; /* (the key text is a host copy too) */
  j->t_convert = now_ms() - t0; /* (the key text; the u64 -> Number columns come converted) */
}

static void free_finalizer(napi_env env, void *data, void *hint) {
  (void)env;
  (void)hint;
  free(data);
}

static void set_num(napi_env env, napi_value obj, const char *k, double v) {
  napi_value x;
  napi_create_double(env, v, &x);
  napi_set_named_property(env, obj, k, x);
}

/* build the JS result object; the columns move into external ArrayBuffers (JS thread) */
static napi_value dec_result(napi_env env, dec_job *j) {
  napi_value res;
  if (napi_create_object(env, &res) != napi_ok) return NULL;
  set_num(env, res, "n", (double)j->nf);
  set_num(env, res, "errFrame", j->ec ? (double)j->ef : -1);
  set_num(env, res, "errCode", j->ec);
  set_num(env, res, "errDetail", j->ed);
  set_num(env, res, "consumed", (double)j->carry.consumed);
  set_num(env, res, "tailKind", j->carry.tail_kind);
  set_num(env, res, "blobRemaining", (double)j->carry.blob_remaining);
  set_num(env, res, "frameBytes", (double)j->carry.frame_bytes);
  napi_value t, kt;
  if (j->kblk && j->nkeys != ~(uint64_t)0) {
    if (napi_create_string_latin1(env, (const char *)j->kblk->p, j->nkeys, &kt) != napi_ok) return NULL;
    col_put(j->kblk);
    j->kblk = NULL;
  } else if (j->keys) {
    if (napi_create_string_latin1(env, j->keys, j->nkeys, &kt) != napi_ok) return NULL;
    free(j->keys);
    j->keys = NULL;
  } else {
    napi_get_null(env, &kt);
  }
  napi_set_named_property(env, res, "keyText", kt);
  if (napi_create_object(env, &t) == napi_ok) {
    set_num(env, t, "h2d", j->t_h2d);
    set_num(env, t, "h2dBytes", j->h2d_bytes);
    set_num(env, t, "h2dSkipped", j->h2d_skipped);
    set_num(env, t, "hostCopied", j->host_copied);
    set_num(env, t, "gpu", j->t_gpu);
    set_num(env, t, "d2h", j->t_d2h);
    set_num(env, t, "convert", j->t_convert);
    set_num(env, t, "pinnedColumns", j->blk ? 1 : 0);
    napi_set_named_property(env, res, "t", t);
  }
  /* the columns' block as one external Buffer (one finalizer returns it: a pinned block to its
     pool, a malloc'd one to the allocator) and each column a typed array over its ArrayBuffer */
  napi_value buf, ab;
  void *base = j->blk ? j->blk->p : j->mem;
  napi_status stt;
  if (j->blk) {
    stt = napi_create_external_buffer(env, j->bytes, base, col_finalize, j->blk, &buf);
    if (stt == napi_ok) {
      int64_t adj;
      napi_adjust_external_memory(env, (int64_t)j->blk->cap, &adj); /* (so V8 collects spent batches soon) */
      j->blk->refs = 1;
      j->blk = NULL; /* (the Buffer owns it now) */
    }
  } else {
    stt = napi_create_external_buffer(env, j->bytes, base, free_finalizer, NULL, &buf);
    if (stt == napi_ok) j->mem = NULL;
  }
  if (stt != napi_ok) return NULL;
  size_t blen = 0, boff = 0;
  void *bdata = NULL;
  napi_typedarray_type bty;
  if (napi_get_typedarray_info(env, buf, &bty, &blen, &bdata, &ab, &boff) != napi_ok) return NULL;
  size_t off = boff;
  for (int i = 0; i < NCOL; i++) {
    napi_value ta;
    if (napi_create_typedarray(env, COL_T[i], j->rows, ab, off, &ta) != napi_ok) return NULL;
    napi_set_named_property(env, res, COL_NAME[i], ta);
    off += al64(j->rows * COL_W[i] + 8);
  }
  napi_value kpa;
  if (napi_create_typedarray(env, napi_uint32_array, j->rows, ab, off, &kpa) != napi_ok) return NULL;
  napi_set_named_property(env, res, "kp", kpa);
  off += al64(j->rows * 4 + 8);
  if (j->khash) {
    napi_value ta;
    if (napi_create_typedarray(env, napi_biguint64_array, j->rows, ab, off, &ta) != napi_ok) return NULL;
    napi_set_named_property(env, res, "keyHash", ta);
  }
  for (int i = 0; i < NCOL; i++) j->col[i] = NULL;
  j->khash = NULL;
  j->kp = NULL;
  return res;
}

static void dec_execute(napi_env env, void *data) {
  (void)env;
  dec_run((dec_job *)data);
}

static void dec_complete(napi_env env, napi_status status, void *data) {
  dec_job *j = (dec_job *)data;
  napi_value cb, argv[2], undef;
  napi_get_reference_value(env, j->cb_ref, &cb);
  napi_get_undefined(env, &undef);
  if (status != napi_ok || j->rc != DRP_OK) {
    argv[0] = make_error(env, "decode", status != napi_ok ? DRP_E_INVAL : j->rc);
    argv[1] = undef;
  } else {
    napi_get_null(env, &argv[0]);
    argv[1] = dec_result(env, j);
    if (!argv[1]) {
      argv[0] = make_error(env, "decode (result)", DRP_E_NOMEM);
      argv[1] = undef;
    }
  }
  napi_delete_reference(env, j->buf_ref);
  napi_delete_reference(env, j->cb_ref);
  napi_delete_async_work(env, j->work);
  free_job(j);
  napi_call_function(env, undef, cb, 2, argv, NULL);
}

/* the batch argument: a Buffer, or an Array of Buffers (the written chunks, end to end) */
static int batch_chunks(napi_env env, napi_value v, dec_job *j) {
  bool arr = false;
  if (napi_is_array(env, v, &arr) != napi_ok) return 0;
  if (!arr) {
    void *bytes = NULL;
    size_t n = 0;
    if (napi_get_buffer_info(env, v, &bytes, &n) != napi_ok) return 0;
    j->one.bytes = (const uint8_t *)bytes;
    j->one.n = n;
    j->chunks = &j->one;
    j->nchunks = 1;
    return 1;
  }
  uint32_t len = 0;
  if (napi_get_array_length(env, v, &len) != napi_ok) return 0;
  j->chunks = (drp_chunk *)calloc(len ? len : 1, sizeof(drp_chunk));
  if (!j->chunks) return 0;
  j->nchunks = len;
  for (uint32_t k = 0; k < len; k++) {
    napi_value e;
    void *bytes = NULL;
    size_t n = 0;
    if (napi_get_element(env, v, k, &e) != napi_ok || napi_get_buffer_info(env, e, &bytes, &n) != napi_ok) return 0;
    j->chunks[k].bytes = (const uint8_t *)bytes;
    j->chunks[k].n = n;
  }
  return 1;
}

static dec_job *dec_args(napi_env env, napi_callback_info info, size_t want, napi_value *argv) {
  size_t argc = want + 1; /* + optional keyPost */
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < want) {
    napi_throw_type_error(env, NULL, want == 4 ? "decode(ctx, buffer | buffers, blobRemaining, cb)"
                                               : "decodeSync(ctx, buffer | buffers, blobRemaining)");
    return NULL;
  }
  dec_job *j = (dec_job *)calloc(1, sizeof *j);
  if (!j) return NULL;
  double brem = 0;
  if (napi_get_value_external(env, argv[0], (void **)&j->box) != napi_ok || !batch_chunks(env, argv[1], j) ||
      napi_get_value_double(env, argv[2], &brem) != napi_ok) {
    free_job(j);
    napi_throw_type_error(env, NULL, "decode: bad arguments");
    return NULL;
  }
  j->st = env_get(env);
  if (j->st) { /* the worker thread uses it (col_get): held until free_job, so a torn-down
                  environment (a terminated worker_thread) cannot free it under the job */
    pthread_mutex_lock(&j->st->mu);
    j->st->refs++;
    pthread_mutex_unlock(&j->st->mu);
  }
  j->carry.blob_remaining = (uint64_t)brem;
  if (argc > want) {
    bool kp = false;
    napi_get_value_bool(env, argv[want], &kp);
    j->key_post = kp;
  }
  return j;
}

static napi_value js_decode(napi_env env, napi_callback_info info) {
  napi_value argv[5];
  dec_job *j = dec_args(env, info, 4, argv);
  if (!j) return NULL;
  napi_value name;
  NAPI_CALL(env, napi_create_string_utf8(env, "drp.decode", NAPI_AUTO_LENGTH, &name));
  NAPI_CALL(env, napi_create_reference(env, argv[1], 1, &j->buf_ref)); /* keep the bytes alive */
  NAPI_CALL(env, napi_create_reference(env, argv[3], 1, &j->cb_ref));
  NAPI_CALL(env, napi_create_async_work(env, NULL, name, dec_execute, dec_complete, j, &j->work));
  NAPI_CALL(env, napi_queue_async_work(env, j->work));
  return NULL;
}

static napi_value js_decode_sync(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  dec_job *j = dec_args(env, info, 3, argv);
  if (!j) return NULL;
  dec_run(j);
  napi_value res = NULL;
  if (j->rc != DRP_OK) throw_rc(env, "decode", j->rc);
  else if (!(res = dec_result(env, j))) napi_throw_error(env, NULL, "drp addon: result allocation failed");
  free_job(j);
  return res;
}

/* ---- encode ---------------------------------------------------------------------------- */

typedef struct {
  napi_async_work work;
  napi_ref ref[12]; /* heap, 10 columns, cb */
  ctx_box *box;
  const uint8_t *heap;
  size_t heap_n;
  uint64_t n;
  void *col[10];
  int rc;
  uint8_t *out;
  uint64_t total;
} enc_job;

static void enc_execute(napi_env env, void *data) {
  (void)env;
  enc_job *j = (enc_job *)data;
  const uint64_t n = j->n;
  /* JS Numbers (Float64Array) -> u64 for heap offsets and change/from/to */
  uint64_t *u[6] = {NULL};
  const int src[6] = {0, 2, 4, 6, 7, 8};
  for (int k = 0; k < 6; k++) {
    u[k] = (uint64_t *)malloc(n * 8 + 8);
    if (!u[k]) {
      j->rc = DRP_E_NOMEM;
      goto done;
    }
    const double *d = (const double *)j->col[src[k]];
    for (uint64_t i = 0; i < n; i++) u[k][i] = (uint64_t)d[i];
  }
  {
    drp_change_src s = {u[0], j->col[1], u[1], j->col[3], u[2], j->col[5], u[3], u[4], u[5], j->col[9]};
    pthread_mutex_lock(&j->box->mu);
    j->rc = drp_encode_size(j->box->c, &s, n, &j->total);
    if (j->rc == DRP_OK) {
      j->out = (uint8_t *)malloc(j->total ? j->total : 1);
      if (!j->out) j->rc = DRP_E_NOMEM;
    }
    uint64_t written = 0;
    if (j->rc == DRP_OK) j->rc = drp_encode_batch(j->box->c, &s, j->heap, j->heap_n, n, j->out, j->total, &written);
    pthread_mutex_unlock(&j->box->mu);
    if (j->rc == DRP_OK && written != j->total) j->rc = DRP_E_INVAL; /* never expected: one kernel sizes both */
  }
done:
  for (int k = 0; k < 6; k++) free(u[k]);
  if (j->rc != DRP_OK) {
    free(j->out);
    j->out = NULL;
  }
}

static void enc_complete(napi_env env, napi_status status, void *data) {
  enc_job *j = (enc_job *)data;
  napi_value cb, argv[2], undef;
  napi_get_reference_value(env, j->ref[11], &cb);
  napi_get_undefined(env, &undef);
  argv[1] = undef;
  if (status != napi_ok || j->rc != DRP_OK) {
    argv[0] = make_error(env, "encode", status != napi_ok ? DRP_E_INVAL : j->rc);
  } else if (napi_create_external_buffer(env, j->total, j->out ? (void *)j->out : (void *)"", j->out ? free_finalizer : NULL,
                                         NULL, &argv[1]) != napi_ok) {
    argv[0] = make_error(env, "encode (result)", DRP_E_NOMEM);
    argv[1] = undef;
    free(j->out);
  } else {
    napi_get_null(env, &argv[0]);
  }
  for (int k = 0; k < 12; k++) napi_delete_reference(env, j->ref[k]);
  napi_delete_async_work(env, j->work);
  free(j);
  napi_call_function(env, undef, cb, 2, argv, NULL);
}

/* encode(ctx, heap: Buffer, n, keyOff, keyLen, subsetOff, subsetLen, valueOff, valueLen,
 *        change, from, to, flags, cb) — offsets/numbers as Float64Array, lengths Uint32Array,
 *        flags Uint8Array; cb(err, Buffer with the wire bytes of n change frames). */
static napi_value js_encode(napi_env env, napi_callback_info info) {
  size_t argc = 14;
  napi_value argv[14];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 14) {
    napi_throw_type_error(env, NULL, "encode(ctx, heap, n, 10 column arrays, cb)");
    return NULL;
  }
  enc_job *j = (enc_job *)calloc(1, sizeof *j);
  if (!j) {
    napi_throw_error(env, NULL, "drp addon: out of memory");
    return NULL;
  }
  void *heap = NULL;
  double nd = 0;
  if (napi_get_value_external(env, argv[0], (void **)&j->box) != napi_ok ||
      napi_get_buffer_info(env, argv[1], &heap, &j->heap_n) != napi_ok ||
      napi_get_value_double(env, argv[2], &nd) != napi_ok) {
    free(j);
    napi_throw_type_error(env, NULL, "encode: bad arguments");
    return NULL;
  }
  j->heap = (const uint8_t *)heap;
  j->n = (uint64_t)nd;
  for (int i = 0; i < 10; i++) {
    napi_typedarray_type t;
    size_t len, boff;
    napi_value ab;
    if (napi_get_typedarray_info(env, argv[3 + i], &t, &len, &j->col[i], &ab, &boff) != napi_ok || len < j->n) {
      free(j);
      napi_throw_range_error(env, NULL, "encode: column missing or shorter than n");
      return NULL;
    }
  }
  napi_value name;
  NAPI_CALL(env, napi_create_string_utf8(env, "drp.encode", NAPI_AUTO_LENGTH, &name));
  NAPI_CALL(env, napi_create_reference(env, argv[1], 1, &j->ref[0]));
  for (int i = 0; i < 10; i++) NAPI_CALL(env, napi_create_reference(env, argv[3 + i], 1, &j->ref[1 + i]));
  NAPI_CALL(env, napi_create_reference(env, argv[13], 1, &j->ref[11]));
  NAPI_CALL(env, napi_create_async_work(env, NULL, name, enc_execute, enc_complete, j, &j->work));
  NAPI_CALL(env, napi_queue_async_work(env, j->work));
  return NULL;
}

/* ---- devices and the multi-GPU global index ---------------------------------------------- */

static napi_value js_device_count(napi_env env, napi_callback_info info) {
  (void)info;
  int n = 0;
  drp_device_count(&n);
  napi_value v;
  NAPI_CALL(env, napi_create_int32(env, n, &v));
  return v;
}

/* indexAllgather(ctxs: [ctx per device], stats: [Float64Array(perGpu * 4) per device])
 *   -> {table: Float64Array(ngpu * perGpu * 4), base: Float64Array(ngpu * perGpu)}
 * The per-stream (frames, changes, blobs, wireBytes) records of every device, all-gathered over
 * RCCL (drp_index_allgather_host: one communicator per device of this process) and scanned into
 * the global index of each stream's first frame. Synchronous. Each ctx's mutex is held for the
 * call (its stream is the one the collective and the scan run on, and its calls are serialised:
 * native.js hands the same contexts to decoders and encoders). The communicators depend only on
 * the device list, so they are created once per device list (drp_comm_init_all) and reused. */
/* the cached communicators of this device list, created on first use (or on a new list) */
static int comms_for(env_state *st, drp_ctx **ctxs, int ng, drp_comm **out) {
  int same = st->comm_ng == ng;
  for (int g = 0; g < ng && same; g++) same = st->comm_dev[g] == drp_device(ctxs[g]);
  if (!same) {
    comm_cache_clear(st);
    int rc = drp_comm_init_all(ctxs, ng, st->comm);
    if (rc != DRP_OK) return rc;
    st->comm_ng = ng;
    for (int g = 0; g < ng; g++) st->comm_dev[g] = drp_device(ctxs[g]);
  }
  for (int g = 0; g < ng; g++) out[g] = st->comm[g];
  return DRP_OK;
}

static napi_value js_index_allgather(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  uint32_t ng = 0, ns = 0;
  bool a0 = false, a1 = false;
  if (argc < 2 || napi_is_array(env, argv[0], &a0) != napi_ok || napi_is_array(env, argv[1], &a1) != napi_ok || !a0 ||
      !a1 || napi_get_array_length(env, argv[0], &ng) != napi_ok || napi_get_array_length(env, argv[1], &ns) != napi_ok ||
      ng < 1 || ng > 64 || ns != ng) {
    napi_throw_type_error(env, NULL, "indexAllgather(ctxs[], stats[]): one ctx and one Float64Array per device");
    return NULL;
  }
  drp_ctx *ctxs[64];
  ctx_box *boxes[64] = {0};
  drp_comm *comms[64] = {0};
  drp_stream_stats *local[64] = {0};
  size_t per = 0;
  int rc = DRP_OK;
  for (uint32_t g = 0; g < ng && rc == DRP_OK; g++) {
    napi_value e, st;
    ctx_box *b = NULL;
    napi_typedarray_type ty;
    size_t len = 0, boff = 0;
    void *data = NULL;
    napi_value ab;
    if (napi_get_element(env, argv[0], g, &e) != napi_ok || napi_get_value_external(env, e, (void **)&b) != napi_ok ||
        napi_get_element(env, argv[1], g, &st) != napi_ok ||
        napi_get_typedarray_info(env, st, &ty, &len, &data, &ab, &boff) != napi_ok || ty != napi_float64_array ||
        len % 4 || (g && len / 4 != per)) {
      rc = DRP_E_INVAL;
      break;
    }
    per = len / 4;
    ctxs[g] = b->c;
    boxes[g] = b;
    local[g] = (drp_stream_stats *)malloc(per * sizeof(drp_stream_stats) + 8);
    if (!local[g]) {
      rc = DRP_E_NOMEM;
      break;
    }
    const double *d = (const double *)data;
    for (size_t i = 0; i < per; i++) {
      local[g][i].frames = (uint64_t)d[4 * i];
      local[g][i].changes = (uint64_t)d[4 * i + 1];
      local[g][i].blobs = (uint64_t)d[4 * i + 2];
      local[g][i].wire_bytes = (uint64_t)d[4 * i + 3];
    }
  }
  drp_stream_stats *global = NULL;
  uint64_t *base = NULL;
  if (rc == DRP_OK) {
    global = (drp_stream_stats *)malloc(ng * per * sizeof(drp_stream_stats) + 8);
    base = (uint64_t *)malloc(ng * per * 8 + 8);
    if (!global || !base) rc = DRP_E_NOMEM;
  }
  /* lock every ctx (in list order; a ctx listed twice is locked once): this is the only caller
     that holds more than one, and it runs on the JS thread, so the order cannot invert */
  uint32_t locked = 0;
  if (rc == DRP_OK) {
    for (; locked < ng; locked++) {
      int dup = 0;
      for (uint32_t k = 0; k < locked && !dup; k++) dup = boxes[k] == boxes[locked];
      if (!dup) pthread_mutex_lock(&boxes[locked]->mu);
    }
    env_state *st = env_get(env);
    rc = st ? comms_for(st, ctxs, (int)ng, comms) : DRP_E_INVAL;
    if (rc == DRP_OK)
      rc = drp_index_allgather_host(ctxs, comms, (int)ng, (const drp_stream_stats *const *)local, per, global, base);
    if (rc != DRP_OK && st) comm_cache_clear(st); /* (a failed collective leaves nothing cached) */
  }
  for (uint32_t g = locked; g-- > 0;) {
    int dup = 0;
    for (uint32_t k = 0; k < g && !dup; k++) dup = boxes[k] == boxes[g];
    if (!dup) pthread_mutex_unlock(&boxes[g]->mu);
  }
  for (uint32_t g = 0; g < ng; g++) free(local[g]);
  napi_value out = NULL;
  if (rc == DRP_OK) {
    napi_value tab_ab, base_ab, tab, bs;
    double *td = NULL, *bd = NULL;
    if (napi_create_object(env, &out) != napi_ok ||
        napi_create_arraybuffer(env, ng * per * 32, (void **)&td, &tab_ab) != napi_ok ||
        napi_create_arraybuffer(env, ng * per * 8, (void **)&bd, &base_ab) != napi_ok ||
        napi_create_typedarray(env, napi_float64_array, ng * per * 4, tab_ab, 0, &tab) != napi_ok ||
        napi_create_typedarray(env, napi_float64_array, ng * per, base_ab, 0, &bs) != napi_ok) {
      out = NULL;
      rc = DRP_E_NOMEM;
    } else {
      for (size_t i = 0; i < ng * per; i++) {
        td[4 * i] = (double)global[i].frames;
        td[4 * i + 1] = (double)global[i].changes;
        td[4 * i + 2] = (double)global[i].blobs;
        td[4 * i + 3] = (double)global[i].wire_bytes;
        bd[i] = (double)base[i];
      }
      napi_set_named_property(env, out, "table", tab);
      napi_set_named_property(env, out, "base", bs);
    }
  }
  free(global);
  free(base);
  if (rc != DRP_OK) return throw_rc(env, "indexAllgather", rc);
  return out;
}

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"open", NULL, js_open, NULL, NULL, NULL, napi_enumerable, NULL},
      {"decode", NULL, js_decode, NULL, NULL, NULL, napi_enumerable, NULL},
      {"decodeSync", NULL, js_decode_sync, NULL, NULL, NULL, napi_enumerable, NULL},
      {"encode", NULL, js_encode, NULL, NULL, NULL, napi_enumerable, NULL},
      {"deviceCount", NULL, js_device_count, NULL, NULL, NULL, napi_enumerable, NULL},
      {"indexAllgather", NULL, js_index_allgather, NULL, NULL, NULL, napi_enumerable, NULL},
  };
  napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
  env_state *st = (env_state *)calloc(1, sizeof *st);
  if (!st) {
    napi_throw_error(env, NULL, "drp addon: out of memory");
    return NULL;
  }
  pthread_mutex_init(&st->mu, NULL);
  st->refs = 1;
  if (napi_set_instance_data(env, st, env_finalize, NULL) != napi_ok) {
    env_unref(st);
    napi_throw_error(env, NULL, "drp addon: napi_set_instance_data failed");
    return NULL;
  }
  napi_value v;
  napi_create_int32(env, drp_abi_version(), &v);
  napi_set_named_property(env, exports, "abiVersion", v);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
