/*
 * drp_napi.c — thin N-API addon over libdrp's C ABI (include/drp.h).
 *
 * This is the binding a maintainer adds under the reference's streaming API: the JS
 * Decoder (decode.js in this package) hands each written chunk to decode(), which runs
 * the gfx950 frame split + Change decode and returns the frame table and Change columns;
 * the JS Encoder hands batches of Change rows to encode(). No CPU decode path exists:
 * if libdrp or the GPU is unavailable the calls throw.
 *
 *   open(device)                       -> ctx (external)
 *   decode(ctx, buf, blobRemaining)    -> {n, errFrame, errCode, errDetail, consumed,
 *                                          tailKind, blobRemaining, off, len, type, ko, kl,
 *                                          so, sl, vo, vl, change, from, to, flags}
 *   encode(ctx, heap, rows, cols...)   -> Buffer of wire bytes
 */
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/drp.h"

#define NAPI_CALL(env, call)                                        \
  do {                                                              \
    if ((call) != napi_ok) {                                        \
      napi_throw_error((env), NULL, "drp addon: N-API call failed"); \
      return NULL;                                                  \
    }                                                               \
  } while (0)

static void ctx_finalize(napi_env env, void *data, void *hint) {
  (void)env;
  (void)hint;
  drp_close((drp_ctx *)data);
}

static napi_value throw_rc(napi_env env, const char *what, int rc) {
  char msg[128];
  snprintf(msg, sizeof msg, "libdrp %s failed (%d)", what, rc);
  napi_throw_error(env, NULL, msg);
  return NULL;
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
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, c, ctx_finalize, NULL, &ext));
  return ext;
}

/* allocate an ArrayBuffer of n*size bytes and a typed array view over it */
static napi_value make_ta(napi_env env, napi_typedarray_type ty, size_t n, size_t size, void **data) {
  napi_value ab, ta;
  if (napi_create_arraybuffer(env, (n * size) != 0 ? n * size : 8, data, &ab) != napi_ok) return NULL;
  if (napi_create_typedarray(env, ty, n, ab, 0, &ta) != napi_ok) return NULL;
  return ta;
}

static void set_num(napi_env env, napi_value obj, const char *k, double v) {
  napi_value x;
  napi_create_double(env, v, &x);
  napi_set_named_property(env, obj, k, x);
}

static napi_value js_decode(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 2) {
    napi_throw_type_error(env, NULL, "decode(ctx, buffer[, blobRemaining])");
    return NULL;
  }
  drp_ctx *c = NULL;
  NAPI_CALL(env, napi_get_value_external(env, argv[0], (void **)&c));
  void *bytes = NULL;
  size_t n = 0;
  NAPI_CALL(env, napi_get_buffer_info(env, argv[1], &bytes, &n));
  double brem = 0;
  if (argc > 2) napi_get_value_double(env, argv[2], &brem);

  const uint64_t cap = n / 2 + 2; /* a delivered frame is at least 2 bytes */
  uint64_t *off = malloc(cap * 8);
  uint32_t *len = malloc(cap * 4), *ko = malloc(cap * 4), *kl = malloc(cap * 4), *so = malloc(cap * 4),
           *sl = malloc(cap * 4), *vo = malloc(cap * 4), *vl = malloc(cap * 4);
  uint64_t *ch = malloc(cap * 8), *fr = malloc(cap * 8), *to = malloc(cap * 8);
  uint8_t *ty = malloc(cap), *fl = malloc(cap);
  if (!off || !len || !ko || !kl || !so || !sl || !vo || !vl || !ch || !fr || !to || !ty || !fl) {
    napi_throw_error(env, NULL, "drp addon: out of memory");
    return NULL;
  }
  drp_frames frames = {off, len, ty};
  drp_changes cols = {ko, kl, so, sl, vo, vl, ch, fr, to, fl};
  drp_carry carry = {(uint64_t)brem, 0, 0, 0};
  uint64_t nf = 0, ef = 0;
  uint32_t ec = 0, ed = 0;
  int rc = drp_decode_batch(c, (const uint8_t *)bytes, n, &carry, &frames, &cols, cap, &nf, &ef, &ec, &ed);
  napi_value res = NULL;
  if (rc != DRP_OK) {
    throw_rc(env, "decode", rc);
    goto out;
  }
  {
    /* rows to expose: delivered frames plus a malformed Change (its flags say why) */
    uint64_t rows = nf + ((ec == DRP_ERR_CHANGE || ec == DRP_ERR_REQUIRED) ? 1 : 0);
    if (rows > cap) rows = cap;
    if (napi_create_object(env, &res) != napi_ok) goto out;
    set_num(env, res, "n", (double)nf);
    set_num(env, res, "errFrame", ec ? (double)ef : -1);
    set_num(env, res, "errCode", ec);
    set_num(env, res, "errDetail", ed);
    set_num(env, res, "consumed", (double)carry.consumed);
    set_num(env, res, "tailKind", carry.tail_kind);
    set_num(env, res, "blobRemaining", (double)carry.blob_remaining);
    struct {
      const char *k;
      napi_typedarray_type t;
      void *src;
      int w; /* 8: u64 -> f64, 4: u32, 1: u8 */
    } cs[] = {{"off", napi_float64_array, off, 8}, {"len", napi_uint32_array, len, 4},
              {"type", napi_uint8_array, ty, 1},   {"ko", napi_uint32_array, ko, 4},
              {"kl", napi_uint32_array, kl, 4},    {"so", napi_uint32_array, so, 4},
              {"sl", napi_uint32_array, sl, 4},    {"vo", napi_uint32_array, vo, 4},
              {"vl", napi_uint32_array, vl, 4},    {"change", napi_float64_array, ch, 8},
              {"from", napi_float64_array, fr, 8}, {"to", napi_float64_array, to, 8},
              {"flags", napi_uint8_array, fl, 1}};
    for (size_t i = 0; i < sizeof cs / sizeof cs[0]; i++) {
      void *d = NULL;
      napi_value ta = make_ta(env, cs[i].t, rows, cs[i].w, &d);
      if (!ta) goto out;
      if (cs[i].w == 8) {
        double *dd = d;
        const uint64_t *s = cs[i].src;
        for (uint64_t r = 0; r < rows; r++) dd[r] = (double)s[r]; /* JS Numbers, as varint.decode */
      } else if (rows) {
        memcpy(d, cs[i].src, rows * cs[i].w);
      }
      napi_set_named_property(env, res, cs[i].k, ta);
    }
  }
out:
  free(off); free(len); free(ko); free(kl); free(so); free(sl); free(vo); free(vl);
  free(ch); free(fr); free(to); free(ty); free(fl);
  return res;
}

/* encode(ctx, heap: Buffer, n, keyOff, keyLen, subsetOff, subsetLen, valueOff, valueLen,
 *        change, from, to, flags) — offsets/numbers as Float64Array, lengths Uint32Array,
 *        flags Uint8Array. Returns a Buffer with the wire bytes of n change frames. */
static napi_value js_encode(napi_env env, napi_callback_info info) {
  size_t argc = 13;
  napi_value argv[13];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 13) {
    napi_throw_type_error(env, NULL, "encode(ctx, heap, n, 10 column arrays)");
    return NULL;
  }
  drp_ctx *c = NULL;
  NAPI_CALL(env, napi_get_value_external(env, argv[0], (void **)&c));
  void *heap = NULL;
  size_t heap_n = 0;
  NAPI_CALL(env, napi_get_buffer_info(env, argv[1], &heap, &heap_n));
  double nd = 0;
  NAPI_CALL(env, napi_get_value_double(env, argv[2], &nd));
  const uint64_t n = (uint64_t)nd;
  void *col[10];
  for (int i = 0; i < 10; i++) {
    napi_typedarray_type t;
    size_t len, boff;
    napi_value ab;
    NAPI_CALL(env, napi_get_typedarray_info(env, argv[3 + i], &t, &len, &col[i], &ab, &boff));
    if (len < n) {
      napi_throw_range_error(env, NULL, "encode: column shorter than n");
      return NULL;
    }
  }
  /* JS Numbers (Float64Array) -> u64 for heap offsets and change/from/to */
  uint64_t *ko = malloc(n * 8 + 8), *so = malloc(n * 8 + 8), *vo = malloc(n * 8 + 8), *ch = malloc(n * 8 + 8),
           *fr = malloc(n * 8 + 8), *to = malloc(n * 8 + 8);
  if (!ko || !so || !vo || !ch || !fr || !to) {
    napi_throw_error(env, NULL, "drp addon: out of memory");
    free(ko); free(so); free(vo); free(ch); free(fr); free(to);
    return NULL;
  }
  for (uint64_t i = 0; i < n; i++) {
    ko[i] = (uint64_t)((double *)col[0])[i];
    so[i] = (uint64_t)((double *)col[2])[i];
    vo[i] = (uint64_t)((double *)col[4])[i];
    ch[i] = (uint64_t)((double *)col[6])[i];
    fr[i] = (uint64_t)((double *)col[7])[i];
    to[i] = (uint64_t)((double *)col[8])[i];
  }
  drp_change_src src = {ko, col[1], so, col[3], vo, col[5], ch, fr, to, col[9]};
  uint64_t total = 0;
  napi_value out = NULL;
  int rc = drp_encode_size(c, &src, n, &total);
  if (rc != DRP_OK) {
    throw_rc(env, "encode_size", rc);
    goto done;
  }
  {
    void *ob = NULL;
    if (napi_create_buffer(env, total ? total : 1, &ob, &out) != napi_ok) goto done;
    uint64_t written = 0;
    rc = drp_encode_batch(c, &src, heap, heap_n, n, ob, total, &written);
    if (rc != DRP_OK) {
      out = NULL;
      throw_rc(env, "encode", rc);
      goto done;
    }
    if (written != total) { /* never expected: both sizes come from the same kernel */
      napi_throw_error(env, NULL, "libdrp encode size mismatch");
      out = NULL;
    }
  }
done:
  free(ko); free(so); free(vo); free(ch); free(fr); free(to);
  return out;
}

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"open", NULL, js_open, NULL, NULL, NULL, napi_enumerable, NULL},
      {"decode", NULL, js_decode, NULL, NULL, NULL, napi_enumerable, NULL},
      {"encode", NULL, js_encode, NULL, NULL, NULL, napi_enumerable, NULL},
  };
  napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
  napi_value v;
  napi_create_int32(env, drp_abi_version(), &v);
  napi_set_named_property(env, exports, "abiVersion", v);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
