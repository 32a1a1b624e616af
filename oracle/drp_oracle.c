/*
 * drp_oracle.c — TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline).
 *
 * A plain-C, single-threaded restatement of the reference hot path of
 * mafintosh/dat-replication-protocol v4.1.2 (read-only at /root/reference):
 *
 *   - Decoder streaming state machine  decode.js:63-262 (restated: _write :124-133,
 *     _consume :144-169, _onheader :251-262, _onchangedata :216-249,
 *     _onchangeend :205-214, _onblobdata/_onblobend :171-202)
 *   - Encoder framing                  encode.js:102-137 (change + _header)
 *   - Change codec                     messages/index.js:5 over messages/schema.proto:1-8,
 *     generated at require time by protocol-buffers@^2.1.4 (package.json:27) — NOT
 *     vendored in /root/reference; its published algorithm (proto2 wire format, the
 *     generated switch-on-tag decoder, fields written in schema order) is restated here.
 *   - varint@^3.0.0 (package.json:28) — NOT vendored; LEB128 restated.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline. The product (libdrp +
 * the N-API addon) never links it.
 *
 * Pinning: see oracle/README.md and tests/test_oracle_golden.py — the codec is checked
 * against google.protobuf 7.35.1 (an independent proto2 implementation) and the
 * framing/codec against the known answers of /root/reference/test/basic.js.
 *
 * "policy" below marks inputs on which the reference is undefined, crashes or is
 * chunk-size dependent; the oracle and libdrp agree on the policy.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/drp.h"

#define ORACLE_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------- */
/* varint@3 decode restated: LEB128, res += (b & 0x7f) * 2^shift while b >= 0x80.   */
/* Policy: more than 10 bytes, or a value >= 2^64, is malformed (returns -1).       */
/* Returns bytes consumed, 0 if the buffer ends first, -1 if malformed.             */
static int vdec(const uint8_t *p, uint64_t avail, uint64_t *out) {
  uint64_t v = 0;
  for (int i = 0; i < 10; i++) {
    if ((uint64_t)i >= avail) return 0;
    uint8_t b = p[i];
    uint64_t bits = (uint64_t)(b & 0x7f);
    if (i == 9 && bits > 1) return -1; /* >= 2^64 */
    v |= bits << (7 * i);
    if (!(b & 0x80)) {
      *out = v;
      return i + 1;
    }
  }
  return -1;
}

/* varint@3 encode restated (encode.js:132-133 via varint.encode): 7 bits per byte,
 * MSB = continuation. Exact for every integer the JS Number can hold. */
static int venc(uint64_t v, uint8_t *o) {
  int n = 0;
  while (v >= 0x80) {
    o[n++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  o[n++] = (uint8_t)v;
  return n;
}
static int vlen64(uint64_t v) {
  int n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}

/* ------------------------------------------------------------------------- */
/* Change decode — restatement of the protocol-buffers@2 generated decoder for   */
/* schema.proto:1-8. Defaults: subset '', key '', numbers 0, value null. The     */
/* loop switches on tag = prefix >> 3 only (the wire type of a known tag is not  */
/* checked); unknown tags are skipped by wire type (0 varint, 1 fixed64,         */
/* 2 length-delimited, 5 fixed32; 3/4/6/7 throw). Duplicates: last wins.        */
/* Policy: a field running past the payload, a varint > 10 bytes / >= 2^53 where */
/* a JS Number is formed, a group/unknown wire type, and a missing required      */
/* field are reported as errors (DRP_ERR_CHANGE / DRP_ERR_REQUIRED).             */
typedef struct {
  uint32_t key_off, key_len, subset_off, subset_len, value_off, value_len;
  uint64_t change, from, to;
  uint8_t flags;
  uint32_t err; /* DRP_ERR_NONE / DRP_ERR_CHANGE / DRP_ERR_REQUIRED */
} oracle_change;

#define JS_SAFE (1ull << 53)

ORACLE_API int oracle_change_decode(const uint8_t *p, uint64_t len, oracle_change *c) {
  memset(c, 0, sizeof(*c));
  int found = 0; /* bit0 key, bit1 change, bit2 from, bit3 to */
  uint64_t off = 0;
  while (off < len) {
    uint64_t prefix;
    int k = vdec(p + off, len - off, &prefix);
    if (k <= 0 || prefix >= JS_SAFE) goto bad;
    off += (uint64_t)k;
    /* JS: tag = prefix >> 3 (ToInt32 then arithmetic shift); wire = prefix & 7 */
    int32_t tag = ((int32_t)(uint32_t)prefix) >> 3;
    uint32_t wire = (uint32_t)(prefix & 7);
    switch (tag) {
    case 1: case 2: case 6: { /* string / string / bytes: varint length + bytes */
      uint64_t l;
      k = vdec(p + off, len - off, &l);
      if (k <= 0 || l >= JS_SAFE) goto bad;
      off += (uint64_t)k;
      if (l > len - off) goto bad; /* policy: JS would clamp the slice */
      if (tag == 1) { c->subset_off = (uint32_t)off; c->subset_len = (uint32_t)l; c->flags |= DRP_F_SUBSET; }
      else if (tag == 2) { c->key_off = (uint32_t)off; c->key_len = (uint32_t)l; found |= 1; }
      else { c->value_off = (uint32_t)off; c->value_len = (uint32_t)l; c->flags |= DRP_F_VALUE; }
      off += l;
      break;
    }
    case 3: case 4: case 5: { /* uint32 via varint.decode: full value, no 32-bit mask */
      uint64_t v;
      k = vdec(p + off, len - off, &v);
      if (k <= 0) goto bad;
      off += (uint64_t)k;
      if (tag == 3) { c->change = v; found |= 2; }
      else if (tag == 4) { c->from = v; found |= 4; }
      else { c->to = v; found |= 8; }
      break;
    }
    default: /* skip(prefix & 7, buf, offset) */
      if (wire == 0) {
        uint64_t v;
        k = vdec(p + off, len - off, &v);
        if (k <= 0) goto bad;
        off += (uint64_t)k;
      } else if (wire == 1) {
        if (len - off < 8) goto bad;
        off += 8;
      } else if (wire == 2) {
        uint64_t l;
        k = vdec(p + off, len - off, &l);
        if (k <= 0 || l >= JS_SAFE) goto bad;
        off += (uint64_t)k;
        if (l > len - off) goto bad;
        off += l;
      } else if (wire == 5) {
        if (len - off < 4) goto bad;
        off += 4;
      } else {
        goto bad; /* groups (3/4) and wire types 6/7 throw */
      }
    }
  }
  if (found != 15) {
    c->err = DRP_ERR_REQUIRED;
    c->flags |= DRP_F_BAD | DRP_F_MISSING;
  }
  return (int)c->err;
bad:
  c->err = DRP_ERR_CHANGE;
  c->flags |= DRP_F_BAD;
  return (int)c->err;
}

/* Change encode — protocol-buffers@2 generated encoder: fields in schema order,
 * subset/value only when defined (an empty string/buffer IS defined and encoded),
 * key/change/from/to required. Returns the payload length; writes if out != NULL. */
ORACLE_API uint64_t oracle_change_encode(const uint8_t *subset, uint32_t subset_len, int has_subset,
                                         const uint8_t *key, uint32_t key_len, uint64_t change,
                                         uint64_t from, uint64_t to, const uint8_t *value,
                                         uint32_t value_len, int has_value, uint8_t *out) {
  uint64_t n = 0;
  if (has_subset) n += 1 + (uint64_t)vlen64(subset_len) + subset_len;
  n += 1 + (uint64_t)vlen64(key_len) + key_len;
  n += 1 + (uint64_t)vlen64(change) + 1 + (uint64_t)vlen64(from) + 1 + (uint64_t)vlen64(to);
  if (has_value) n += 1 + (uint64_t)vlen64(value_len) + value_len;
  if (!out) return n;
  uint8_t *o = out;
  if (has_subset) {
    *o++ = 0x0a;
    o += venc(subset_len, o);
    memcpy(o, subset, subset_len);
    o += subset_len;
  }
  *o++ = 0x12;
  o += venc(key_len, o);
  memcpy(o, key, key_len);
  o += key_len;
  *o++ = 0x18;
  o += venc(change, o);
  *o++ = 0x20;
  o += venc(from, o);
  *o++ = 0x28;
  o += venc(to, o);
  if (has_value) {
    *o++ = 0x32;
    o += venc(value_len, o);
    memcpy(o, value, value_len);
    o += value_len;
  }
  return n;
}

/* Encoder.change + Encoder._header (encode.js:102-117, 124-137) for n rows given as
 * columns with absolute heap offsets: varint(len+1), 0x01, payload. Returns bytes
 * written (or needed when out == NULL). */
ORACLE_API uint64_t oracle_encode_changes(const uint8_t *heap, uint64_t n, const uint64_t *key_off,
                                          const uint32_t *key_len, const uint64_t *subset_off,
                                          const uint32_t *subset_len, const uint64_t *value_off,
                                          const uint32_t *value_len, const uint64_t *change,
                                          const uint64_t *from, const uint64_t *to,
                                          const uint8_t *flags, uint8_t *out) {
  uint64_t w = 0;
  for (uint64_t i = 0; i < n; i++) {
    int hs = (flags[i] & DRP_F_SUBSET) != 0, hv = (flags[i] & DRP_F_VALUE) != 0;
    uint64_t plen = oracle_change_encode(heap + subset_off[i], subset_len[i], hs, heap + key_off[i],
                                         key_len[i], change[i], from[i], to[i],
                                         heap + value_off[i], value_len[i], hv, NULL);
    if (out) {
      w += (uint64_t)venc(plen + 1, out + w);
      out[w++] = DRP_TYPE_CHANGE;
      oracle_change_encode(heap + subset_off[i], subset_len[i], hs, heap + key_off[i], key_len[i],
                           change[i], from[i], to[i], heap + value_off[i], value_len[i], hv, out + w);
    } else {
      w += (uint64_t)vlen64(plen + 1) + 1;
    }
    w += plen;
  }
  return w;
}

/* Blob header of Encoder.blob(len) (encode.js:77-91): varint(len+1), 0x02. */
ORACLE_API int oracle_blob_header(uint64_t len, uint8_t *out) {
  int k = venc(len + 1, out);
  out[k] = DRP_TYPE_BLOB;
  return k + 1;
}

/* ------------------------------------------------------------------------- */
/* Streaming decoder — restatement of decode.js with synchronous callbacks.      */
/* Events are written into SoA arrays (the libdrp layout) instead of callbacks.  */
typedef struct {
  /* decode.js:75-81 */
  uint8_t header[50];
  int ptr;
  int id;
  int64_t missing;
  uint8_t *buffer; /* _buffer: partial change payload (non-fast-track) */
  uint64_t buffer_len, buffer_cap;
  int in_change_buffer; /* _buffer != null */
  int in_blob; /* _blob != null */
  /* bookkeeping for the SoA view */
  uint64_t abs;         /* absolute offset of the next byte to be written */
  uint64_t frame_start; /* absolute offset of the current frame's header */
  uint64_t payload_abs; /* absolute offset of the current frame's payload */
  uint64_t payload_len; /* L-1 */
  uint64_t blob_frame;  /* frame index of the open blob */
  /* counters decode.js:68-70 */
  uint64_t bytes, changes, blobs;
  int destroyed;
  uint32_t err_code, err_detail;
  uint64_t err_frame;
  /* outputs */
  uint64_t nframes, cap;
  uint64_t *payload_off;
  uint32_t *plen;
  uint8_t *type;
  uint32_t *key_off, *key_len, *subset_off, *subset_len, *value_off, *value_len;
  uint64_t *change, *from, *to;
  uint8_t *flags;
  int overflow; /* cap exceeded */
} oracle_dec;

static void emit_frame(oracle_dec *d, uint8_t type, uint64_t off, uint64_t len) {
  if (d->nframes >= d->cap) {
    d->overflow = 1;
    d->nframes++;
    return;
  }
  d->payload_off[d->nframes] = off;
  d->plen[d->nframes] = len > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len;
  d->type[d->nframes] = type;
  d->nframes++;
}

static void destroy(oracle_dec *d, uint32_t code, uint32_t detail) {
  /* Decoder.destroy (decode.js:104-110): no further frames are delivered. */
  if (d->destroyed) return;
  d->destroyed = 1;
  d->err_code = code;
  d->err_detail = detail;
  d->err_frame = d->nframes;
}

/* _onchangeend (decode.js:205-214): messages.Change.decode + changes++ + callback */
static void onchangeend(oracle_dec *d, const uint8_t *payload) {
  d->id = 0;
  d->ptr = 0;
  oracle_change c;
  oracle_change_decode(payload, d->payload_len, &c);
  uint64_t f = d->nframes;
  emit_frame(d, DRP_TYPE_CHANGE, d->payload_abs, d->payload_len);
  if (f < d->cap) {
    d->key_off[f] = c.key_off;
    d->key_len[f] = c.key_len;
    d->subset_off[f] = c.subset_off;
    d->subset_len[f] = c.subset_len;
    d->value_off[f] = c.value_off;
    d->value_len[f] = c.value_len;
    d->change[f] = c.change;
    d->from[f] = c.from;
    d->to[f] = c.to;
    d->flags[f] = c.flags;
  }
  d->in_change_buffer = 0;
  d->buffer_len = 0;
  if (c.err) {
    /* policy: the reference throws out of _write; we stop after the earlier frames */
    d->destroyed = 1;
    d->err_code = c.err;
    d->err_detail = 0;
    d->err_frame = f;
    return;
  }
  d->changes++;
}

/* _onheader (decode.js:251-262), with the header policy applied where the reference
 * reads the id byte. `at` = absolute offset of data[0]. Returns 1 when a header was
 * completed (the reference returns data.slice(i+1), truthy even when empty), 0 when
 * every byte went into the partial header (returns null). *used = bytes consumed. */
static int onheader(oracle_dec *d, uint64_t at, const uint8_t *data, uint64_t len, uint64_t *used) {
  for (uint64_t i = 0; i < len; i++) {
    if (d->ptr == 0) d->frame_start = at + i;
    if (d->ptr < 50) d->header[d->ptr] = data[i]; /* writes past a Buffer's end are dropped */
    d->ptr++;
    /* header[ptr-2] past index 49 is `undefined`, and undefined & 0x80 == 0 */
    if (d->ptr > 1 && (d->ptr - 2 >= 50 || !(d->header[d->ptr - 2] & 0x80))) {
      int vl = d->ptr - 1;
      uint64_t L = 0;
      uint32_t id = data[i];
      *used = i + 1;
      d->ptr = 0;
      if (vl > 10 || vdec(d->header, (uint64_t)vl, &L) != vl) { /* policy */
        destroy(d, DRP_ERR_VARINT, 0);
        return 1;
      }
      d->id = (int)id;
      d->payload_abs = at + i + 1;
      d->payload_len = L - 1;
      d->missing = (int64_t)(L - 1);
      if (id >= 3) { /* decode.js:159-161 */
        destroy(d, DRP_ERR_TYPE, id);
        return 1;
      }
      if (id != 0 && L == 0) { /* policy: _missing = -1 is chunk-size dependent */
        destroy(d, DRP_ERR_LEN, id);
        return 1;
      }
      if (id != 0 && L - 1 > (1ull << 62)) d->missing = (int64_t)(1ull << 62); /* never completes */
      return 1;
    }
  }
  *used = len;
  return 0;
}

/* _onblobdata + _onblobend (decode.js:171-202). Returns bytes consumed. */
static uint64_t onblobdata(oracle_dec *d, uint64_t len) {
  if (!d->in_blob) {
    d->blobs++;
    d->in_blob = 1;
    d->blob_frame = d->nframes;
    emit_frame(d, DRP_TYPE_BLOB, d->payload_abs, d->payload_len);
  }
  if ((int64_t)len >= d->missing) {
    uint64_t used = (uint64_t)d->missing;
    d->in_blob = 0;
    d->id = 0;
    d->ptr = 0;
    return used;
  }
  d->missing -= (int64_t)len;
  return len;
}

/* _onchangedata (decode.js:216-249). Returns bytes consumed. */
/* The reference allocates Buffer(_missing) up front (decode.js:227); the restatement grows its
 * buffer with the bytes that actually arrive, so a frame that declares a huge length and is
 * cut by EOF costs only what was received. Returns 0 when the buffer cannot grow. */
static int grow(oracle_dec *d, uint64_t need) {
  if (need <= d->buffer_cap) return 1;
  uint64_t cap = d->buffer_cap ? d->buffer_cap : 64;
  while (cap < need) cap *= 2;
  if (cap > (uint64_t)d->missing + d->buffer_len) cap = (uint64_t)d->missing + d->buffer_len;
  uint8_t *b = (uint8_t *)realloc(d->buffer, (size_t)cap);
  if (!b) return 0;
  d->buffer = b;
  d->buffer_cap = cap;
  return 1;
}

static uint64_t onchangedata(oracle_dec *d, const uint8_t *data, uint64_t len) {
  if (!d->in_change_buffer) { /* fast track: the whole payload is in this slice */
    if ((int64_t)len >= d->missing) {
      uint64_t used = (uint64_t)d->missing;
      onchangeend(d, data);
      return used;
    }
    d->in_change_buffer = 1;
    d->buffer_len = 0;
  }
  uint64_t used = (int64_t)len < d->missing ? len : (uint64_t)d->missing;
  if (!grow(d, d->buffer_len + used)) {
    destroy(d, DRP_ERR_CHANGE, 0); /* out of memory: treated as a malformed frame */
    return len;
  }
  if (used) memcpy(d->buffer + d->buffer_len, data, used);
  d->buffer_len += used;
  d->missing -= (int64_t)used;
  if (d->missing > 0) return used;
  onchangeend(d, d->buffer);
  return used;
}

/* Decoder._write + _consume (decode.js:124-133, 144-169) for one chunk, with every
 * callback acknowledged synchronously (_pending never > 0). */
static void dec_write(oracle_dec *d, const uint8_t *data, uint64_t len) {
  uint64_t base = d->abs;
  d->bytes += len;
  uint64_t off = 0;
  int have = 1; /* this._overflow is non-null */
  while (have && !d->destroyed) {
    uint64_t rest = len - off, used;
    switch (d->id) {
    case 0:
      if (rest == 0) { have = 0; break; }
      have = onheader(d, base + off, data + off, rest, &used);
      off += used;
      break;
    case 1:
      used = onchangedata(d, data + off, rest);
      have = rest > used; /* overflow = data.slice(missing) only when more bytes follow */
      off += used;
      break;
    case 2:
      used = onblobdata(d, rest);
      have = rest > used;
      off += used;
      break;
    default:
      destroy(d, DRP_ERR_TYPE, (uint32_t)d->id);
      have = 0;
    }
  }
  d->abs = base + len;
}

/* Shared body of oracle_decode_batch / oracle_decode_writes. */
static int decode_writes(const uint8_t *bytes, uint64_t n, const uint64_t *sizes, uint64_t nsizes,
                         uint64_t blob_remaining, uint64_t cap, uint64_t *payload_off,
                                   uint32_t *plen, uint8_t *type, uint32_t *key_off,
                                   uint32_t *key_len, uint32_t *subset_off, uint32_t *subset_len,
                                   uint32_t *value_off, uint32_t *value_len, uint64_t *change,
                                   uint64_t *from, uint64_t *to, uint8_t *flags,
                                   uint64_t *out /* [0]=nframes [1]=err_frame [2]=err_code
                                                    [3]=err_detail [4]=consumed [5]=tail_kind
                                                    [6]=blob_remaining [7]=changes [8]=blobs */) {
  oracle_dec d;
  memset(&d, 0, sizeof(d));
  d.cap = cap;
  d.payload_off = payload_off;
  d.plen = plen;
  d.type = type;
  d.key_off = key_off;
  d.key_len = key_len;
  d.subset_off = subset_off;
  d.subset_len = subset_len;
  d.value_off = value_off;
  d.value_len = value_len;
  d.change = change;
  d.from = from;
  d.to = to;
  d.flags = flags;
  d.err_frame = UINT64_MAX;
  if (blob_remaining) {
    /* continuation of a blob opened in an earlier batch (BlobStream already handed out) */
    d.id = 2;
    d.in_blob = 1;
    d.missing = (int64_t)blob_remaining;
    d.payload_abs = 0;
    d.payload_len = blob_remaining;
    d.blob_frame = 0;
    emit_frame(&d, DRP_TYPE_BLOB | DRP_FRAME_CONT, 0, blob_remaining);
  }
  /* one _write per piece; sizes are cycled (a 0 entry means "the rest of the batch") */
  for (uint64_t o = 0, k = 0; o < n && !d.destroyed; k++) {
    uint64_t want = sizes[k % nsizes];
    uint64_t l = (want == 0 || n - o < want) ? n - o : want;
    dec_write(&d, bytes + o, l);
    o += l;
  }
  uint64_t consumed = n, tail = DRP_TAIL_NONE, brem = 0;
  if (!d.destroyed) {
    if (d.id == 0 && d.ptr > 0) {
      tail = DRP_TAIL_HEADER;
      consumed = d.frame_start;
    } else if (d.id == 1) {
      tail = DRP_TAIL_CHANGE;
      consumed = d.frame_start;
    } else if (d.id == 2) {
      tail = DRP_TAIL_BLOB;
      brem = (uint64_t)d.missing;
      if (d.blob_frame < d.cap) d.type[d.blob_frame] |= DRP_FRAME_PARTIAL;
    }
  }
  free(d.buffer);
  uint64_t nf = d.nframes;
  if (d.err_frame != UINT64_MAX && d.err_frame < nf) nf = d.err_frame;
  out[0] = nf;
  out[1] = d.err_frame;
  out[2] = d.err_code;
  out[3] = d.err_detail;
  out[4] = consumed;
  out[5] = tail;
  out[6] = brem;
  out[7] = d.changes;
  out[8] = d.blobs;
  return d.overflow ? DRP_E_CAPACITY : DRP_OK;
}

/* Batch view used by the parity tests and the CPU baseline: feed bytes[0,n) in
 * `chunk`-byte writes (0 = one write) starting with `blob_remaining` bytes of an open
 * blob, and report SoA frames + tail exactly as drp_decode_batch does. */
ORACLE_API int oracle_decode_batch(const uint8_t *bytes, uint64_t n, uint64_t chunk,
                                   uint64_t blob_remaining, uint64_t cap, uint64_t *payload_off,
                                   uint32_t *plen, uint8_t *type, uint32_t *key_off,
                                   uint32_t *key_len, uint32_t *subset_off, uint32_t *subset_len,
                                   uint32_t *value_off, uint32_t *value_len, uint64_t *change,
                                   uint64_t *from, uint64_t *to, uint8_t *flags, uint64_t *out) {
  return decode_writes(bytes, n, &chunk, 1, blob_remaining, cap, payload_off, plen, type, key_off,
                       key_len, subset_off, subset_len, value_off, value_len, change, from, to, flags,
                       out);
}

/* The same with an explicit list of write sizes (cycled; 0 = the rest): a stream written the
 * way a fixture of the reference was (tests/golden/ref_framing.json). */
ORACLE_API int oracle_decode_writes(const uint8_t *bytes, uint64_t n, const uint64_t *sizes,
                                    uint64_t nsizes, uint64_t blob_remaining, uint64_t cap,
                                    uint64_t *payload_off, uint32_t *plen, uint8_t *type,
                                    uint32_t *key_off, uint32_t *key_len, uint32_t *subset_off,
                                    uint32_t *subset_len, uint32_t *value_off, uint32_t *value_len,
                                    uint64_t *change, uint64_t *from, uint64_t *to, uint8_t *flags,
                                    uint64_t *out) {
  if (!sizes || !nsizes) return DRP_E_INVAL;
  return decode_writes(bytes, n, sizes, nsizes, blob_remaining, cap, payload_off, plen, type,
                       key_off, key_len, subset_off, subset_len, value_off, value_len, change, from,
                       to, flags, out);
}

ORACLE_API uint64_t oracle_change_struct_size(void) { return sizeof(oracle_change); }
