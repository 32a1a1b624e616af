/*
 * drp.h — C ABI of libdrp, the MI355X (gfx950) batch codec for the
 * dat-replication-protocol hot path: varint-length-prefixed multibuffer
 * framing + protobuf `Change` decode/encode.
 *
 * Reference interface each entry point replaces (mafintosh/dat-replication-protocol v4.1.2):
 *   drp_decode_batch / drp_decode_device
 *       -> Decoder._write/_consume/_onheader/_onchangedata/_onchangeend/_onblobdata
 *          (decode.js:124-133, 144-169, 251-262, 216-249, 205-214, 179-202)
 *          + messages.Change.decode (messages/index.js:5, schema messages/schema.proto:1-8)
 *   drp_carry
 *       -> the decoder's cross-chunk state _header/_ptr/_id/_missing/_buffer/_blob
 *          (decode.js:75-81)
 *   drp_encode_size / drp_encode_batch / drp_encode_device
 *       -> Encoder.change + Encoder._header (encode.js:102-117, 124-137)
 *          + messages.Change.encode (messages/index.js:5)
 *   drp_stream_stats + drp_index_scan
 *       -> no reference counterpart (the reference is single-stream); they build the
 *          global frame index after the per-GPU stats tables are all-gathered.
 *
 * Rules: every function returns DRP_OK (0) or a negative DRP_E_* code and never
 * throws or aborts across the ABI. All buffers are caller-owned; libdrp never
 * frees caller memory and never returns heap pointers. Pointers passed to the
 * *_device entry points must be device (HBM) pointers; drp_decode_batch /
 * drp_encode_batch accept host or device pointers and stage as needed.
 * One drp_ctx per device; a ctx must not be used from two threads at once.
 */
#ifndef DRP_H
#define DRP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
/* libdrp is built with -fvisibility=hidden: the declarations below are its only exports. */
#pragma GCC visibility push(default)

#define DRP_ABI_VERSION 5

/* ---- return codes -------------------------------------------------------- */
#define DRP_OK 0
#define DRP_E_INVAL (-1)    /* bad argument */
#define DRP_E_HIP (-2)      /* HIP runtime error */
#define DRP_E_NOMEM (-3)    /* device/host allocation failed */
#define DRP_E_CAPACITY (-4) /* output capacity too small */
#define DRP_E_NODEV (-5)    /* no gfx950 device */
#define DRP_E_RETRY (-6)    /* internal: speculation failed and strict re-run also failed */
#define DRP_E_COMM (-7)     /* RCCL error (multi-GPU index) */

/* ---- frame types (the id byte, decode.js:146-161) ------------------------ */
#define DRP_TYPE_CHANGE 1
#define DRP_TYPE_BLOB 2
/* OR-ed into type[] for a blob whose payload continues past the end of the batch */
#define DRP_FRAME_PARTIAL 0x80

/* ---- per-Change flags ---------------------------------------------------- */
#define DRP_F_SUBSET 0x01 /* optional string subset = 1 present */
#define DRP_F_VALUE 0x02  /* optional bytes value = 6 present (value may be empty) */
#define DRP_F_BAD 0x04    /* payload is not a well-formed Change (see err codes) */
#define DRP_F_MISSING 0x08 /* with DRP_F_BAD: a required field (key/change/from/to) is missing */
/* key post-processing (only when drp_changes.key_hash is non-NULL / drp_set_key_post is on): */
#define DRP_F_KEY_ASCII 0x10 /* every key byte < 0x80 */
#define DRP_F_KEY_UTF8 0x20  /* the key bytes are well-formed UTF-8 (so toString('utf-8') is lossless) */

/* ---- stream error codes (first failing frame, see DESIGN.md "policy") ---- */
#define DRP_ERR_NONE 0
#define DRP_ERR_TYPE 1     /* id byte >= 3: 'Protocol error, unknown type: N' (decode.js:159-161) */
#define DRP_ERR_LEN 2      /* length varint 0 on a change/blob frame (reference is chunk-size dependent) */
#define DRP_ERR_VARINT 3   /* header varint longer than 10 bytes or >= 2^64 */
#define DRP_ERR_CHANGE 4   /* malformed Change payload (truncated field, bad wire type, huge varint) */
#define DRP_ERR_REQUIRED 5 /* Change payload lacks a required field (key/change/from/to) */

/* ---- tail kinds: what the caller must carry into the next batch ---------- */
#define DRP_TAIL_NONE 0   /* batch ended on a frame boundary */
#define DRP_TAIL_HEADER 1 /* batch ended inside a frame header: carry bytes [consumed, n) */
#define DRP_TAIL_CHANGE 2 /* batch ended inside a change payload: carry bytes [consumed, n) */
#define DRP_TAIL_BLOB 3   /* batch ended inside a blob payload: blob_remaining bytes still to come */

typedef struct drp_ctx drp_ctx;

/* Frame table, one entry per delivered frame (changes and blobs, in stream order). */
typedef struct drp_frames {
  uint64_t *payload_off; /* offset of payload byte 0 in the batch buffer */
  uint32_t *payload_len; /* declared payload length L-1 (saturates at 0xFFFFFFFF) */
  uint8_t *type;         /* DRP_TYPE_CHANGE / DRP_TYPE_BLOB (| DRP_FRAME_PARTIAL) */
} drp_frames;

/* Change columns, indexed by frame index (the entries of blob frames are unspecified: the device
 * leaves them untouched; a host fetch copies whatever the device columns held there).
 * Offsets are relative to payload_off of the same frame. */
typedef struct drp_changes {
  uint32_t *key_off, *key_len;
  uint32_t *subset_off, *subset_len;
  uint32_t *value_off, *value_len;
  uint64_t *change, *from, *to;
  uint8_t *flags;
  /* optional (NULL = not computed): XXH64 (seed 0) of the key bytes; when set, flags also get
   * DRP_F_KEY_ASCII / DRP_F_KEY_UTF8 (decode.js:210-213 builds a string of every key) */
  uint64_t *key_hash;
} drp_changes;

/* Encoder input: one Change per row; offsets are absolute into `heap`. */
typedef struct drp_change_src {
  const uint64_t *key_off;
  const uint32_t *key_len;
  const uint64_t *subset_off;
  const uint32_t *subset_len;
  const uint64_t *value_off;
  const uint32_t *value_len;
  const uint64_t *change, *from, *to;
  const uint8_t *flags; /* DRP_F_SUBSET / DRP_F_VALUE */
} drp_change_src;

/* Cross-batch carry (mirrors decode.js:75-81). The caller owns the carried bytes:
 * on return, bytes [consumed, n) of the batch must be prepended to the next batch
 * (tail HEADER/CHANGE); for tail BLOB the next batch starts with blob_remaining
 * bytes of blob payload. */
typedef struct drp_carry {
  uint64_t blob_remaining; /* in/out */
  uint64_t consumed;       /* out */
  uint32_t tail_kind;      /* out: DRP_TAIL_* */
  uint32_t reserved;
  uint64_t frame_bytes;    /* out, tail CHANGE: size of the carried frame (header + id + payload), so
                              the caller can collect exactly that many bytes once (decode.js:229-247
                              fills _buffer the same way) instead of re-sending a growing carry */
} drp_carry;

/* Per-stream result of a (multi-)stream decode. */
typedef struct drp_stream_result {
  uint64_t frame_begin;    /* index of the stream's first frame in the output columns */
  uint64_t frames;         /* delivered frames (stop before err_frame) */
  uint64_t changes;        /* delivered change frames */
  uint64_t blobs;          /* delivered blob frames (partial included) */
  uint64_t consumed;       /* stream-relative offset where the carry starts */
  uint64_t blob_remaining; /* tail BLOB: payload bytes still to come */
  uint64_t err_frame;      /* UINT64_MAX if no error, else stream-relative index of failing frame */
  uint32_t err_code;       /* DRP_ERR_* */
  uint32_t err_detail;     /* DRP_ERR_TYPE: the id byte */
  uint32_t tail_kind;      /* DRP_TAIL_* */
  uint32_t reserved;
  uint64_t tail_frame_bytes; /* tail CHANGE: header + id + payload bytes of the carried frame */
} drp_stream_result;

/* The 32-byte per-stream record exchanged by the multi-GPU all-gather. */
typedef struct drp_stream_stats {
  uint64_t frames, changes, blobs, wire_bytes;
} drp_stream_stats;

/* Timing of the last device launch sequence on a ctx (HIP events, milliseconds). */
typedef struct drp_timing {
  float decode_ms;   /* main decode kernel */
  float finalize_ms; /* per-stream finalize kernel */
  float total_ms;    /* memset + decode + finalize (+ strict re-run if any) */
  uint32_t strict_reruns; /* 1: the speculative decode fell back to the exact kernel */
  uint32_t spec_repairs;  /* verify passes that repaired failed predictions in place */
  uint32_t exact_retries; /* 1: the exact kernel's bounded look-back wait expired and it was re-run */
  uint32_t verify_relisted; /* tiles verify_lite handed to verify_counts (a re-walk or a longer look-back) */
  uint32_t seg_repairs;     /* streams whose claims the segmented repair recomputed (miss cascades) */
  uint32_t reserved;
  /* host-batch calls (drp_decode_stage / drp_decode_fetch / drp_decode_batch), wall clock: */
  float h2d_ms;   /* staging the batch into HBM */
  float d2h_ms;   /* copying the columns back (drp_decode_fetch; a pipelined batch: the rows left after its copy) */
  uint64_t h2d_bytes;   /* bytes of the last host batch staged into HBM */
  uint64_t h2d_skipped; /* its blob payload bytes never staged (pass-through, drp_set_blob_skip) */
  uint64_t host_copied; /* bytes of a chunked batch gathered on the host (drp_decode_stage_v) */
} drp_timing;

/* ---- context ------------------------------------------------------------- */
int drp_abi_version(void);
/* Number of HIP devices visible to the process (0 when none; gfx950 is checked by drp_open). */
int drp_device_count(int *n);
int drp_open(int device, drp_ctx **out);
void drp_close(drp_ctx *ctx);
/* The hipStream_t (as void*) all kernels of this ctx are launched on. */
void *drp_stream(drp_ctx *ctx);
/* The HIP device of this ctx. */
int drp_device(drp_ctx *ctx);
int drp_synchronize(drp_ctx *ctx);
int drp_last_timing(drp_ctx *ctx, drp_timing *out);
/* Tunables (0 = default 8192). tile_bytes is 4096 or 8192 (64 lanes x 64 or 128 bytes). */
int drp_set_tile(drp_ctx *ctx, uint32_t tile_bytes);
/* 1: always run the exact decode kernel (per-tile transfer functions); 0 (default): run the
 * speculate-and-verify kernel and fall back to the exact one when a prediction fails.
 * Results are identical either way; drp_timing.strict_reruns reports a fallback. */
int drp_set_exact(drp_ctx *ctx, int exact);
/* Key post-processing on every decode of the ctx (drp_keys.hip):
 * DRP_KEY_POST_HASH (1): the key hash column (drp_decode_stage: fetched when the caller's
 *   drp_changes.key_hash is non-NULL) and the key flags DRP_F_KEY_ASCII / DRP_F_KEY_UTF8;
 * DRP_KEY_POST_FLAGS (2): the key flags only (no hash column);
 * DRP_KEY_POST_OFF (0, default): neither. */
#define DRP_KEY_POST_OFF 0
#define DRP_KEY_POST_HASH 1
#define DRP_KEY_POST_FLAGS 2
int drp_set_key_post(drp_ctx *ctx, int mode);
/* Look-back composes exact inclusive exits only, never the per-tile maps agg_t. Test hook. */
int drp_set_strict(drp_ctx *ctx, int strict);
/* Host batches (drp_decode_stage / drp_decode_batch): blob payloads are pass-through ranges into
 * the caller's buffer, so their bytes need not reach HBM (decode.js:179-202 only slices them).
 * DRP_BLOB_SKIP_AUTO (default): a ctx whose last batch was mostly blob payload stages the next
 * batches in pieces, each ending a little past the next blob header (sized from the runs between
 * blobs seen so far); a piece that ends inside a blob resumes after it, skipping its payload.
 * DRP_BLOB_SKIP_ALWAYS: every host batch in pieces; DRP_BLOB_SKIP_OFF: every batch staged whole.
 * Results are identical in every mode; drp_timing.h2d_bytes / h2d_skipped report the bytes. */
#define DRP_BLOB_SKIP_OFF 0
#define DRP_BLOB_SKIP_AUTO 1
#define DRP_BLOB_SKIP_ALWAYS 2
int drp_set_blob_skip(drp_ctx *ctx, int mode);
/* Device scratch bytes needed to decode `n` bytes split into `nstreams` streams. */
uint64_t drp_decode_scratch_bytes(drp_ctx *ctx, uint64_t n, uint64_t nstreams);

/* Page-locked host memory (hipHostMalloc) for staging host batches: a batch the caller assembles
 * there is copied into HBM by DMA at the full PCIe rate instead of through the runtime's pageable
 * bounce buffer (the N-API addon coalesces small writes into such blocks). */
int drp_host_alloc(uint64_t bytes, void **out);
void drp_host_free(void *p);

/* ---- decode -------------------------------------------------------------- */
/* Decode `nstreams` independent streams laid end to end in `bytes` (device ptr, 16-byte
 * aligned, `nbytes` long).
 * stream_off[nstreams+1] (device) gives stream s = bytes[stream_off[s], stream_off[s+1]);
 * entry[nstreams] (device, may be NULL = all zero) is the stream-relative offset of the
 * first frame header (skips a blob continuation). Frames of all streams are written to
 * `frames`/`cols` (device) in stream order; per-stream results go to results[] (device).
 * Runs on drp_stream(ctx) and returns after completion (the speculation check needs the
 * result); capacity `cap` frames (DRP_E_CAPACITY if more were found). */
int drp_decode_device(drp_ctx *ctx, const uint8_t *bytes, uint64_t nbytes,
                      const uint64_t *stream_off, const uint64_t *entry, uint64_t nstreams,
                      const drp_frames *frames, const drp_changes *cols, uint64_t cap,
                      drp_stream_result *results);

/* Synchronous single-stream decode of one batch (host or device pointers).
 * carry->blob_remaining in: leading blob continuation; out: carry for the next batch.
 * Returns frames delivered in *n_frames, first failing frame in *err_frame
 * (UINT64_MAX if none) with *err_code and *err_detail. A leading blob continuation is
 * reported as frame 0 with type DRP_TYPE_BLOB|0x40 (continuation).
 * A host batch of 256 MiB or more in page-locked memory is decoded as it is copied (128 MiB DMA
 * chunks on a second stream of the ctx, one piece decoded per chunk; the rows of each piece are
 * copied into the host columns by a ctx-internal worker thread during the next chunk's copy):
 * the results are those of one whole-batch decode, and the call still returns only when every
 * row is in the columns. A ctx stays single-threaded for its callers. */
#define DRP_FRAME_CONT 0x40
int drp_decode_batch(drp_ctx *ctx, const uint8_t *bytes, uint64_t n, drp_carry *carry,
                     const drp_frames *frames, const drp_changes *cols, uint64_t cap,
                     uint64_t *n_frames, uint64_t *err_frame, uint32_t *err_code,
                     uint32_t *err_detail);

/* Two-step form of drp_decode_batch for callers that size their host columns from the
 * result (the N-API addon, which runs it on a worker thread): drp_decode_stage decodes one
 * host batch into device columns owned by the ctx (capacity grows as needed) and reports the
 * same counts, error and carry as drp_decode_batch; drp_decode_fetch then copies rows
 * [first, first + rows) into caller-owned HOST columns. Rows = *n_frames, plus one for a
 * malformed Change (DRP_ERR_CHANGE / DRP_ERR_REQUIRED: its flags say why). The staged result
 * stays valid until the next decode call on the ctx. A leading blob continuation's bytes
 * (carry->blob_remaining) are never copied to the device. */
int drp_decode_stage(drp_ctx *ctx, const uint8_t *bytes, uint64_t n, drp_carry *carry,
                     uint64_t *n_frames, uint64_t *err_frame, uint32_t *err_code, uint32_t *err_detail);
int drp_decode_fetch(drp_ctx *ctx, const drp_frames *frames, const drp_changes *cols, uint64_t first,
                     uint64_t rows);
/* drp_decode_fetch into one caller-owned HOST block [block, block + block_bytes) that libdrp may
 * write anywhere in (padding between the columns included): column k at block + col_off[k], in
 * the order payload_off, payload_len, type, key_off, key_len, subset_off, subset_len, value_off,
 * value_len, change, from, to, flags, key_hash (col_off[13] = UINT64_MAX: no key hash column).
 * The columns are packed on the device in that layout and copied in one transfer (page-locked
 * blocks: one DMA instead of one per column). Replaces the same per-frame loop as
 * drp_decode_fetch (decode.js:144-169 with messages.Change.decode). */
#define DRP_FETCH_COLS 14
int drp_decode_fetch_block(drp_ctx *ctx, void *block, uint64_t block_bytes, const uint64_t *col_off, uint64_t first,
                           uint64_t rows);
/* drp_decode_fetch_block with column forms for a JavaScript host: flags DRP_FETCH_F64 writes
 * payload_off, change, from and to as IEEE doubles (the Numbers decode.js hands out: exact below
 * 2^53, the nearest double above, as a host (double) cast rounds), converted on the device before
 * the transfer. flags 0: drp_decode_fetch_block. */
#define DRP_FETCH_F64 1u
int drp_decode_fetch_block_ex(drp_ctx *ctx, void *block, uint64_t block_bytes, const uint64_t *col_off,
                              uint64_t first, uint64_t rows, uint32_t flags);
/* The keys of the staged rows [first, first + rows) whose key the key post-processing flagged
 * ASCII (drp_set_key_post; Change rows without DRP_F_BAD), end to end: kp[r] = the text length
 * before row r (every row), text = those keys (at most text_cap bytes), *text_len = its length.
 * Built on the device from the staged batch (a JavaScript host makes one string of it and cuts
 * each key as a substring, the same string the key bytes' UTF-8 decode would give). text = NULL:
 * only kp and *text_len. DRP_E_CAPACITY: the text is longer than text_cap (kp and *text_len are
 * still written). DRP_E_INVAL when the batch was staged in more than one piece (blob skipping:
 * its earlier pieces are no longer on the device) or the keys were not flagged. Replaces the key
 * string of messages.Change.decode (decode.js:205-214). */
int drp_decode_fetch_keys(drp_ctx *ctx, uint64_t first, uint64_t rows, uint32_t *kp, char *text, uint64_t text_cap,
                          uint64_t *text_len);
/* drp_decode_stage over a batch the caller holds as chunks (its queued writes), laid end to end:
 * the caller never concatenates them. The ranges the decode stages into HBM (all of the batch,
 * or with blob skipping everything but the blob payloads) are gathered from the chunks into
 * page-locked memory of the ctx and copied by DMA; drp_timing.host_copied reports the bytes
 * gathered, so blob payloads are copied neither on the host nor to the device. Offsets in the
 * result are batch offsets (the chunks' concatenation). Replaces the per-write _consume loop's
 * input side (decode.js:144-169: each written chunk is parsed in place). */
typedef struct drp_chunk {
  const uint8_t *bytes;
  uint64_t n;
} drp_chunk;
int drp_decode_stage_v(drp_ctx *ctx, const drp_chunk *chunks, uint64_t nchunks, drp_carry *carry,
                       uint64_t *n_frames, uint64_t *err_frame, uint32_t *err_code, uint32_t *err_detail);

/* ---- encode -------------------------------------------------------------- */
/* Wire size of encoding rows [0,n) as change frames (varint(len+1) 0x01 payload). */
int drp_encode_size(drp_ctx *ctx, const drp_change_src *src, uint64_t n, uint64_t *wire_bytes);
/* Device pointers; asynchronous. frame_off[n+1] (device scratch, written) receives the
 * exclusive prefix of frame sizes (frame_off[n] = wire bytes). A row whose key/subset/value
 * range leaves [0, heap_bytes) sets frame_off[n] = UINT64_MAX and nothing is written. */
int drp_encode_device(drp_ctx *ctx, const drp_change_src *src, const uint8_t *heap, uint64_t heap_bytes,
                      uint64_t n, uint64_t *frame_off, uint8_t *out, uint64_t cap);
/* Synchronous; host or device pointers. DRP_E_INVAL if a row's range leaves the heap. */
int drp_encode_batch(drp_ctx *ctx, const drp_change_src *src, const uint8_t *heap,
                     uint64_t heap_bytes, uint64_t n, uint8_t *out, uint64_t cap,
                     uint64_t *written);

/* ---- multi-GPU global index ---------------------------------------------- */
/* stats[nranks*per_rank] (device): all-gathered per-stream tables in rank order.
 * Writes base[nranks*per_rank] (device): exclusive prefix of frames = global index of
 * each stream's first frame. Asynchronous. */
int drp_index_scan(drp_ctx *ctx, const drp_stream_stats *stats, uint64_t count, uint64_t *base);
/* results[nstreams] (device) -> stats[nstreams] (device), asynchronous. */
int drp_stream_stats_from_results(drp_ctx *ctx, const drp_stream_result *results,
                                  const uint64_t *stream_off, uint64_t nstreams,
                                  drp_stream_stats *stats);

/* ---- multi-GPU all-gather over RCCL ----------------------- */
/* The only collective of the codec: independent streams are sharded across GPUs (contiguous
 * blocks of stream ids), each GPU decodes its block (drp_decode_device) and builds its stats
 * (drp_stream_stats_from_results); the records are all-gathered (ncclAllGather over xGMI)
 * and scanned on every GPU into the global index of each stream's first frame.
 * No reference counterpart (the reference is one stream on one thread). */
#define DRP_COMM_ID_BYTES 128
typedef struct drp_comm drp_comm;
/* One process per GPU: rank 0 creates the id (ncclGetUniqueId), the launcher hands the bytes
 * to every rank, each rank joins with its ctx. */
int drp_comm_id(uint8_t *id /* [DRP_COMM_ID_BYTES] */);
int drp_comm_init_rank(drp_ctx *ctx, const uint8_t *id, int nranks, int rank, drp_comm **out);
/* One process driving ngpu devices: one comm per ctx (ncclCommInitAll). */
int drp_comm_init_all(drp_ctx **ctxs, int ngpu, drp_comm **comms);
void drp_comm_destroy(drp_comm *comm);
/* local[per_rank] -> global[nranks * per_rank] (rank order) and base[nranks * per_rank]: the
 * exclusive prefix of frames = the global index of every stream's first frame (a short block
 * is padded with zero records). Device pointers; returns after completion. */
int drp_index_allgather(drp_ctx *ctx, drp_comm *comm, const drp_stream_stats *local, uint64_t per_rank,
                        drp_stream_stats *global, uint64_t *base);
/* The same for ngpu contexts in one process (one grouped all-gather). */
int drp_index_allgather_multi(drp_ctx **ctxs, drp_comm **comms, int ngpu, const drp_stream_stats *const *local,
                              uint64_t per_gpu, drp_stream_stats *const *global, uint64_t *const *base);
/* drp_index_allgather_multi from HOST arrays (a host that keeps its per-stream counters on the
 * CPU, e.g. the N-API addon): local[g][per_gpu] are staged to device g, all-gathered over RCCL,
 * scanned on every device, and device 0's table and bases are copied to global[ngpu * per_gpu]
 * and base[ngpu * per_gpu]. Returns after completion. */
int drp_index_allgather_host(drp_ctx **ctxs, drp_comm **comms, int ngpu, const drp_stream_stats *const *local,
                             uint64_t per_gpu, drp_stream_stats *global, uint64_t *base);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif /* DRP_H */
