/*
 * sanitize_fuzz.c — TEST INFRASTRUCTURE ONLY: an AddressSanitizer + UBSan build of the oracle
 * (SURVEY §5 "Race detection / sanitizers"), driven over seeded random inputs: framed streams
 * cut at random points and written in random chunk sizes (carry, blob continuations, tails),
 * pure random bytes (every policy error path), random Change payloads through the codec, and
 * encoder rows with max-width varints. Any out-of-bounds access, use after free, leak or UB
 * aborts the run (tests/test_sanitizers.py builds and runs it: `make -C oracle fuzz`).
 *     usage: sanitize_fuzz [iterations] [seed]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/drp.h"

int oracle_decode_batch(const uint8_t *, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t *, uint32_t *, uint8_t *,
                        uint32_t *, uint32_t *, uint32_t *, uint32_t *, uint32_t *, uint32_t *, uint64_t *, uint64_t *,
                        uint64_t *, uint8_t *, uint64_t *);
int oracle_decode_writes(const uint8_t *, uint64_t, const uint64_t *, uint64_t, uint64_t, uint64_t, uint64_t *,
                         uint32_t *, uint8_t *, uint32_t *, uint32_t *, uint32_t *, uint32_t *, uint32_t *,
                         uint32_t *, uint64_t *, uint64_t *, uint64_t *, uint8_t *, uint64_t *);
uint64_t oracle_encode_changes(const uint8_t *, uint64_t, const uint64_t *, const uint32_t *, const uint64_t *,
                               const uint32_t *, const uint64_t *, const uint32_t *, const uint64_t *,
                               const uint64_t *, const uint64_t *, const uint8_t *, uint8_t *);
int oracle_blob_header(uint64_t, uint8_t *);

static uint64_t rs;
static uint64_t rnd(void) { /* xorshift64* */
  rs ^= rs >> 12;
  rs ^= rs << 25;
  rs ^= rs >> 27;
  return rs * 2685821657736338717ull;
}
static uint64_t below(uint64_t n) { return n ? rnd() % n : 0; }

typedef struct {
  uint64_t *off, *ch, *fr, *to;
  uint32_t *len, *ko, *kl, *so, *sl, *vo, *vl;
  uint8_t *ty, *fl;
  uint64_t cap;
} cols;

static void cols_alloc(cols *c, uint64_t cap) {
  c->cap = cap;
  c->off = malloc(cap * 8); c->ch = malloc(cap * 8); c->fr = malloc(cap * 8); c->to = malloc(cap * 8);
  c->len = malloc(cap * 4); c->ko = malloc(cap * 4); c->kl = malloc(cap * 4); c->so = malloc(cap * 4);
  c->sl = malloc(cap * 4); c->vo = malloc(cap * 4); c->vl = malloc(cap * 4);
  c->ty = malloc(cap); c->fl = malloc(cap);
}
static void cols_free(cols *c) {
  free(c->off); free(c->ch); free(c->fr); free(c->to); free(c->len); free(c->ko); free(c->kl);
  free(c->so); free(c->sl); free(c->vo); free(c->vl); free(c->ty); free(c->fl);
}

/* a random stream of encoded rows and blobs (+ occasional id-0 / bad headers) */
static uint64_t make_stream(uint8_t *out, uint64_t room) {
  uint64_t w = 0;
  while (w + 600 < room) {
    const uint64_t r = below(100);
    if (r < 8) { /* blob */
      uint64_t n = below(300);
      w += (uint64_t)oracle_blob_header(n, out + w);
      for (uint64_t i = 0; i < n; i++) out[w++] = (uint8_t)rnd();
    } else if (r < 10) { /* id 0 header */
      out[w++] = (uint8_t)below(0x80);
      out[w++] = 0;
    } else if (r < 11) { /* raw junk */
      uint64_t n = below(6);
      for (uint64_t i = 0; i < n; i++) out[w++] = (uint8_t)rnd();
    } else { /* one change via the encoder */
      uint8_t heap[400];
      uint32_t kl = (uint32_t)below(150), vl = (uint32_t)below(200), sl = (uint32_t)below(5);
      for (uint32_t i = 0; i < kl + vl + sl; i++) heap[i] = (uint8_t)rnd();
      uint64_t ko = 0, vo = kl, so = kl + vl;
      uint64_t num[3];
      for (int k = 0; k < 3; k++) num[k] = below(4) == 0 ? ~0ull >> below(64) : below(300);
      uint8_t fl = (uint8_t)below(4);
      w += oracle_encode_changes(heap, 1, &ko, &kl, &so, &sl, &vo, &vl, &num[0], &num[1], &num[2], &fl, out + w);
    }
  }
  return w;
}

int main(int argc, char **argv) {
  const long iters = argc > 1 ? atol(argv[1]) : 300;
  rs = argc > 2 ? strtoull(argv[2], NULL, 10) : 88172645463325252ull;
  const uint64_t room = 1 << 16;
  uint8_t *buf = malloc(room);
  cols c;
  cols_alloc(&c, room / 2 + 2);
  uint64_t meta[9], frames = 0;
  for (long it = 0; it < iters; it++) {
    uint64_t n = it % 4 == 3 ? below(room) : make_stream(buf, room);
    if (it % 4 == 3)
      for (uint64_t i = 0; i < n; i++) buf[i] = (uint8_t)rnd();
    n = below(n + 1); /* cut anywhere: tails of every kind */
    /* a private copy of exactly n bytes, so reads past the batch are caught */
    uint8_t *w = malloc(n ? n : 1);
    memcpy(w, buf, n);
    uint64_t sizes[4] = {1 + below(7), 1 + below(100), 1 + below(70000), 0};
    const uint64_t brem = below(3) == 0 ? below(n + 10) : 0;
    oracle_decode_writes(w, n, sizes, 1 + below(4), brem, c.cap, c.off, c.len, c.ty, c.ko, c.kl, c.so, c.sl,
                         c.vo, c.vl, c.ch, c.fr, c.to, c.fl, meta);
    frames += meta[0];
    oracle_decode_batch(w, n, 0, 0, 1 + below(8), c.off, c.len, c.ty, c.ko, c.kl, c.so, c.sl, c.vo, c.vl, c.ch,
                        c.fr, c.to, c.fl, meta); /* tiny capacity: the overflow path */
    free(w);
  }
  cols_free(&c);
  free(buf);
  printf("sanitize_fuzz ok: %ld iterations, %llu frames\n", iters, (unsigned long long)frames);
  return 0;
}
