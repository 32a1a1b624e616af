"""CPU checks of the region syncs' prefilters (drp_walk.hip wk_shape16 / sync_pairs136, compiled
here as host C++ from the kernel's own source text): they mark exactly the positions their
contracts say, so the syncs never miss a shaped Change header."""
import os
import random
import re
import subprocess
import tempfile

import numpy as np
import pytest

import _oracle as O
import _streams as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "dat-replication-protocol_amd", "csrc", "drp_walk.hip")

def functions(src, names):
    out = []
    for nm in names:
        m = re.search(r"^__device__ __forceinline__ \w+ " + nm + r"\(.*?^}\n", src, re.S | re.M)
        assert m, nm
        out.append(m.group(0))
    return "\n".join(out)


SHAPE_HARNESS = r"""
#include <cstdint>
#include <cstdio>
#include <cstring>
#define __device__
#define __forceinline__
%s
int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb");
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  static uint8_t *buf = new uint8_t[n + 64]();
  if (fread(buf, 1, n, f) != (size_t)n) return 1;
  for (long p = 0; p + 16 <= n; p += 16) {
    uint32_t w[5];
    memcpy(w, buf + p, 20);
    printf("%%u\n", wk_shape16(w[0], w[1], w[2], w[3], w[4]));
  }
  return 0;
}
"""


def test_shape_prefilter_is_exact():
    """wk_shape16 (drp_walk.hip; the region syncs only check the positions it marks): bit i is set
    exactly when position i starts a length varint of 1..3 bytes, then the id 1, then the tag
    0x0a or 0x12, on random bytes and on C2/C5 streams (whose every Change header is marked)."""
    src = open(SRC).read()
    code = SHAPE_HARNESS % functions(src, ["wk_shape16"])
    d = tempfile.mkdtemp()
    cpp, exe, wp = os.path.join(d, "s.cpp"), os.path.join(d, "s"), os.path.join(d, "w.bin")
    open(cpp, "w").write(code)
    subprocess.run(["g++", "-O1", "-o", exe, cpp], check=True)
    rng = random.Random(3)
    data = bytes(rng.choice([0, 1, 2, 0x0a, 0x12, 0x80, 0x85, 0xff, rng.randrange(256)]) for _ in range(60000))
    data += S.c2_stream(500).tobytes() + S.c5_stream(rng, 10)
    data = data[:len(data) // 16 * 16]
    open(wp, "wb").write(data + b"\0" * 16)
    masks = [int(x) for x in subprocess.run([exe, wp], capture_output=True, text=True, check=True).stdout.split()]

    def want(p):
        for k in (1, 2, 3):
            v = data[p:p + k]
            if len(v) < k or any(b < 0x80 for b in v[:-1]) or v[-1] >= 0x80:
                continue
            if data[p + k:p + k + 1] == b"\x01" and data[p + k + 1:p + k + 2] in (b"\x0a", b"\x12"):
                return True
        return False
    got = [(masks[p // 16] >> (p % 16)) & 1 for p in range(len(data))]
    assert got == [int(want(p)) for p in range(len(data))]
    r = O.decode_batch(S.c5_stream(random.Random(1), 1))
    assert r["nframes"] == 1


PAIRS_HARNESS = r"""
#include <cstdint>
#include <cstdio>
#include <cstring>
#define __device__
#define __forceinline__
#define __builtin_amdgcn_alignbit(a, b, s) ((uint32_t)((((uint64_t)(a) << 32) | (uint32_t)(b)) >> (s)))
%s
int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb");
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  static uint8_t *buf = new uint8_t[n + 256]();
  if (fread(buf, 1, n, f) != (size_t)n) return 1;
  for (long p = 0; p + 136 <= n; p += 8) {
    uint64_t x[17];
    memcpy(x, buf + p, sizeof x);
    printf("%%d\n", sync_pairs136(x) ? 1 : 0);
  }
  return 0;
}
"""


def test_pair_prefilter_covers_shape_candidates():
    """sync_pairs136 (drp_walk.hip) gates the exact shape masks of a 128-byte block: it passes
    exactly when a byte 0x01 at q in [0, 132) is followed by 0x0a or 0x12, so every block holding a
    shape candidate (whose id byte and first tag are such a pair) passes; random blocks rarely do."""
    src = open(SRC).read()
    code = PAIRS_HARNESS % functions(src, ["sync_pairs136"])
    d = tempfile.mkdtemp()
    cpp, exe, wp = os.path.join(d, "p.cpp"), os.path.join(d, "p"), os.path.join(d, "w.bin")
    open(cpp, "w").write(code)
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, cpp], check=True)
    rng = random.Random(5)
    data = bytes(rng.choice([0, 1, 1, 0x0a, 0x12, 0x80, 0x85, rng.randrange(256)]) for _ in range(30000))
    data += S.c2_stream(300).tobytes() + S.c5_stream(rng, 6) + bytes(rng.randrange(256) for _ in range(200000))
    open(wp, "wb").write(data)
    got = [int(x) for x in subprocess.run([exe, wp], capture_output=True, text=True, check=True).stdout.split()]

    def pair(q):
        return data[q] == 1 and data[q + 1] in (0x0a, 0x12)

    def shaped(p):
        for k in (1, 2, 3):
            v = data[p:p + k]
            if any(b < 0x80 for b in v[:-1]) or v[-1] >= 0x80:
                continue
            if data[p + k] == 1 and data[p + k + 1] in (0x0a, 0x12):
                return True
        return False
    starts = list(range(0, len(data) - 136 + 1, 8))
    assert len(got) == len(starts)
    for i, p in enumerate(starts):
        want = int(any(pair(q) for q in range(p, p + 132)))
        assert got[i] == want, p
        if any(shaped(c) for c in range(p, p + 128)):
            assert got[i] == 1, p
    tail = starts[-(200000 // 8) + 32:]  # (random bytes: ~1 block in 200 passes)
    assert sum(got[-len(tail):]) < len(tail) // 50
