"""CPU check of claims_fast's per-frame record decode (drp_decode_spec.hip crec_frame /
crec_general, compiled here as host C++ from the kernel's own source text): every Change frame it
records gets exactly the columns the oracle's Change decode (protocol-buffers@2 restated,
messages/index.js:5) gives, once expanded as emit_recs expands a record; every frame in the
record's shape is recorded; and frames in other shapes are refused (their tiles then take the
wire-reading emission, whose general decoder handles them). The GPU tests check the whole record
path (claims, verification, emit_recs) against the oracle (tests/test_gpu_configs.py,
test_gpu_decode.py with DRP_CREC=1 contexts)."""
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
SRC = os.path.join(ROOT, "dat-replication-protocol_amd", "csrc", "drp_decode_spec.hip")

HARNESS = r"""
#include <cstdint>
#include <cstdio>
#include <cstring>
#define __device__
#define __forceinline__
#define __builtin_amdgcn_alignbit(a, b, s) ((uint32_t)((((uint64_t)(a) << 32) | (uint32_t)(b)) >> (s)))
constexpr uint32_t CR_WORDS = 6;
%s
int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb");
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  static uint8_t *buf = new uint8_t[n + 256]();
  if (fread(buf, 1, n, f) != (size_t)n) return 1;
  fclose(f);
  FILE *g = fopen(argv[2], "r");
  unsigned long long o, id, tb;
  while (fscanf(g, "%%llu %%llu %%llu", &o, &id, &tb) == 3) {
    const unsigned long long base = o & ~8191ull;  // (tile-relative offsets, as on the device)
    const uint32_t *w32 = reinterpret_cast<const uint32_t *>(buf + base);
    uint32_t w[CR_WORDS];
    const bool ok = crec_frame(w32, (uint32_t)(o - base), (uint32_t)(n - base), (uint32_t)id, tb != 0, w);
    printf("%%d %%llu %%u %%u %%u %%u %%u %%u\n", ok, base, w[0], w[1], w[2], w[3], w[4], w[5]);
  }
  return 0;
}
"""


def functions(src, names):
    out = []
    for nm in names:
        m = re.search(r"^__device__ __forceinline__ \w+ " + nm + r"\(.*?^}\n", src, re.S | re.M)
        assert m, nm
        out.append(m.group(0))
    return "\n".join(out)


@pytest.fixture(scope="module")
def decoder():
    code = HARNESS % functions(open(SRC).read(), ["crec_general", "crec_frame"])
    d = tempfile.mkdtemp()
    cpp, exe = os.path.join(d, "crec.cpp"), os.path.join(d, "crec")
    open(cpp, "w").write(code)
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe, cpp], check=True)
    return exe, d


def run(decoder, wire, frames):
    exe, d = decoder
    wp, fp = os.path.join(d, "wire.bin"), os.path.join(d, "frames.txt")
    open(wp, "wb").write(wire + b"\0" * 64)
    with open(fp, "w") as f:
        for o, i, tb in frames:
            f.write(f"{o} {i} {tb}\n")
    out = subprocess.run([exe, wp, fp], capture_output=True, text=True, check=True).stdout.split("\n")
    return [list(map(int, ln.split())) for ln in out if ln]


def header_starts(r, wire):
    """Each row's header offset: its payload offset minus the id byte and the length varint."""
    out = []
    for i in range(r["nframes"]):
        po, pl = int(r["payload_off"][i]), int(r["payload_len"][i])
        for k in (1, 2, 3):
            o = po - 1 - k
            if o < 0:
                continue
            v = wire[o:o + k]
            if all(b >= 0x80 for b in v[:-1]) and v[-1] < 0x80:
                L = sum((b & 0x7F) << (7 * j) for j, b in enumerate(v))
                if L == pl + 1 or (r["type"][i] & 0x80):
                    out.append(o)
                    break
        else:
            out.append(None)  # (a length varint of 4+ bytes: never a claims_fast node)
    return out


@pytest.mark.parametrize("seed", range(4))
def test_records_match_change_decode(decoder, seed):
    rng = random.Random(seed)
    wire = S.random_stream(rng, 2500, blob_p=0.05, subset_p=0.2) + S.c2_stream(300).tobytes() + S.c5_stream(rng, 20)
    r = O.decode_batch(wire)
    hs = header_starts(r, wire)
    rows = [i for i in range(r["nframes"]) if hs[i] is not None and r["type"][i] & 0x3F in (1, 2)]
    recs = run(decoder, wire, [(hs[i], int(r["type"][i]) & 0x3F, 0) for i in rows])
    recorded = shaped = 0
    for i, (ok, base, w0, pl, w2, n0, n1, n2) in zip(rows, recs):
        ty = int(r["type"][i]) & 0x3F
        assert base + (w0 & 0x3FFF) == int(r["payload_off"][i]) and pl == int(r["payload_len"][i]), i
        assert (w0 >> 14) & 3 == ty
        if ty == 2:
            assert ok == 1
            continue
        # the record's shape: no subset, canonical order (the oracle decodes no error), numbers
        # < 2^32, a key length varint of <= 2 bytes, the field headers >= 36 bytes before the end
        fits = (max(int(r["change"][i]), int(r["from"][i]), int(r["to"][i])) < 2 ** 32 and
                int(r["flags"][i]) & 0x0D == 0 and int(r["key_len"][i]) < 2 ** 14)
        if fits:
            shaped += 1
        if not ok:
            continue
        assert fits, i
        recorded += 1
        hv = (w0 >> 17) & 1
        vo = w2 >> 16 if hv else 0
        got = {"key_off": 1 + ((w0 >> 18) & 3), "key_len": w2 & 0xFFFF, "subset_off": 0, "subset_len": 0,
               "value_off": vo, "value_len": pl - vo if hv else 0, "change": n0, "from": n1, "to": n2,
               "flags": 2 if hv else 0}
        for k, v in got.items():
            assert int(r[k][i]) == v, (i, k, int(r[k][i]), v)
    assert recorded > 800 and recorded == shaped, (recorded, shaped)


def test_records_refuse_other_shapes(decoder):
    """Payloads outside the record's shape are refused: a subset (its offsets are not recorded),
    field order, wire types, unknown fields, an empty payload, a value that does not end the payload,
    a repeated value, numbers of 2^32 or more."""
    bad = [b"", b"\x0a\x01s\x12\x01k\x18\x01\x20\x02\x28\x03", b"\x18\x01\x12\x01k\x20\x02\x28\x03",
           b"\x12\x01k\x18\x01\x20\x02", b"\x12\x01k\x18\x01\x20\x02\x28\x03\x38\x01",
           b"\x12\x01k\x18\x01\x20\x02\x28\x03\x32\x05ab", b"\x10\x01\x18\x01\x20\x02\x28\x03",
           b"\x12\x01k\x18\x01\x20\x02\x28\x03\x32\x01a\x32\x01b",
           b"\x12\x01k\x18" + S.varint(2 ** 32) + b"\x20\x02\x28\x03"]
    good = [b"\x12\x01k\x18\x01\x20\x02\x28\x03", b"\x12\x01k\x18\x01\x20\x02\x28\x03\x32\x02ab",
            b"\x12\x01k\x18" + S.varint(2 ** 32 - 1) + b"\x20" + S.varint(300) + b"\x28\x03\x32\x02ab",
            b"\x12\x81\x01" + b"k" * 129 + b"\x18\x01\x20\x02\x28\x03\x32\x90\x01" + b"v" * 144]
    wire, frames = b"", []
    for p in bad + good:
        frames.append((len(wire), 1, 0))
        wire += S.frame(p)
    wire += b"\0" * 64
    got = [ok for ok, *_ in run(decoder, wire, frames)]
    assert got == [0] * len(bad) + [1] * len(good), got


def test_partial_blob_record(decoder):
    """A blob cut by the stream end (delivered, PARTIAL) keeps its declared length."""
    wire = S.frame(b"x" * 300, 2)[:100]
    (ok, base, w0, pl, *_), = run(decoder, wire, [(0, 2, 1)])
    assert ok == 1 and (w0 >> 16) & 1 == 1 and pl == 300 and (w0 & 0x3FFF) == 3
