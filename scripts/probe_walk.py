"""Region walkers vs claims_fast on one input (measurement / debugging, GPU): decodes the same
wire with DRP_CLAIMS=walk (DRP_STATS=1: the first misses on stderr) and DRP_CLAIMS=fast, prints
each context's repair counters and compares the two decodes column by column.

    python scripts/probe_walk.py [c2|c5|multi|random] [frames]
"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _gpu  # noqa: E402,F401
import _streams as S  # noqa: E402
import drp_amd  # noqa: E402
import numpy as np  # noqa: E402


def wire_for(kind, n, seed=1):
    if kind == "c2":
        return S.c2_stream(n, seed=seed).tobytes()
    if kind == "c5":
        return S.c5_stream(random.Random(seed), n)
    if kind == "random":
        return S.random_stream(random.Random(9), n)
    raise SystemExit(kind)


def run(mode, wire, stats):
    os.environ["DRP_CLAIMS"] = mode
    os.environ["DRP_WALK_MIN"] = "0"
    if stats:
        os.environ["DRP_STATS"] = "1"
    else:
        os.environ.pop("DRP_STATS", None)
    with drp_amd.Ctx() as ctx:
        if os.environ.get("PROBE_NOSKIP"):
            ctx.set_blob_skip(drp_amd.BLOB_SKIP_OFF)
        dump = os.environ.get("PROBE_DUMP") if mode == "walk" else None
        if dump:
            os.environ["DRP_DUMP_CLAIMS"] = dump
            if os.path.exists(dump):
                os.remove(dump)
        g = ctx.decode_batch(wire)
        os.environ.pop("DRP_DUMP_CLAIMS", None)
        t = ctx.timing()
        t0 = time.time()
        g = ctx.decode_batch(wire)
        dt = time.time() - t0
        t = ctx.timing()
    print(f"{mode}: frames={g['nframes']} repairs={t.spec_repairs} relisted={t.verify_relisted} seg={t.seg_repairs} "
          f"strict={t.strict_reruns} decode_ms={t.decode_ms:.3f} wall={dt * 1e3:.1f} ms", flush=True)
    return g


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    wire = wire_for(kind, n, int(sys.argv[3]) if len(sys.argv) > 3 else 1)
    print(f"{kind}: {n} frames, {len(wire)} bytes", flush=True)
    a = run("walk", wire, True)
    b = run("fast", wire, False)
    same = all(np.array_equal(a[k], b[k]) for k in a if isinstance(a[k], np.ndarray))
    same &= all(a[k] == b[k] for k in a if not isinstance(a[k], np.ndarray))
    print("walk == fast:", same, flush=True)
    dump = os.environ.get("PROBE_DUMP")
    if dump and os.path.exists(dump):
        check_dump(wire, dump)


def true_chain(wire):
    """Frame starts of the exact chain of a single stream at offset 0 (decode.js's walk): list of
    (position, id, tail)."""
    out, p, n = [], 0, len(wire)
    while p < n:
        L, k, sh = 0, 0, 0
        while True:
            if p + k >= n:
                return out
            b = wire[p + k]
            L |= (b & 0x7F) << sh
            sh += 7
            k += 1
            if b < 0x80:
                break
        if p + k >= n:
            return out
        i = wire[p + k]
        if i > 2 or (i and L == 0):
            out.append((p, i, "err"))
            return out
        nxt = p + k + (L if i else 1)
        if i and nxt > n:
            out.append((p, i, "tail"))
            return out
        out.append((p, i, ""))
        p = nxt
    return out


def check_dump(wire, dump):
    """The walker's claims (first decode's head, DRP_DUMP_CLAIMS) against the exact chain."""
    TILE, IMG = 8192, 8192 + 512
    raw = open(dump, "rb").read()
    ntl = int(np.frombuffer(raw[:8], np.uint64)[0])
    cl = np.frombuffer(raw[8:8 + 8 * ntl], np.uint64)
    ch = true_chain(wire)
    pos = np.array([c[0] for c in ch], np.int64)
    MT, CID = 1 << 61, 1 << 62
    bad = 0
    for t in range(ntl):
        A = t * TILE
        if A + IMG > len(wire):
            continue
        i0, i1 = np.searchsorted(pos, A), np.searchsorted(pos, A + TILE)
        if i1 == i0:
            want = CID
        else:
            last = ch[i1 - 1]
            want = (MT | last[0]) if last[2] == "tail" else int(pos[i1]) if i1 < len(pos) else None
        if want is not None and int(cl[t]) != want:
            bad += 1
            if bad <= 8:
                fr = [(hex(c[0]), c[1], c[2]) for c in ch[i0:min(i1, i0 + 4)]]
                print(f"  tile {t}: claim {int(cl[t]):#x} want {want:#x} frames {i1 - i0} first {fr}", flush=True)
    print(f"dump: {bad} of {ntl} tiles differ from the exact chain", flush=True)


if __name__ == "__main__":
    main()
