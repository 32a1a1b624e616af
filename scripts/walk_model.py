"""CPU model of drp_walk.hip's sync (debugging aid): which candidate the region walker takes in
a tile, by the same rules (live mask, Change shape + next header, survival, near / far).

    python scripts/walk_model.py random 200000 147
"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _streams as S  # noqa: E402

WB, K = 128, 8


def hdr(w, p):
    x = int.from_bytes(w[p:p + 8].ljust(8, b"\0"), "little")
    tm = ~x & 0x8080808080
    if not tm:
        return 0, 0, 0xFF
    k = ((tm & -tm).bit_length() - 1) // 8 + 1
    v = 0
    for i in range(k):
        v |= (w[p + i] & 0x7F) << (7 * i)
    return k, v, (x >> (8 * k)) & 0xFF


def shape(w, po, pl):
    off, last = 0, 0
    for _ in range(6):
        if off >= pl:
            break
        b0 = w[po + off]
        fn, wt = b0 >> 3, b0 & 7
        if b0 >= 0x80 or fn < 1 or fn > 6 or fn <= last:
            return False
        num = 3 <= fn <= 5
        if wt != (0 if num else 2):
            return False
        if (fn == 3 and last < 2) or (fn > 3 and last != fn - 1):
            return False
        kb, v = 0, 0
        while True:
            b = w[po + off + 1 + kb]
            v |= (b & 0x7F) << (7 * kb)
            kb += 1
            if b < 0x80 or kb > 10:
                break
        if kb > 10 or (not num and kb > 5):
            return False
        if 1 + kb > pl - off:
            return False
        off += 1 + kb
        if not num:
            if v > pl - off:
                return False
            off += v
        last = fn
    return off == pl and last >= 5


def shaped(w, c, se):
    if c >= se:
        return False
    k, L, i = hdr(w, c)
    if k == 0 or i != 1 or L <= 1 or L - 1 > se - c - k - 1:
        return False
    if not shape(w, c + k + 1, L - 1):
        return False
    n = c + k + L
    if n >= se:
        return True
    k2, L2, i2 = hdr(w, n)
    return k2 != 0 and i2 <= 2 and (i2 == 0 or L2 != 0)


def survives(w, c, se):
    """(survives, near: every frame of the chain within the two ring windows)"""
    p, near = c, True
    for f in range(K):
        if p >= se:
            return p == se and f >= 2, near
        k, L, i = hdr(w, p)
        if k == 0 or i > 2 or (i and L == 0):
            return False, near
        if i == 0:
            p += k + 1
            continue
        if L > se - p - k:
            return f >= 2 and se - p <= 16384, near  # (SY_TAIL)
        near = near and k + L <= 2 * WB
        if i == 1 and L > 1 and w[p + k + 1] not in (0x0A, 0x12, 0x18, 0x20, 0x28, 0x32):
            return False, near
        p += k + L
    return True, near


def live(w, p):
    def ok(q):
        return w[q] < 0x80 and w[q + 1] <= 2
    return ok(p) or (w[p] >= 0x80 and (ok(p + 1) or (w[p + 1] >= 0x80 and ok(p + 2))))


def sync_tile(w, A, se, verbose=True):
    """The walker's choice in the tile at A (TILE 8192), scanning window by window."""
    far = None
    for q in range(64):
        W0 = A + q * WB
        if far and far[1] < W0 + WB:
            return ("far-taken", far)
        for o in range(0, WB + 112):
            c = W0 + o
            if far and c >= far[1]:
                if far[1] - far[0] <= 2 * WB and shaped(w, far[1], se):
                    return ("far-successor", far[1])
                break
            if not live(w, c):
                continue
            k, L, i = hdr(w, c)
            if k == 0 or i > 2 or (i and L == 0):
                continue
            sh = shaped(w, c, se)
            sv, near = (False, False) if sh else survives(w, c, se)
            if verbose and (sh or sv):
                print(f"  q={q} o={o} c={c:#x} k={k} L={L} id={i} shape={sh} survives={sv}")
            if not sh and not sv:
                continue
            if sh or near:
                n1 = c + k + (L if i else 1)
                if not sh and n1 < W0 + WB + 112 and shaped(w, n1, se):
                    return ("taken-next", n1)
                return ("taken", c)
            if not far and o < WB:
                far = (c, c + k + L)
    return ("far-at-end", far)


def main():
    kind, n, t = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    w = S.random_stream(random.Random(9), n) if kind == "random" else S.c2_stream(n).tobytes()
    print(sync_tile(w, t * 8192, len(w)))


if __name__ == "__main__":
    main()
