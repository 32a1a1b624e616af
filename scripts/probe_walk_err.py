"""Debugging aid (GPU): test_gpu_walk.py::test_errors_and_tails[0]'s b'\\x01\\x01' case through the
region walkers and through claims_fast, with the walkers' claims dumped and compared to the exact
chain (scripts/probe_walk.py's check)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import _gpu  # noqa: E402,F401
import _oracle as O  # noqa: E402
import _streams as S  # noqa: E402
import drp_amd  # noqa: E402
import numpy as np  # noqa: E402
from probe_walk import check_dump  # noqa: E402


def main():
    rng = random.Random(200)
    base = S.random_stream(rng, 3000)
    wires = []
    for b in [b"\x03\x07ab", b"\x00\x01", b"\x80" * 10 + b"\x01\x01", b"\x01\x01", S.frame(b"\x12\x05k")]:
        cut = O.decode_batch(base[:rng.randint(0, len(base))])["consumed"]
        wires.append((b, base[:cut] + b + base, cut))
    for b, wire, cut in wires:
        r = O.decode_batch(wire)
        out = {}
        for mode in ["walk", "fast"]:
            os.environ.update({"DRP_CLAIMS": mode, "DRP_WALK_MIN": "0", "DRP_STATS": "1"})
            with drp_amd.Ctx(0) as c:
                c.set_blob_skip(0)
                if mode == "walk":
                    os.environ["DRP_DUMP_CLAIMS"] = "/tmp/err_dump.bin"
                    if os.path.exists("/tmp/err_dump.bin"):
                        os.remove("/tmp/err_dump.bin")
                g = c.decode_batch(wire)
                os.environ.pop("DRP_DUMP_CLAIMS", None)
                t = c.timing()
            out[mode] = g
            print(f"{b!r} cut {cut} {mode}: nframes {g['nframes']} err {g['err_code']}/{g['err_frame']} "
                  f"(oracle {r['nframes']} {r['err_code']}/{r['err_frame']}) repairs {t.spec_repairs} "
                  f"relisted {t.verify_relisted}", flush=True)
        if os.path.exists("/tmp/err_dump.bin"):
            check_dump(wire, "/tmp/err_dump.bin")
        a, f = out["walk"], out["fast"]
        n = min(a["nframes"], f["nframes"])
        for k in ["payload_off", "payload_len", "type", "flags"]:
            d = np.flatnonzero(a[k][:n] != f[k][:n])
            if d.size:
                print(f"  {k}: {d.size} rows differ, first {d[0]}: walk {a[k][d[0]]} fast {f[k][d[0]]}", flush=True)


if __name__ == "__main__":
    main()
