"""Debugging aid (GPU): the claims of a short C5 batch (a 64 KiB blob-skip piece) by the region
walkers and by claims_fast, tile by tile (DRP_DUMP_CLAIMS), with each mode's repair counters."""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _gpu  # noqa: E402,F401
import _streams as S  # noqa: E402
import drp_amd  # noqa: E402


def main():
    wire = S.c5_stream(random.Random(5), 40)
    for size in (65536, 131072, 200000):
        w = wire[:size]
        for mode in ("walk", "fast"):
            os.environ.update({"DRP_CLAIMS": mode, "DRP_WALK_MIN": "0", "DRP_DUMP_CLAIMS": f"/tmp/cl_{mode}.bin"})
            if os.path.exists(f"/tmp/cl_{mode}.bin"):
                os.remove(f"/tmp/cl_{mode}.bin")
            with drp_amd.Ctx(0) as c:
                c.set_blob_skip(drp_amd.BLOB_SKIP_OFF)
                g = c.decode_batch(w)
                t = c.timing()
            raw = np.fromfile(f"/tmp/cl_{mode}.bin", dtype=np.uint64)
            nt = int(raw[0])
            print(size, mode, "frames", g["nframes"], "repairs", t.spec_repairs, "relisted", t.verify_relisted,
                  "claims", [hex(int(x)) for x in raw[1:1 + nt]], flush=True)


if __name__ == "__main__":
    main()
