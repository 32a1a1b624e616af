"""Summarises a per-tile timestamp trace written by a DRP_STATS=1 DRP_TRACE_FILE=... decode
(s_memrealtime, 100 MHz). Usage: python scripts/trace_stats.py trace.bin ntiles"""
import sys

import numpy as np

T = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8)
n = int(sys.argv[2]) if len(sys.argv) > 2 else int((T[:, 5] != 0).sum())
T = T[:n].astype(np.int64)
t0 = T[:, 0].min()
st, dp, agg, x, cn, en = [(T[:, k] - t0) * 0.01 for k in range(6)]  # microseconds
g = np.arange(n) % 4 == 0
pc = [10, 50, 90, 99]
prev = np.concatenate([[0], np.maximum.accumulate(agg)[:-1]])
print(f"tiles {n} span {en.max():.1f} us")
for name, d in [("stage+dp", dp - st), ("agg after dp", agg - dp), ("x after dp (group-first)", (x - dp)[g]),
                ("x after dp (siblings)", (x - dp)[~g]), ("x after all pred maps (first)", (x - prev)[g][100:]),
                ("pred maps after own dp (first)", (prev - dp)[g][100:]), ("count base after x", cn - x),
                ("emit", en - cn), ("whole tile", en - st)]:
    print(f"{name:34s}", " ".join(f"{v:8.2f}" for v in np.percentile(d, pc)))
