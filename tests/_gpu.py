"""Helpers for GPU tests: load the libdrp binding (never a fallback)."""
import os
import sys

import torch  # noqa: E402

# torch's HIP runtime initialises before libdrp's (the order bench.py uses): a process that
# loads libdrp first then fails torch's lazy device init ("no ROCm-capable device")
if torch.cuda.is_available():
    torch.cuda.init()

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dat-replication-protocol_amd", "python"))
import drp_amd  # noqa: E402,F401

import numpy as np  # noqa: E402

import _oracle as O  # noqa: E402

CMP_KEYS = ["payload_off", "payload_len", "type"]
COL_KEYS = O.COLS32 + O.COLS64 + ["flags"]


def assert_same(g, r, label=""):
    """Bit-exact comparison of a libdrp decode with the oracle."""
    for k in ["nframes", "err_code", "err_detail", "consumed", "tail", "blob_remaining"]:
        assert g[k] == r[k], (label, k, g[k], r[k])
    if r["err_code"]:
        assert g["err_frame"] == r["err_frame"], (label, "err_frame", g["err_frame"], r["err_frame"])
    n = len(r["type"])
    assert len(g["type"]) == n, (label, "rows", len(g["type"]), n)
    for k in CMP_KEYS:
        np.testing.assert_array_equal(g[k], r[k], err_msg=f"{label}:{k}")
    ch = (r["type"] & 0x3F) == 1
    for k in COL_KEYS:
        np.testing.assert_array_equal(g[k][ch], r[k][ch], err_msg=f"{label}:{k}")
