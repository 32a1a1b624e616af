"""GPU probe: repair passes of the speculative decode over shadow-stream parameters (16 MB each).
Usage: python scripts/probe_adversarial_sweep.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import _gpu  # noqa: E402,F401
import _streams as S  # noqa: E402
import drp_amd  # noqa: E402

with drp_amd.Ctx(0) as ctx:
    for period in [8192, 6000, 12000, 3000]:
        for at in [3, 20, 70, 200, 1000, 2500]:
            for small in [4, 10, 40, 200]:
                if at + small + 8 > period:
                    continue
                n = int(16 * 2**20 / period)
                wire = S.shadow_stream(n, period=period, shadow_at=at, small=small)
                g = ctx.decode_batch(wire)
                t = ctx.timing()
                print(f"period {period:5d} at {at:5d} small {small:4d}: frames {g['nframes']} repairs {t.spec_repairs} "
                      f"exact {t.strict_reruns} relisted {t.verify_relisted} decode {t.decode_ms:.2f} ms", flush=True)
