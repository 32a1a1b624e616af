import os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import _gpu
import _streams as S
from _gpu import drp_amd
wire = S.shadow_stream(int(16 * 2**20 / 6000), period=6000, shadow_at=200, small=40)
with drp_amd.Ctx(0) as ctx:
    g = ctx.decode_batch(wire)
    t = ctx.timing()
    print("strict", t.strict_reruns, "repairs", t.spec_repairs, "seg", t.seg_repairs, "relisted", t.verify_relisted, flush=True)
