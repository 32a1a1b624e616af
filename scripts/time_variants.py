"""Times decode_device over a C2 stream for several libdrp builds (measurement builds may
produce incomplete output; nothing is verified here). Usage: python scripts/time_variants.py
frames lib1.so lib2.so ...  (each build runs in its own child process)."""
import os
import subprocess
import sys

if len(sys.argv) > 2 and sys.argv[1] == "--child":
    import ctypes as C

    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import drp_amd
    n = int(sys.argv[2])
    dev = torch.device("cuda", 0)
    wire = bench.c2_on_device(n, seed=5, dev=dev)
    so = torch.tensor([0, wire.numel()], dtype=torch.int64, device=dev)
    outs = bench.alloc_outputs(n + 64, dev)
    res = torch.zeros(C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    ctx = drp_amd.Ctx(0)
    ms = []
    for i in range(6):
        ctx.decode_device(wire, so, None, outs, n + 64, res)
        if i:
            ms.append(ctx.timing().decode_ms)
    print(f"{os.path.basename(os.environ.get('DRP_LIB', 'default'))} {min(ms):.3f} ms min "
          f"{sum(ms) / len(ms):.3f} avg", flush=True)
    sys.exit(0)

frames = sys.argv[1]
for lib in sys.argv[2:]:
    env = dict(os.environ, DRP_LIB=os.path.abspath(lib))
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", frames], env=env,
                       timeout=300)
    if r.returncode:
        sys.exit(r.returncode)
