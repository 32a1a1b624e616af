"""Calibration ratio reference-JS / C restatement (BASELINE.md "Calibration"), this container.

Times the UNMODIFIED reference decoder (/root/reference/decode.js required in place, shims in
oracle/ref_js/shims, DRP_REF_CODEC=full) and the oracle's C restatement on the same C2 sample
in 64 KiB writes, one core each, and writes profiles/calibration_ref_js.json. bench.py reports
the ratio beside its cpu_baseline (the reference itself cannot run on the GPU box).
    python scripts/calibrate_reference.py [--frames N] [--seconds S]
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _oracle as O  # noqa: E402
import _streams as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1_000_000)
    ap.add_argument("--seconds", type=float, default=10.0)
    a = ap.parse_args()
    wire = S.c2_stream(a.frames, seed=7).tobytes()
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(wire)
        path = f.name
    try:
        env = dict(os.environ, NODE_PATH=os.path.join(ROOT, "oracle", "ref_js", "shims"), DRP_REF_CODEC="full",
                   NODE_NO_WARNINGS="1")
        ref = json.loads(subprocess.check_output(
            ["node", os.path.join(ROOT, "oracle", "ref_js", "ref_run.js"), "bench", path, "65536", str(a.seconds)],
            env=env, text=True))
    finally:
        os.unlink(path)
    outs = O.alloc_outputs(a.frames + 16)
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        r = O.decode_batch(wire, chunk=65536, outs=outs)
        assert r["nframes"] == a.frames
        reps += 1
    dt = time.perf_counter() - t0
    port = reps * a.frames / dt
    doc = {"workload": f"C2 sample, {a.frames} frames x 86 B, 64 KiB writes, 1 core each",
           "reference_js": {"frames_per_s": ref["frames_per_s"], "node": ref["node"],
                            "what": "/root/reference/decode.js in place + oracle/ref_js shims (full codec)"},
           "port_c": {"frames_per_s": port, "what": "oracle/drp_oracle.c (decode.js + protocol-buffers@2 restatement)"},
           "ratio_ref_js_over_port": ref["frames_per_s"] / port,
           "host": platform.processor() or platform.machine(), "generated_by": "scripts/calibrate_reference.py"}
    out = os.path.join(ROOT, "profiles", "calibration_ref_js.json")
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
