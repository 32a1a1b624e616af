"""CPU: the oracle built with AddressSanitizer + UBSan (oracle/sanitize_fuzz.c, `make -C oracle
fuzz`) survives seeded random streams cut anywhere, random bytes through every policy error,
random chunkings and blob continuations, a tiny output capacity, and encoder rows with
max-width varints (SURVEY §5 "Race detection / sanitizers")."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_under_asan_ubsan():
    # one test builds once and runs every seed (parallel workers must not relink the binary
    # while another one executes it)
    subprocess.check_call(["make", "-s", "-B", "-C", os.path.join(ROOT, "oracle"), "fuzz"])
    exe = os.path.join(ROOT, "oracle", "_build", "sanitize_fuzz")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    for seed in (1, 2, 3):
        out = subprocess.run([exe, "1500", str(seed)], capture_output=True, text=True, timeout=300, env=env)
        assert out.returncode == 0, f"seed {seed}: " + out.stdout + out.stderr[-3000:]
        assert "sanitize_fuzz ok" in out.stdout
