"""Host-only sanitizer run: the C oracle under ASan + UBSan.  CPU only."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_build/oracle_asan"], check=True)
    r = subprocess.run([os.path.join(ROOT, "oracle", "_build", "oracle_asan")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout
