"""Native runtime under ThreadSanitizer: the shm SPSC ring's producer and
consumer threads move variable-size records through a small ring (constant wrap-around)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("sanitize", ["thread", None])
def test_ring_stress(tmp_path, sanitize):
    exe = str(tmp_path / "ring_stress")
    cmd = ["g++", "-std=c++17", "-O1", "-g", os.path.join(REPO, "csrc/runtime/shm_ring.cpp"),
           os.path.join(REPO, "csrc/runtime/tests/ring_stress.cpp"), "-o", exe, "-lrt", "-lpthread"]
    if sanitize:
        cmd.insert(1, f"-fsanitize={sanitize}")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and sanitize and "sanitize" in r.stderr:
        pytest.skip("sanitizer runtime unavailable")
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    p = subprocess.run([exe, "5000"], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0 and "OK 5000 records" in p.stdout, p.stderr[-3000:]
    assert "WARNING: ThreadSanitizer" not in p.stderr
