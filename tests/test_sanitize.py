"""Host sanitizers over the C oracle (round-2 review: no ASan/UBSan build of host code).

oracle/epnp_ransac.c (the C restatement of OpenCV 4.4's solvePnPRansac(EPNP), test
infrastructure) is compiled with -fsanitize=address,undefined together with
tests/sanitize/oracle_driver.c and run over exact, noisy, outlier-heavy, duplicated and
degenerate (n = 0..6) scenes.  Any out-of-bounds access, leak or undefined behaviour aborts the
run (halt_on_error); the test asserts a clean exit and no sanitizer report.  CPU only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_asan")
    cmd = ["gcc", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", os.path.join(REPO, "oracle", "epnp_ransac.c"),
           os.path.join(HERE, "sanitize", "oracle_driver.c"), "-o", exe, "-lm"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    report = r.stdout + r.stderr
    assert r.returncode == 0, report[-4000:]
    assert "runtime error" not in report and "AddressSanitizer" not in report, report[-4000:]
    assert report.count("status") == 12
