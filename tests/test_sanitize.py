"""Host sanitizers (round-2 review: no ASan/UBSan build of host code).

1. oracle/epnp_ransac.c (the C restatement of OpenCV 4.4's solvePnPRansac(EPNP), test
infrastructure) is compiled with -fsanitize=address,undefined together with
tests/sanitize/oracle_driver.c and run over exact, noisy, outlier-heavy, duplicated and
degenerate (n = 0..6) scenes.  Any out-of-bounds access, leak or undefined behaviour aborts the
run (halt_on_error); the test asserts a clean exit and no sanitizer report.
2. libonepose_hip's host code (packers, size queries) with host-side ASan/UBSan
   (tests/sanitize/host_driver.cpp).  CPU only: no GPU call is made."""
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


SRCS = ("matcher", "gemm", "pnp", "frame_ops", "superpoint")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_library_host_code_under_asan_ubsan(tmp_path):
    """The library's host code (weight packers, every workspace / cache size query over ragged,
    tiny, batched and sharded shapes) in a build with -fsanitize=address,undefined on the host
    side only (-Xarch_host; the gfx950 code is built as usual and never launched)."""
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined"]
    inc = ["-I", os.path.join(REPO, "onepose_amd", "csrc"), "-I", os.path.join(REPO, "include")]
    procs = []
    for f in SRCS:
        cmd = [HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-fPIC", "-std=c++17",
               "-fno-omit-frame-pointer", *san, *inc, "-c",
               os.path.join(REPO, "onepose_amd", "csrc", f + ".hip"), "-o", str(tmp_path / (f + ".o"))]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    for p in procs:
        out, err = p.communicate(timeout=600)
        assert p.returncode == 0, err[-4000:]
    lib = str(tmp_path / "libonepose_asan.so")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", *san, "-o", lib,
                        *[str(tmp_path / (f + ".o")) for f in SRCS]], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    exe = str(tmp_path / "host_driver")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", *san, "-I",
                        os.path.join(REPO, "include"), os.path.join(HERE, "sanitize", "host_driver.cpp"),
                        "-o", exe, f"-L{tmp_path}", "-lonepose_asan", f"-Wl,-rpath,{tmp_path}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    report = r.stdout + r.stderr
    assert r.returncode == 0, report[-4000:]
    assert "runtime error" not in report and "AddressSanitizer" not in report, report[-4000:]
    assert "size queries ok" in report
