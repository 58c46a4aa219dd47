"""In-tree build of libonepose_hip.so (hipcc, gfx950) and of the C oracle.

    python -m onepose_amd.build            # product library
    python -m onepose_amd.build --oracle   # also oracle/liboracle.so (test infrastructure)

Objects are cached under onepose_amd/_build/ and rebuilt when a source or header is newer.
The built .so files stay in the tree (git-ignored) so they travel to the GPU box.
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libonepose_hip.so")
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIP_FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-Wall",
             "-Wno-unused-function", "-Wno-unused-variable"]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build_lib(verbose=False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h"))
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer(o, [s, *headers, __file__]):
            jobs.append([HIPCC, *HIP_FLAGS, "-c", s, "-o", o])
    workers = min(len(jobs), int(os.environ.get("MAX_JOBS", "8")) or 1) if jobs else 1
    with ThreadPoolExecutor(max_workers=workers) as ex:
        for r, cmd in zip(ex.map(_run, jobs), jobs):
            if verbose:
                print(" ".join(cmd[-3:]), file=sys.stderr)
    if _newer(LIB, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB])
    return LIB


def build_oracle() -> str:
    src = os.path.join(ORACLE_DIR, "epnp_ransac.c")
    if _newer(ORACLE_LIB, [src, __file__]):
        _run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-fPIC", "-shared", src, "-lm",
              "-o", ORACLE_LIB])
    return ORACLE_LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build_lib(a.verbose))
    if a.oracle:
        print(build_oracle())


if __name__ == "__main__":
    main()
