"""Build the in-tree HIP library ghost_amd/libghost_amd.so for gfx950.

    python -m ghost_amd.build          # incremental
    python -m ghost_amd.build --force  # rebuild everything

Each ``csrc/*.hip`` is compiled by ``hipcc --offload-arch=gfx950`` to an object
(in parallel), then linked into one shared library exporting the C ABI declared in
``include/ghost_amd.h``.  The .so is git-ignored but travels to the GPU box with the
gpurun snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
TUNING = os.environ.get("GHOST_TUNING") == "1"   # A/B build: GHOST_KNOB switches read the environment
OBJ = os.path.join(HERE, "_build_tuning" if TUNING else "_build")
LIB = os.path.join(HERE, "libghost_amd_tuning.so" if TUNING else "libghost_amd.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I" + CSRC, "-I" + INCLUDE,
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable"] + (["-DGHOST_TUNING"] if TUNING else [])


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return hs


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OBJ, os.path.basename(src)[:-4] + ".o")
    newest_dep = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _headers()])
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj
    cmd = [HIPCC] + CFLAGS + ["-c", src, "-o", obj]
    if os.path.exists(obj):
        os.remove(obj)            # a failed compile must not leave the old object looking current
    r = subprocess.run(cmd, capture_output=True, text=True)
    # hipcc can report an assembler failure of the device pass ("failed to execute") with exit status 0:
    # trust the object file, not the status alone
    if r.returncode != 0 or not os.path.exists(obj) or "failed to execute" in r.stderr:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-4000:]}")
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=min(len(srcs), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    if verbose:
        print(f"[ghost_amd] built {LIB}")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
