"""In-tree build of libcodec_hip.so for gfx950 (no torch extension machinery: the
library is a plain C-ABI shared object loaded with ctypes).

    python -m codec_tcc_amd.build            # or __graft_entry__.build()

-ffp-contract=off is REQUIRED: the decision kernel reproduces numpy's float64 sums bit
for bit and must not fuse multiplies into adds.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", "codec_hip.hip"), os.path.join(HERE, "csrc", "codec_pee.hip"),
        os.path.join(HERE, "csrc", "codec_quality.hip")]
HDRS = [os.path.join(HERE, "csrc", "codec_common.h")]
OUT = os.path.join(HERE, "libcodec_hip.so")
INC = os.path.join(REPO, "include")
ARCH = os.environ.get("CODEC_OFFLOAD_ARCH", "gfx950")

FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", f"--offload-arch={ARCH}",
         "-Wall", "-Wno-unused-function"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _obj(src: str) -> str:
    return os.path.join(HERE, "build_obj", os.path.basename(src) + ".o")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _common_deps():
    return HDRS + [os.path.join(INC, "codec_tcc.h"), __file__]


def needs_build() -> bool:
    return _stale(OUT, SRCS + _common_deps())


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile each translation unit to an object (in parallel, only the stale ones), then
    link the shared library."""
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.join(HERE, "build_obj"), exist_ok=True)
    jobs = []
    for src in SRCS:
        obj = _obj(src)
        if force or _stale(obj, [src] + _common_deps()):
            cmd = [hipcc(), *[f for f in FLAGS if f != "-shared"], f"-I{INC}", "-c", src, "-o", obj + ".tmp"]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            jobs.append((obj, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
    errs = []
    for obj, p in jobs:
        _out, err = p.communicate()
        if p.returncode != 0:
            errs.append(f"hipcc failed ({p.returncode}) for {os.path.basename(obj)}:\n{err[-6000:]}")
        else:
            os.replace(obj + ".tmp", obj)
    if errs:
        raise RuntimeError("\n".join(errs))
    tmp = OUT + ".tmp"
    cmd = [hipcc(), *FLAGS, *[_obj(s) for s in SRCS], "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc link failed ({r.returncode}):\n{r.stderr[-6000:]}")
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
