"""In-tree build of libcodec_hip.so for gfx950 (no torch extension machinery: the
library is a plain C-ABI shared object loaded with ctypes).

    python -m codec_tcc_amd.build            # or __graft_entry__.build()

-ffp-contract=off is REQUIRED: the decision kernel reproduces numpy's float64 sums bit
for bit and must not fuse multiplies into adds.

Staleness is decided by content, not by mtime: the library embeds a
SHA-256 of its sources, headers and compiler flags (`codec_build_digest()`), every object
keeps the digest of its own inputs beside it, and `_lib.load()` refuses an in-tree library
whose digest differs from the tree's -- a copied-in or stale binary cannot pass for the
committed sources.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", "codec_hip.hip"), os.path.join(HERE, "csrc", "codec_pee.hip"),
        os.path.join(HERE, "csrc", "codec_quality.hip"), os.path.join(HERE, "csrc", "codec_records.hip")]
HDRS = [os.path.join(HERE, "csrc", "codec_common.h")]
OUT = os.path.join(HERE, "libcodec_hip.so")
INC = os.path.join(REPO, "include")
ARCH = os.environ.get("CODEC_OFFLOAD_ARCH", "gfx950")
# extra -D... flags of a diagnostic build (part of the digest, so such a build never passes
# for the release library)
EXTRA = os.environ.get("CODEC_BUILD_DEFS", "").split()

FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", f"--offload-arch={ARCH}",
         "-Wall", "-Wno-unused-function"] + EXTRA
DIGEST_TAG = b"codec-src-sha256:"
FLAGS_TAG = b"codec-build-flags:"   # the flags the digest covers, embedded beside it


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _obj(src: str) -> str:
    return os.path.join(HERE, "build_obj", os.path.basename(src) + ".o")


def _common_deps():
    return HDRS + [os.path.join(INC, "codec_tcc.h")]


def _digest(paths, flags) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.relpath(p, REPO).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def source_digest(flags=None) -> str:
    """Digest of everything the library is compiled from (sources, headers, flags); `flags`
    defaults to this process's build flags (CODEC_OFFLOAD_ARCH / CODEC_BUILD_DEFS)."""
    missing = [p for p in SRCS + _common_deps() if not os.path.exists(p)]
    if missing:
        raise RuntimeError(f"cannot check libcodec_hip.so against its sources: {', '.join(missing)} absent "
                           "(an installed package without csrc/? rebuild in a source tree)")
    return _digest(SRCS + _common_deps(), FLAGS if flags is None else flags)


def library_digest(path: str = OUT):
    """The digest embedded in a built library (read from its bytes, without loading it), or
    None when it has none."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(DIGEST_TAG)
    if i < 0:
        return None
    hexd = data[i + len(DIGEST_TAG): i + len(DIGEST_TAG) + 64]
    return hexd.decode("ascii", "replace")


def _c_escape(text: str) -> str:
    return text.replace("\\", "\\\\").replace('"', '\\"')


def library_flags(path: str = OUT):
    """The build flags embedded in a built library (list), or None when it has none."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(FLAGS_TAG)
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i + len(FLAGS_TAG): j].decode("utf-8", "replace").split("\x1f")


def _obj_stale(src: str, force: bool) -> bool:
    obj = _obj(src)
    if force or not os.path.exists(obj) or not os.path.exists(obj + ".digest"):
        return True
    with open(obj + ".digest") as f:
        return f.read().strip() != _digest([src] + _common_deps(), FLAGS)


def needs_build() -> bool:
    return library_digest(OUT) != source_digest()


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile each translation unit to an object (in parallel, only those whose inputs
    changed), then link the shared library with the source digest embedded."""
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.join(HERE, "build_obj"), exist_ok=True)
    jobs = []
    for src in SRCS:
        obj = _obj(src)
        if _obj_stale(src, force):
            cmd = [hipcc(), *[f for f in FLAGS if f != "-shared"], f"-I{INC}", "-c", src, "-o", obj + ".tmp"]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            jobs.append((src, obj, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
    errs = []
    for src, obj, p in jobs:
        _out, err = p.communicate()
        if p.returncode != 0:
            errs.append(f"hipcc failed ({p.returncode}) for {os.path.basename(obj)}:\n{err[-6000:]}")
        else:
            os.replace(obj + ".tmp", obj)
            with open(obj + ".digest", "w") as f:
                f.write(_digest([src] + _common_deps(), FLAGS))
    if errs:
        raise RuntimeError("\n".join(errs))
    # the digest lives in a one-function translation unit of its own
    dsrc = os.path.join(HERE, "build_obj", "codec_digest.cpp")
    with open(dsrc, "w") as f:
        f.write("// generated by codec_tcc_amd/build.py: digest of the library's sources and flags\n"
                f'static const char k_digest[] = "{DIGEST_TAG.decode()}{source_digest()}";\n'
                f'extern "C" const char k_codec_build_flags[] = "{FLAGS_TAG.decode()}'
                + "\\037".join(_c_escape(f) for f in FLAGS) + '";\n'
                'extern "C" const char* codec_build_digest(void) '
                f"{{ return k_digest + {len(DIGEST_TAG)}; }}\n")
    dobj = os.path.join(HERE, "build_obj", "codec_digest.o")
    r = subprocess.run(["g++", "-O2", "-fPIC", "-c", dsrc, "-o", dobj], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"digest object failed:\n{r.stderr[-2000:]}")
    tmp = OUT + ".tmp"
    cmd = [hipcc(), *FLAGS, *[_obj(s) for s in SRCS], dobj, "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc link failed ({r.returncode}):\n{r.stderr[-6000:]}")
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
