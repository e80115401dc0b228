"""ctypes binding of libcodec_hip.so (include/codec_tcc.h).

The library is built in-tree (codec_tcc_amd/libcodec_hip.so, see build.py).  There is no
CPU fallback: if the library cannot be loaded, every entry point raises RuntimeError.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CODEC_TCC_LIB: an alternative build of the same library (A/B benchmarking, tools/archive/ab_bench.sh)
_DEFAULT_PATH = os.path.join(_HERE, "libcodec_hip.so")
LIB_PATH = os.environ.get("CODEC_TCC_LIB") or _DEFAULT_PATH

MAX_PLANES = 16
MODE_HYBRID = 0
MODE_MULTI = 1
FLAG_OVERLAP = 1
FLAG_LOSSY = 2
FLAG_BADLUT = 4
FLAG_DECIDE_TIMEOUT = 8   # split decision: a plane workgroup never reported (status 2)
FLAG_INFO_FAST = 16      # s decided by the guard band: mi[] = H(X), cum_info their sum
FLAG_GUARD_FALLBACK = 32 # a prefix within 1e-9 of the target: the exact numpy-order sums decided

I16 = C.c_int32 * MAX_PLANES
D16 = C.c_double * MAX_PLANES


class Params(C.Structure):
    _fields_ = [
        ("B", C.c_int32), ("H", C.c_int32), ("W", C.c_int32),
        ("in_bytes", C.c_int32), ("out_bytes", C.c_int32), ("nbits", C.c_int32),
        ("block", C.c_int32), ("align", C.c_int32), ("mode", C.c_int32),
        ("fixed_s", C.c_int32), ("fixed_offset", C.c_int32), ("all_mi", C.c_int32),
        ("payload_words", C.c_int32), ("map_words", C.c_int32), ("n_classes", C.c_int32),
        ("reserved", C.c_int32), ("beta", C.c_double),
    ]


class Layout(C.Structure):
    _fields_ = [("sizes", I16), ("perm", I16), ("src", I16), ("len", I16)]


class SliceMeta(C.Structure):
    _fields_ = [
        ("s", C.c_int32), ("start_offset", C.c_int32), ("total_used", C.c_int32),
        ("flags", C.c_uint32), ("npix", C.c_int32), ("nbits", C.c_int32),
        ("status", C.c_int32), ("nonzero_bins", C.c_int32),
        ("perm", I16), ("sizes", I16), ("n", I16), ("src", I16), ("off", I16), ("cat", I16),
        ("entropy", C.c_double), ("target", C.c_double), ("cum_info", C.c_double),
        ("span_lo", C.c_int32), ("span_len", C.c_int32), ("mi", D16),
    ]


class PeeParams(C.Structure):
    _fields_ = [("B", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("bytes", C.c_int32),
                ("T", C.c_int32), ("maxval", C.c_int32), ("payload_words", C.c_int32), ("lm_words", C.c_int32)]


class PeeMeta(C.Structure):
    _fields_ = [("T", C.c_int32), ("maxval", C.c_int32), ("L", C.c_int32), ("end", C.c_int32),
                ("nc", C.c_int32), ("ntiles", C.c_int32), ("tile_end", C.c_int32), ("status", C.c_int32),
                ("capacity", C.c_int32), ("lm_count", C.c_int32), ("h", C.c_int32), ("w", C.c_int32),
                ("flags", C.c_int32), ("reserved", C.c_int32 * 3)]


def tuning_knob(name: str, default: int) -> int:
    """A Python-side launch-shape knob, honoured like the library's (include/codec_tcc.h,
    codec_set_tuning): the environment value only when CODEC_TUNING=1, else the default."""
    if os.environ.get("CODEC_TUNING", "0") != "1":
        return default
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


PEE_PARTIAL = 1
PEE_RECORD_HDR_WORDS = 8   # CODEC_PEE_RECORD_HDR_WORDS: codec_pee_meta in uint64 words
META_BYTES = C.sizeof(SliceMeta)
PEE_META_BYTES = C.sizeof(PeeMeta)
CODEC_PEE_ELOOKBACK = 2  # meta.status: look-back gave up (include/codec_tcc.h)
LAYOUT_BYTES = C.sizeof(Layout)

_VP = C.c_void_p
_SIGS = {
    "codec_abi_version": (C.c_int, []),
    "codec_build_digest": (C.c_char_p, []),
    "codec_set_tuning": (C.c_int, [C.c_int32]),
    "codec_last_error": (C.c_char_p, []),
    "codec_workspace_bytes": (C.c_size_t, [C.POINTER(Params)]),
    "codec_plan": (C.c_int, [C.POINTER(Params), _VP, _VP, _VP, C.c_int64, _VP, _VP, _VP, _VP, C.c_size_t, _VP]),
    "codec_embed": (C.c_int, [C.POINTER(Params), _VP, _VP, _VP, _VP, _VP, _VP]),
    "codec_encode": (C.c_int, [C.POINTER(Params), _VP, _VP, _VP, C.c_int64, _VP, _VP, _VP, _VP, C.c_size_t,
                               _VP, _VP, _VP]),
    "codec_extract": (C.c_int, [C.POINTER(Params), _VP, _VP, _VP, _VP, _VP, _VP]),
    "codec_refdecode": (C.c_int, [C.POINTER(Params), _VP, _VP, _VP, _VP, C.c_int32, _VP, _VP]),
    "codec_refdecode_dense": (C.c_int, [C.POINTER(Params), _VP, C.c_int32, _VP, C.c_int32, _VP, _VP,
                                        C.c_int32, _VP, _VP]),
    "codec_expand_maps": (C.c_int, [C.POINTER(Params), _VP, _VP, _VP, C.c_int32, _VP]),
    "codec_restore_dense": (C.c_int, [C.POINTER(Params), _VP, _VP, C.c_int32, _VP, _VP, _VP]),
    "codec_unpack_planes": (C.c_int, [C.POINTER(Params), _VP, C.c_int32, C.c_int32, _VP, C.c_int32, _VP]),
    "codec_merge_planes": (C.c_int, [C.POINTER(Params), _VP, C.c_int32, C.c_int32, _VP, _VP]),
    "codec_pee_workspace_bytes": (C.c_size_t, [C.POINTER(PeeParams)]),
    "codec_pee_extract_flag_offset": (C.c_size_t, [C.POINTER(PeeParams)]),
    "codec_pee_diag_offset": (C.c_size_t, [C.POINTER(PeeParams)]),
    "codec_pee_reset": (C.c_int, [C.POINTER(PeeParams), _VP, C.c_size_t, _VP]),
    "codec_debug_res_trace": (C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    "codec_pee_embed": (C.c_int, [C.POINTER(PeeParams), _VP, _VP, _VP, _VP, _VP, _VP, _VP, C.c_size_t, _VP]),
    "codec_pee_extract": (C.c_int, [C.POINTER(PeeParams), _VP, _VP, _VP, _VP, _VP, _VP, C.c_size_t, _VP]),
    "codec_pee_embed_ts": (C.c_int, [C.POINTER(PeeParams), _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, C.c_size_t, _VP]),
    "codec_pee_capacity": (C.c_int, [C.POINTER(PeeParams), _VP, C.c_int32, _VP, _VP, _VP, _VP, C.c_size_t, _VP]),
    "codec_pee_embed_auto": (C.c_int, [C.POINTER(PeeParams), _VP, _VP, _VP, _VP, C.c_int32, _VP, _VP, _VP, _VP,
                                       C.c_size_t, _VP]),
    "codec_pee_multi_embed_pass": (C.c_int, [C.POINTER(PeeParams), C.c_int32, _VP, _VP, _VP, _VP, _VP, _VP, _VP,
                                             C.c_size_t, _VP]),
    "codec_pee_multi_extract_pass": (C.c_int, [C.POINTER(PeeParams), C.c_int32, _VP, _VP, _VP, _VP, _VP, _VP,
                                               C.c_size_t, _VP]),
    "codec_pee_multi_embed": (C.c_int, [C.POINTER(PeeParams), _VP, _VP, _VP, _VP, _VP, _VP, _VP, C.c_size_t, _VP]),
    "codec_pee_multi_extract": (C.c_int, [C.POINTER(PeeParams), _VP, _VP, _VP, _VP, _VP, _VP, C.c_size_t, _VP]),
    "codec_pee_pack_records": (C.c_int, [C.c_int32, C.c_int32, _VP, _VP, C.c_int32, _VP, _VP]),
    "codec_pee_unpack_records": (C.c_int, [C.c_int32, C.c_int32, _VP, C.c_int32, _VP, _VP, _VP]),
    "codec_quality_moments": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, _VP, _VP, _VP, _VP]),
    "codec_block_variance": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _VP, _VP, _VP]),
    "codec_lsb_runs": (C.c_int, [C.c_int32, C.c_int64, C.c_int32, _VP, _VP, _VP, C.c_int64, _VP, C.c_int32, _VP]),
    "codec_profile_begin": (C.c_int, [C.c_int32]),
    "codec_profile_end": (C.c_int, [_VP, _VP, C.c_int32]),
}
KERNEL_TAGS = {1: "k_scan_fast", 2: "k_scan_generic", 3: "k_block_exact", 4: "k_decide",
               5: "k_embed", 6: "k_restore", 7: "k_gather", 8: "other", 9: "k_pee_scan", 10: "k_pee_locate",
               11: "k_pee_embed", 12: "k_pee_copy", 13: "k_pee_dcount", 14: "k_pee_recover",
               15: "k_pee_embed1", 16: "k_pee_extract1", 17: "k_scan_read", 18: "k_unxor",
               19: "k_scan_rows", 20: "k_scan_rows_read", 21: "k_quality", 22: "k_decide_embed",
               23: "k_pee_capacity", 24: "k_pee_embed_ss", 25: "k_pee_extract_ss",
               26: "k_pee_embed_ss_auto", 27: "k_pee_embed_res", 28: "k_scan_decide",
               29: "k_pee_lat_count", 30: "k_pee_lat_embed", 31: "k_pee_lat_dcount", 32: "k_pee_lat_recover",
               33: "k_pee_lat_ss_embed", 34: "k_pee_lat_ss_extract"}
EXPORTS = tuple(_SIGS)

_lib = None
_load_error = None
# -D flags of diagnostic builds (tools/): never the product library
_DIAG_DEFINES = {"-DDECIDE_TS", "-DDECIDE_TS_SCAN_ONLY", "-DCODEC_ST_SC", "-DPEE_LB_TRACE", "-DPEE_SS_TRACE",
                 "-DCODEC_DEBUG_KNOBS", "-DRES_TRACE", "-DPEE_X_COPYONLY"}


def load(path: str = LIB_PATH):
    """Load (once) and return the library; raise RuntimeError if it is missing."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    # torch must be imported first: it ships its own libamdhip64 (soname libamdhip64.so.7).
    # Loaded first, it is the one our NEEDED entry binds to; loaded second, the process
    # would hold two HIP runtimes and device pointers from one are unknown to the other.
    import torch  # noqa: F401
    if not os.path.exists(path):
        raise RuntimeError(f"libcodec_hip.so not found at {path}: build it with "
                           f"`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback)")
    in_tree = os.path.abspath(path) == os.path.abspath(_DEFAULT_PATH)
    if in_tree:
        _check_digest(path)
    try:
        lib = C.CDLL(path)
    except OSError as e:  # pragma: no cover - environment specific
        _load_error = e
        raise RuntimeError(f"cannot load {path}: {e}") from e
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if name == "codec_build_digest" and not in_tree:   # a diagnostic build (tools/)
                continue
            raise RuntimeError(f"{path} does not export {name}")
        fn.restype = res
        fn.argtypes = args
    if lib.codec_abi_version() != 1:
        raise RuntimeError("libcodec_hip.so ABI mismatch")
    _lib = lib
    return lib


def _check_digest(path: str):
    """Refuse an in-tree library not built from the tree's sources: its
    embedded digest (build.library_digest, read from the file before loading it) must equal
    the digest of csrc/*, include/codec_tcc.h and the build flags.  No rebuild here: on the
    GPU box the prebuilt library is the product, and a mismatch there is an error."""
    from . import build
    # the flags the library was built with travel inside it: a build for another
    # CODEC_OFFLOAD_ARCH / CODEC_BUILD_DEFS loads without that environment, and a mismatch
    # names the sources as the cause only when they are
    flags = build.library_flags(path)
    # a diagnostic build matches its own digest but is not the product: phase
    # stamps, a scan that returns before deciding (DECIDE_TS_SCAN_ONLY), trace buffers ...
    diag = sorted({f for f in (flags or []) if f.split("=")[0] in _DIAG_DEFINES})
    if diag and os.environ.get("CODEC_ALLOW_DIAG_LIB") != "1":
        raise RuntimeError(f"{path} is a diagnostic build ({' '.join(diag)}); rebuild the product library with "
                           "`python -c 'import __graft_entry__ as g; g.build()'` (CODEC_ALLOW_DIAG_LIB=1 loads it anyway)")
    if flags is not None and flags != build.FLAGS and not diag:
        import warnings
        warnings.warn(f"{path} was built with non-default flags {' '.join(flags)}", RuntimeWarning, stacklevel=3)
    have, want = build.library_digest(path), build.source_digest(flags)
    if have != want:
        extra = "" if flags is None or flags == build.FLAGS else \
            f" (built with flags {' '.join(flags)}; this environment's are {' '.join(build.FLAGS)})"
        raise RuntimeError(f"{path} was not built from these sources (library digest {have}, sources {want}){extra}: "
                           "rebuild it with `python -c 'import __graft_entry__ as g; g.build()'`")


def check(rc: int, what: str):
    if rc != 0:
        msg = load().codec_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    """Raw device pointer of a torch tensor (or None)."""
    return None if t is None else t.data_ptr()
