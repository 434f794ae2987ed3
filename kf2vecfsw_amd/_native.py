"""ctypes binding of the in-tree HIP library ``libkf2vec_gpu.so`` (C-ABI in
``include/kf2vec_gpu.h``).

There is no CPU fallback: if the library is missing or fails to load, every
entry point raises :class:`NativeError` -- the product path never silently
routes around the HIP code.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# KF2VEC_GPU_LIB may point at a profiling build (e.g. libkf2vec_gpu_ablation.so)
LIB_PATH = os.environ.get("KF2VEC_GPU_LIB") or os.path.join(_HERE, "libkf2vec_gpu.so")

KF_OK = 0
KF_EINVAL = -1
KF_EHIP = -2
KF_ERANGE = -3
KF_EFORMAT = -4
KF_MIN_K = 2
KF_MAX_K = 12
KF_SPARSE_MAX_K = 31
KF_ACCUMULATE = 1
KF_FMT_AUTO, KF_FMT_FASTA, KF_FMT_FASTQ = 0, 1, 2

# every symbol declared in include/kf2vec_gpu.h: (restype, argtypes)
_u64, _u32, _i32, _i64, _int = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int
_vp, _cp = ctypes.c_void_p, ctypes.c_char_p
_P64 = ctypes.POINTER(ctypes.c_uint64)
_PI = ctypes.POINTER(ctypes.c_int)
SIGNATURES = {
    "kf_abi_version": (_int, []),
    "kf_last_error": (_cp, []),
    "kf_num_bins": (_u64, [_int]),
    "kf_tables": (_int, [_int, _vp, _vp, _P64]),
    "kf_vocab_text": (_int, [_int, _vp, _u64, _P64]),
    "kf_index_records": (_int, [_vp, _u64, _int, _u64, _vp, _u64, _P64, _PI]),
    "kf_count_batch": (_int, [_vp, _vp, _i32, _vp, _u64, _vp, _vp, _int, _vp, _vp, _u32, _vp]),
    "kf_count_launch_info": (_int, [_int, _PI, _PI, _PI]),
    "kf_workspace_release": (_int, []),
    "kf_workspace_reserve": (_int, [_int, _i32]),
    "kf_build_id": (_cp, []),
    "kf_stream_probe": (_int, [_vp, _u64, _vp, _vp]),
    "kf_synth_fasta": (_int, [_vp, _vp, _i32, _i64, _i64, _u64, _u64, _int, _u64, _vp]),
    "kf_synth_genome_bytes": (_u64, [_i64, _u64, _int, _u64]),
    "kf_synth_header_len": (_u64, [_i64]),
    "kf_format_kf": (_int, [_cp, _vp, _u64, _int, _int, _vp, _u64, _P64]),
    "kf_write_kf_files": (_int, [_cp, ctypes.POINTER(_cp), _i32, _vp, _u64, _int, _int, _int]),
    "kf_write_kf_rows": (_int, [_cp, ctypes.POINTER(_cp), _i32, _vp, _u64, _int, _int, _int]),
    "kf_write_kf_segments": (_int, [_i32, ctypes.POINTER(_cp), _vp, _vp, ctypes.POINTER(_cp), ctypes.POINTER(_cp),
                                    _vp, _vp, _u32, _vp, _u64, _int, _int, _int]),
    "kf_write_kf_segments16": (_int, [_i32, ctypes.POINTER(_cp), _vp, _vp, ctypes.POINTER(_cp), ctypes.POINTER(_cp),
                                      _vp, _vp, _u32, _vp, _u64, _int, _int, _int]),
    "kf_chunk_compact": (_int, [_vp, _u64, _vp, _i32, _vp, _vp, _vp, _u64, _vp]),
    "kf_chunk_gather": (_int, [_vp, _vp, _i32, _u32, _vp, _vp]),
    "kf_index_fasta": (_int, [_vp, _vp, _i32, _u64, _vp, _u64, _vp, _vp, _u64, _vp]),
    "kf_read_files": (_int, [ctypes.POINTER(_cp), _i32, _vp, _vp, _vp, _u64, _int]),
    "kf_sparse_workspace_bytes": (_u64, [_int, _u64, _i32]),
    "kf_sparse_count": (_int, [_vp, _vp, _i32, _u64, _vp, _u64, _int, _vp, _u64, _vp, _vp, _vp, _vp]),
}


class NativeError(RuntimeError):
    pass


_lib = None


def lib() -> ctypes.CDLL:
    """Load libkf2vec_gpu.so (raises NativeError if it is absent: run
    ``python -m kf2vecfsw_amd.build``)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"{LIB_PATH} not found: build it with `python -m kf2vecfsw_amd.build`")
        # PyTorch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7).  Load it
        # first so our NEEDED libamdhip64.so.7 binds to the SAME HIP runtime instance;
        # otherwise the process holds two runtimes and torch's stream handles and
        # device pointers are invalid in ours (hipMemsetAsync fails).
        import torch  # noqa: F401
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - environment specific
            raise NativeError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.kf_abi_version() != 1:
            raise NativeError("libkf2vec_gpu ABI version mismatch")
        bid = L.kf_build_id().decode()
        # Any library must be built from the sources next to it (it travels
        # prebuilt with repo snapshots; build.source_id), whether it is the
        # product path or KF2VEC_GPU_LIB -- except a build that says it differs:
        # a "+prof" / "+flags..." / "+zoo" suffix (profiling, ablation and zoo
        # builds for tools/), or a library from another commit that an A/B tool
        # loads on purpose (KF2VEC_ALLOW_FOREIGN_LIB=1).
        if "+" not in bid and os.environ.get("KF2VEC_ALLOW_FOREIGN_LIB") != "1":
            from .build import source_id
            if bid != source_id():
                raise NativeError(f"{LIB_PATH} was built from other sources (build id {bid}, sources "
                                  f"{source_id()}): rebuild with `python -m kf2vecfsw_amd.build`")
        _lib = L
    return _lib


def build_id() -> str:
    """kf_build_id() of the loaded library (hash of its sources)."""
    return lib().kf_build_id().decode()


def check(rc: int, what: str = "") -> None:
    if rc != KF_OK:
        msg = lib().kf_last_error().decode(errors="replace")
        raise NativeError(f"{what or 'kf2vec_gpu'} failed ({rc}): {msg}")
