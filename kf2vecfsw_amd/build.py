"""Builds the in-tree HIP library ``kf2vecfsw_amd/libkf2vec_gpu.so`` for gfx950.

``python -m kf2vecfsw_amd.build`` (also called by ``__graft_entry__.build()``).
hipcc cross-compiles for gfx950 without a GPU; the .so is git-ignored but ships
to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libkf2vec_gpu.so")
BUILD = os.path.join(HERE, "_build")
ARCH = os.environ.get("KF_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES_HIP = ["kf_count.hip", "kf_bucket.hip", "kf_chunks.hip", "kf_sparse.hip", "kf_index.hip"]
SOURCES_CPP = ["kf_host.cpp"]
DEPS = SOURCES_HIP + SOURCES_CPP + ["kf_internal.h", "kf_front.h", "../../include/kf2vec_gpu.h"]


def source_id() -> str:
    """Hash of the library's sources (csrc/ + the C-ABI header) and target: what
    kf_build_id() of a library built from them returns (16 hex digits)."""
    h = hashlib.sha256(ARCH.encode())
    for d in sorted(DEPS):
        h.update(b"\0" + os.path.basename(d).encode() + b"\0")
        with open(os.path.join(CSRC, d), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def embedded_id(path: str) -> str | None:
    """The build id embedded in a built library (without loading it)."""
    try:
        with open(path, "rb") as f:
            blob = f.read()
    except OSError:
        return None
    i = blob.find(b"KF_BUILD_ID=")
    if i < 0:
        return None
    j = blob.find(b"\0", i)
    return blob[i + 12: j].decode(errors="replace")


def _stale() -> bool:
    """The product library is stale unless its embedded id equals the sources'
    hash (mtimes are not trusted: the .so travels with repo snapshots)."""
    return embedded_id(OUT) != source_id()


def build(force: bool = False, verbose: bool = False, ablation: bool = False, out: str | None = None) -> str:
    """ablation=True: a profiling build of the product (KF_PROFILE_BUILD: the
    bucket kernels' KF_BUCKET_PROFILE / KF_BK_WEIGHTS knobs, KF_K9_BUCKET) from
    the sources with tools/zoo/bucket_ablations.patch applied (KF_BK_ABL=n via
    KF_HIPCC_FLAGS).
    Serialised by a file lock: every rank of a multi-process run may call it."""
    import fcntl
    out = out or OUT
    if not force and not ablation and out == OUT and not _stale():
        return OUT
    os.makedirs(BUILD, exist_ok=True)
    with open(os.path.join(BUILD, ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and not ablation and out == OUT and not _stale():   # another rank built it
            return OUT
        return _build_locked(verbose, ablation, out)


HEADERS = ["kf_internal.h", "kf_front.h", "../../include/kf2vec_gpu.h"]

_TOOLCHAIN: list[bytes] = []


def _toolchain_id() -> bytes:
    """The compilers' identity (`hipcc --version`, `g++ --version`, once per
    process): part of every object's cache key, so a toolchain upgrade never
    relinks stale objects."""
    if not _TOOLCHAIN:
        out = b""
        for cmd in ([HIPCC, "--version"], ["g++", "--version"]):
            try:
                out += subprocess.run(cmd, capture_output=True, check=False).stdout
            except OSError:
                out += b"missing:" + cmd[0].encode()
        _TOOLCHAIN.append(out)
    return _TOOLCHAIN[0]


def _object(src: str, cmd_tail: list[str], csrc: str = CSRC) -> tuple[str, bool]:
    """Object path for `src` compiled with `cmd_tail`, keyed by the hash of the
    source, the shared headers, the command and the compilers' versions (so an
    edit rebuilds only the objects it touches); and whether it already exists."""
    h = hashlib.sha256(" ".join(cmd_tail).encode() + b"\0" + _toolchain_id())
    for d in [src] + HEADERS:
        with open(os.path.join(csrc, d), "rb") as f:
            h.update(f.read())
    o = os.path.join(BUILD, f"{src}.{h.hexdigest()[:16]}.o")
    return o, os.path.exists(o)


ABL_PATCHES = [os.path.join(HERE, "..", "tools", "zoo", "bucket_ablations.patch")]


def _ablation_sources() -> str:
    """A copy of csrc/ (and the header) with tools/zoo/bucket_ablations.patch
    applied: the bucket kernels' KF_BK_ABL=n profiling ablations (wrong counts by
    design), kept out of the product source.  Returns its csrc directory."""
    import shutil
    root = os.path.join(BUILD, "abl_src")
    shutil.rmtree(root, ignore_errors=True)
    shutil.copytree(CSRC, os.path.join(root, "kf2vecfsw_amd", "csrc"))
    os.makedirs(os.path.join(root, "include"))
    shutil.copy(os.path.join(HERE, "..", "include", "kf2vec_gpu.h"), os.path.join(root, "include"))
    for p in ABL_PATCHES:
        subprocess.run(["patch", "-s", "-p1", "-d", root, "-i", os.path.abspath(p)], check=True)
    return os.path.join(root, "kf2vecfsw_amd", "csrc")


def _build_locked(verbose: bool, ablation: bool, out: str) -> str:
    objs = []
    csrc = _ablation_sources() if ablation else CSRC
    # profiling / ablation builds carry a suffix, so the product check refuses them
    flags = os.environ.get("KF_HIPCC_FLAGS", "")
    bid = source_id() + ("+prof" if ablation else "") + \
        ("+flags" + hashlib.sha256(flags.encode()).hexdigest()[:8] if flags.strip() else "")
    for s in SOURCES_HIP:
        tail = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall"] + \
            (["-DKF_PROFILE_BUILD"] if ablation else []) + flags.split()   # KF_HIPCC_FLAGS: tools/ only
        o, have = _object(s, tail, csrc)
        if not have or verbose:
            cmd = [HIPCC] + tail + ["-c", os.path.join(csrc, s), "-o", o + ".tmp"]
            if verbose:
                cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
            subprocess.run(cmd, check=True)
            os.replace(o + ".tmp", o)
        objs.append(o)
    for s in SOURCES_CPP:
        tail = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-pthread", f'-DKF_BUILD_ID="{bid}"']
        o, have = _object(s, tail, csrc)
        if not have:
            subprocess.run(["g++"] + tail + ["-c", os.path.join(csrc, s), "-o", o + ".tmp"], check=True)
            os.replace(o + ".tmp", o)
        objs.append(o)
    tmp = out + ".tmp"
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", *objs, "-o", tmp],
                   check=True)
    os.replace(tmp, out)
    return out


def build_sanitized_host(out: str | None = None) -> str:
    """SURVEY section 5 (sanitizers, host code only): the host half of the library
    (csrc/kf_host.cpp) linked with the driver tests/host_sanitize.cpp under
    AddressSanitizer + UndefinedBehaviorSanitizer (g++; no HIP in this binary)."""
    out = out or os.path.join(BUILD, "host_sanitize")
    os.makedirs(BUILD, exist_ok=True)
    drv = os.path.join(HERE, "..", "tests", "host_sanitize.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-Wall", "-Wextra", "-pthread", drv, os.path.join(CSRC, "kf_host.cpp"),
                    "-o", out], check=True)
    return out


def build_zoo() -> str:
    """tools/zoo/libkf2vec_zoo.so: the round-2 library with every rejected k <= 8
    kernel variant (KF_COUNT_VARIANT, KF_COUNT_PROFILE, KF_BUCKET_MIN_K knobs),
    for tools/ measurements only -- never loaded by the product (KF2VEC_GPU_LIB)."""
    zoo = os.path.join(HERE, "..", "tools", "zoo")
    out = os.path.join(zoo, "libkf2vec_zoo.so")
    bld = os.path.join(BUILD, "zoo")
    os.makedirs(bld, exist_ok=True)
    objs = []
    for s in ["kf_count_zoo.hip", "kf_bucket_zoo.hip"]:
        o = os.path.join(bld, s + ".o")
        subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-DKF_ABLATION",
                        "-DKF_PROFILE_BUILD", "-I", CSRC, "-c", os.path.join(zoo, s), "-o", o]
                       + os.environ.get("KF_HIPCC_FLAGS", "").split(), check=True)
        objs.append(o)
    o = os.path.join(bld, "kf_host.cpp.o")
    subprocess.run(["g++", "-O3", "-std=c++17", "-fPIC", "-pthread", f'-DKF_BUILD_ID="{source_id()}+zoo"',
                    "-c", os.path.join(CSRC, "kf_host.cpp"), "-o", o], check=True)
    objs.append(o)
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", *objs, "-o", out], check=True)
    return out


if __name__ == "__main__":
    if "--zoo" in sys.argv:
        print(build_zoo())
        sys.exit(0)
    if "--sanitize" in sys.argv:
        exe = build_sanitized_host()
        sys.exit(subprocess.run([exe]).returncode)
    abl = "--ablation" in sys.argv
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv, ablation=abl,
                out=os.path.join(HERE, "libkf2vec_gpu_ablation.so") if abl else None))
