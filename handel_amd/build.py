"""Builds the in-tree HIP library handel_amd/_build/libhandel_gpu.so.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU
container (``__graft_entry__.build()``) and the resulting .so travels to the
GPU box with the repo snapshot. ``diag=True`` builds the separate
diagnostic variant (-DHG_DIAG: in-kernel s_memtime phase counters) used only
by tools/diag.py.
"""

from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "libhandel_gpu.so")
DIAG_LIB = os.path.join(OUT_DIR, "libhandel_gpu_diag.so")
SOURCES = ["bn256_verify.hip", "bn256_pair.hip", "bn256_kernels.hip", "bn256_gt.hip", "bn256_sig12.hip", "bn256_sigw2.hip", "hg_api.cpp",
           "hg_batcher.cpp", "hg_packets.hip", "hg_service.cpp"]
HEADERS = ["bn256_fp.h", "bn256_curve.h", "bn256_team.h", "bn256_kernels.h", "bn256_constants.h",
           "bn256_g2team.h", "bn256_g2sched.h", "bn256_pairing.h", "bn256_xprog.h", "bn256_xtab.h", "bn256_inv.h", "bn256_agg.h", "bn256_gt.h", "bn256_decode.h", "hg_packets.h", "hg_shm.h", "hg_codes.h", "bn256_sigfe.h", "bn256_sigteam.h", "bn256_sigsplit.h"]
ARCH = os.environ.get("HG_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def _inputs():
    files = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    files.append(os.path.join(HERE, "..", "include", "handel_gpu.h"))
    files.append(os.path.abspath(__file__))
    return files


def up_to_date(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return False
    t = os.path.getmtime(lib)
    return all(os.path.getmtime(f) <= t for f in _inputs())


def build_library(force: bool = False, verbose: bool = True, diag: bool = False, variant: str = "",
                  defs: tuple = ()) -> str:
    """variant: an A/B build (tools/ab_variants.sh) with extra -D defs, written
    to _build/variants/libhandel_gpu_<variant>.so; never loaded by default."""
    lib = DIAG_LIB if diag else LIB
    if variant:
        lib = os.path.join(OUT_DIR, "variants", f"libhandel_gpu_{variant}.so")
    if not force and not variant and up_to_date(lib):
        return lib
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    suffix = "_diag" if diag else (f"_{variant}" if variant else "")
    extra = (["-DHG_DIAG=1"] if diag else []) + [f"-D{d}" for d in defs]

    def compile_one(src):
        obj = os.path.join(OUT_DIR, os.path.splitext(src)[0] + suffix + ".o")
        cmd = [HIPCC, *CFLAGS, *extra, "-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        return obj

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = lib + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, lib)
    return lib


CLIENT_LIB = os.path.join(OUT_DIR, "libhandel_client.so")


def build_client(force: bool = False, verbose: bool = True) -> str:
    """libhandel_client.so: the verifier service's client side (hg_client.cpp,
    include/handel_client.h), host compiler only — no HIP runtime, so client
    processes never touch the GPU."""
    srcs = [os.path.join(CSRC, "hg_client.cpp"), os.path.join(CSRC, "hg_shm.h"), os.path.join(CSRC, "hg_codes.h"),
            os.path.join(HERE, "..", "include", "handel_client.h"), os.path.join(HERE, "..", "include", "handel_gpu.h"),
            os.path.abspath(__file__)]
    if not force and os.path.exists(CLIENT_LIB) and os.path.getmtime(CLIENT_LIB) >= max(map(os.path.getmtime, srcs)):
        return CLIENT_LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = CLIENT_LIB + ".tmp"
    cmd = ["g++", "-O2", "-fPIC", "-shared", "-std=c++17", "-Wall", "-Wextra", srcs[0], "-lpthread", "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, CLIENT_LIB)
    return CLIENT_LIB


VERIFIERD = os.path.join(OUT_DIR, "hg_verifierd")


def build_verifierd(verbose: bool = True) -> str:
    """hg_verifierd: the GPU-owning verifier process (hg_service_* over one
    context) a single-host simul run starts once; links libhandel_gpu.so."""
    src = os.path.join(CSRC, "hg_verifierd.cpp")
    hdr = os.path.join(HERE, "..", "include", "handel_gpu.h")
    if os.path.exists(VERIFIERD) and os.path.getmtime(VERIFIERD) >= max(map(os.path.getmtime, [src, hdr, LIB])):
        return VERIFIERD
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", src, "-L", OUT_DIR, "-lhandel_gpu", "-lpthread",
           "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib", "-Wl,-rpath,$ORIGIN", "-o", VERIFIERD]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return VERIFIERD


ABI_THREADS = os.path.join(OUT_DIR, "abi_threads")


def build_native_tests(verbose: bool = True) -> str:
    """tests/native/abi_threads.c (the C-level thread-safety test of the ABI),
    linked against the in-tree library only through include/handel_gpu.h. A
    test harness, not product code: built here so the GPU box runs it as is."""
    src = os.path.join(HERE, "..", "tests", "native", "abi_threads.c")
    if os.path.exists(ABI_THREADS) and os.path.getmtime(ABI_THREADS) >= max(os.path.getmtime(src),
                                                                           os.path.getmtime(LIB)):
        return ABI_THREADS
    cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-I", os.path.join(HERE, "..", "include"), src,
           "-L", OUT_DIR, "-lhandel_gpu", "-lpthread", "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib",
           "-Wl,-rpath,$ORIGIN", "-o", ABI_THREADS]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return ABI_THREADS


HANDEL_PROXY = os.path.join(OUT_DIR, "handel_proxy")


def build_proxy(verbose: bool = True) -> str:
    """tests/native/handel_proxy.c: the config-4 process-model proxy (forks
    the processes first, each dlopen()s the library: never linked here)."""
    src = os.path.join(HERE, "..", "tests", "native", "handel_proxy.c")
    hdrs = [os.path.join(HERE, "..", "include", h) for h in ("handel_gpu.h", "handel_client.h")]
    if os.path.exists(HANDEL_PROXY) and os.path.getmtime(HANDEL_PROXY) >= max(map(os.path.getmtime, [src, *hdrs])):
        return HANDEL_PROXY
    os.makedirs(OUT_DIR, exist_ok=True)
    cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-I", os.path.join(HERE, "..", "include"), src, "-ldl",
           "-lpthread", "-o", HANDEL_PROXY]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return HANDEL_PROXY


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, diag="--diag" in sys.argv))
    if "--diag" not in sys.argv:
        print(build_client())
        print(build_verifierd())
        print(build_native_tests())
        print(build_proxy())
