"""Build the native pieces of crossbow_amd in-tree.

* ``crossbow_amd/libcrossbow_sma.so``  -- the C-ABI library (hipcc, gfx950):
  csrc/context.hip + csrc/sync_steps.hip + csrc/sma_kernels.hip + csrc/sma_seam.hip,
  linked against RCCL.
* ``crossbow_amd/libGPU.so``           -- the JNI shim exporting Crossbow's
  ``TheGPU`` model-path natives; built only where ``jni.h`` exists (there is
  no JDK in this image).

Usage: ``python -m crossbow_amd.build [--force]``.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libcrossbow_sma.so")
JNI_LIB = os.path.join(PKG, "libGPU.so")
ARCH = "gfx950"


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the MI355X library needs ROCm's hipcc")


SOURCES = ("context.hip", "sync_steps.hip", "sma_kernels.hip", "sma_seam.hip")
HEADERS = ("context_internal.h", "sma_internal.h")


def _sources():
    return [os.path.join(CSRC, f) for f in SOURCES]


def _deps():
    return _sources() + [os.path.join(CSRC, f) for f in HEADERS] + [os.path.join(ROOT, "include", "crossbow_sma.h"),
                                                                   os.path.abspath(__file__)]


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale(LIB, _deps()):
        return LIB
    tmp = LIB + ".tmp"
    objdir = os.path.join(PKG, "build")
    os.makedirs(objdir, exist_ok=True)
    objs = []
    for src in _sources():
        stem = os.path.splitext(os.path.basename(src))[0]
        obj = os.path.join(objdir, stem + ".o")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               # A fixed compilation-unit id per source instead of one hashed from
               # its path: the device code (and code_object_digest) is then the
               # same wherever the tree is built.
               f"-cuid=crossbow_{stem}",
               # fp32 results must equal the reference's cuBLAS op order bit for bit: every
               # fma is written explicitly, nothing may be contracted behind our back.
               "-ffp-contract=off",
               "-I", os.path.join(ROOT, "include"), "-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-o", tmp] + objs + \
        ["-lrccl", "-lrocprofiler-sdk-roctx", "-lpthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


def code_object_digest(path: str = LIB) -> str:
    """sha256 of the library's device code (its ``.hip_fatbin`` section: the
    gfx950 code objects of every kernel).  profiles/traffic.json stores it
    with each PMC measurement, and bench.py reports a measured HBM traffic
    only for the code object that is running (else null, with the reason)."""
    import hashlib
    import struct
    with open(path, "rb") as f:
        elf = f.read()
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        raise ValueError(f"{path}: not an ELF64 file")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)

    def section(i):
        name, _, _, _, off, size = struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize)
        return name, off, size

    _, stroff, _ = section(shstrndx)
    for i in range(shnum):
        name, off, size = section(i)
        end = elf.index(b"\0", stroff + name)
        if elf[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(elf[off:off + size]).hexdigest()
    raise ValueError(f"{path}: no .hip_fatbin section")


def find_jni_include():
    cands = []
    jh = os.environ.get("JAVA_HOME")
    if jh:
        cands.append(os.path.join(jh, "include"))
    cands += glob.glob("/usr/lib/jvm/*/include")
    for c in cands:
        if os.path.exists(os.path.join(c, "jni.h")):
            return c
    return None


def build_jni(force: bool = False, verbose: bool = False):
    """Build libGPU.so (the JNI drop-in) when a JDK is present; else None."""
    inc = find_jni_include()
    if inc is None:
        return None
    src = os.path.join(CSRC, "jni", "TheGPU_jni.c")
    if not force and not _stale(JNI_LIB, [src, LIB]):
        return JNI_LIB
    cmd = ["gcc", "-O2", "-fPIC", "-shared", "-I", inc, "-I", os.path.join(inc, "linux"),
           "-I", os.path.join(ROOT, "include"), "-o", JNI_LIB, src, "-L", PKG, "-lcrossbow_sma",
           "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return JNI_LIB


def build(force: bool = False, verbose: bool = False) -> str:
    lib = build_lib(force, verbose)
    build_jni(force, verbose)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
