"""Builds the product library sks-homography_amd/lib/libsks_homography_amd.so.

hipcc, gfx950 only.  Numerics flags are part of the contract, not tuning:
  -ffp-contract=off   every product/sum rounded on its own (bit parity with the
                      reference's x86 SSE build); hg_solvers.hpp also pins this
                      with `#pragma clang fp contract(off)`.
  no -ffast-math      IEEE division (v_div_scale/fmas/fixup), NaN/Inf preserved.
"""
from __future__ import annotations

import concurrent.futures
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libsks_homography_amd.so")
TORCH_LIB = os.path.join(LIB_DIR, "libsks_homography_torch.so")
TUNE_LIB = os.path.join(LIB_DIR, "libsks_homography_tune.so")
ARCH = os.environ.get("SKS_AMD_ARCH", "gfx950")

SOURCES = ["hg_kernels.hip", "hg_ransac.hip", "hg_table8.hip", "hg_sks_api.cpp", "hg_host.cpp"]
# kernel-variant sweeps and timing loops (tools/, tests): a separate library so the product
# library carries only the shipped kernels
TUNE_SOURCES = ["hg_tune.hip"]
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
          f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}"]


# The sources a kernel's measured HBM traffic depends on (profiles/pmc_traffic.json records
# their digest; bench.py reports the PMC figure only while the tree still matches it).
TRAFFIC_SOURCES = {
    "aos": ["csrc/hg_aos.hpp", "csrc/hg_solvers.hpp", "csrc/hg_launch.hpp", "csrc/hg_kernels.hip"],
}


def sources_digest(kind: str = "aos") -> dict:
    """sha256 of each file of TRAFFIC_SOURCES[kind] (paths relative to the package) and of
    their concatenation, in a fixed order."""
    import hashlib
    files, whole = {}, hashlib.sha256()
    for rel in TRAFFIC_SOURCES[kind]:
        data = open(os.path.join(HERE, rel), "rb").read()
        files[rel] = hashlib.sha256(data).hexdigest()[:16]
        whole.update(rel.encode() + b"\0" + data)
    flags = " ".join([f"--offload-arch={ARCH}"] + COMMON[:5])  # not the -I paths
    whole.update(flags.encode())
    return {"files": files, "flags": flags, "sha256": whole.hexdigest()[:16]}


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the MI355X library cannot be built")


def _stale(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    cc = hipcc()
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    headers += [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
    headers.append(os.path.abspath(__file__))  # a flag change here rebuilds every object
    objs, tune_objs, cmds = [], [], []
    for src in SOURCES + TUNE_SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(BUILD, os.path.splitext(src)[0] + ".o")
        (tune_objs if src in TUNE_SOURCES else objs).append(obj)
        if not force and not _stale(obj, [path] + headers):
            continue
        cmd = [cc, *COMMON, "-c", path, "-o", obj]
        if src.endswith(".hip"):
            # SLP vectoriser left on: built without it, the library's seeded sampler is 8 %
            # slower, the indexed one 2 % faster, the rest unchanged, bits identical
            # (tools/slp_ab.py, profiles/r01/slp_ab.json)
            cmd[1:1] = [f"--offload-arch={ARCH}"]
        else:
            cmd[1:1] = ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        if verbose:
            print(" ".join(cmd))
        cmds.append(cmd)
    # the translation units are independent: compile them side by side (at most 4 at once)
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(4, max(1, len(cmds)))) as ex:
        for f in [ex.submit(subprocess.run, c, check=True) for c in cmds]:
            f.result()
    if force or _stale(LIB, objs):
        cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    if force or _stale(TUNE_LIB, tune_objs + [LIB]):
        # rocRAND: the checker of the hand-written MRG32K3A generator (hg_tune.hip)
        cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", TUNE_LIB, *tune_objs,
               f"-L{LIB_DIR}", "-lsks_homography_amd", "-Wl,-rpath,$ORIGIN",
               "-L/opt/rocm/lib", "-lrocrand", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    build_torch_ops(verbose, force, headers)
    return LIB


def build_torch_ops(verbose: bool = False, force: bool = False, headers=()) -> str:
    """lib/libsks_homography_torch.so: the native torch.ops.sks_amd operators
    (csrc/hg_torch_ops.cpp), host C++ against torch's headers, linked to the product
    library (found next to it via $ORIGIN)."""
    import torch

    src = os.path.join(CSRC, "hg_torch_ops.cpp")
    if not force and not _stale(TORCH_LIB, [src, LIB, *headers]):
        return TORCH_LIB
    tdir = os.path.dirname(torch.__file__)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", TORCH_LIB, src,
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=sks_homography_torch",
           f"-I{os.path.join(ROOT, 'include')}", f"-I{os.path.join(tdir, 'include')}",
           f"-I{os.path.join(tdir, 'include', 'torch', 'csrc', 'api', 'include')}",
           "-I/opt/rocm/include", f"-L{os.path.join(tdir, 'lib')}", f"-L{LIB_DIR}",
           "-lsks_homography_amd", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
           "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{os.path.join(tdir, 'lib')}"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return TORCH_LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
