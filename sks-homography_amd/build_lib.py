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
MULTI_LIB = os.path.join(LIB_DIR, "libsks_homography_multi.so")
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


# The headline kernels whose HBM traffic profiles/pmc_traffic.json records, by the mangled
# name of their gfx950 entry point (hg::solve_aos<ALGO, true, float, 2, 39>).
TRAFFIC_KERNELS = {
    "aca_f32_aos_norm": "_ZN2hg9solve_aosILi0ELb1EfLi2ELi39EEEvPKT1_S3_PS1_l",
    "sks_f32_aos_norm": "_ZN2hg9solve_aosILi1ELb1EfLi2ELi39EEEvPKT1_S3_PS1_l",
}


def _elf_sections(b: bytes, base: int = 0) -> dict:
    """{name: (sh_addr, sh_offset, sh_size)} of the little-endian ELF64 image at b[base:]."""
    import struct
    shoff = struct.unpack_from("<Q", b, base + 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, base + 0x3A)
    raw = [struct.unpack_from("<IIQQQQ", b, base + shoff + i * shentsize) for i in range(shnum)]
    strtab_off = base + raw[shstrndx][4]
    out = {}
    for name, _typ, _flags, addr, off, size in raw:
        end = b.index(b"\0", strtab_off + name)
        out[b[strtab_off + name:end].decode()] = (addr, base + off, size)
    return out


def kernel_code_digest(lib_path: str = None) -> dict:
    """sha256 (16 hex digits) of the gfx950 machine code of each TRAFFIC_KERNELS entry point,
    read from the built library: the HIP fat binary's offload bundles (.hip_fatbin), the gfx950
    code object in each, that object's symbol table and .text.  What ran is what is hashed, so
    edits that leave the kernel's code unchanged keep its measured traffic valid."""
    import hashlib
    import struct
    b = open(lib_path or LIB, "rb").read()
    _, fat_off, fat_size = _elf_sections(b)[".hip_fatbin"]
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    found = {}
    pos = b.find(magic, fat_off, fat_off + fat_size)
    while pos >= 0:
        count = struct.unpack_from("<Q", b, pos + 24)[0]
        q = pos + 32
        for _ in range(count):
            off, size, idlen = struct.unpack_from("<QQQ", b, q)
            ident = b[q + 24:q + 24 + idlen].decode()
            q += 24 + idlen
            if ARCH not in ident or size == 0:
                continue
            co = pos + off
            secs = _elf_sections(b, co)
            sym_addr, sym_off, sym_size = secs[".symtab"]
            str_off = secs[".strtab"][1]
            text_addr, text_off, _ = secs[".text"]
            for k in range(sym_size // 24):
                st_name, _info, _other, _shndx, value, sz = struct.unpack_from("<IBBHQQ", b, sym_off + 24 * k)
                name = b[str_off + st_name:b.index(b"\0", str_off + st_name)].decode()
                for key, mangled in TRAFFIC_KERNELS.items():
                    if name == mangled and sz:
                        start = text_off + (value - text_addr)
                        found[key] = hashlib.sha256(b[start:start + sz]).hexdigest()[:16]
        pos = b.find(magic, pos + 24, fat_off + fat_size)
    missing = set(TRAFFIC_KERNELS) - set(found)
    if missing:
        raise RuntimeError(f"{lib_path or LIB}: no gfx950 code for {sorted(missing)}")
    return found


def device_code_digests(lib_path: str = None) -> dict:
    """{mangled kernel name: sha256 (16 hex digits) of its gfx950 machine code} for every
    function symbol in the library's gfx950 code objects (kernel_code_digest's walk, all
    symbols whose address lies in .text)."""
    import hashlib
    import struct
    b = open(lib_path or LIB, "rb").read()
    _, fat_off, fat_size = _elf_sections(b)[".hip_fatbin"]
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    found = {}
    pos = b.find(magic, fat_off, fat_off + fat_size)
    while pos >= 0:
        count = struct.unpack_from("<Q", b, pos + 24)[0]
        q = pos + 32
        for _ in range(count):
            off, size, idlen = struct.unpack_from("<QQQ", b, q)
            ident = b[q + 24:q + 24 + idlen].decode()
            q += 24 + idlen
            if ARCH not in ident or size == 0:
                continue
            co = pos + off
            secs = _elf_sections(b, co)
            _, sym_off, sym_size = secs[".symtab"]
            str_off = secs[".strtab"][1]
            text_addr, text_off, text_size = secs[".text"]
            for k in range(sym_size // 24):
                st_name, _info, _other, _shndx, value, sz = struct.unpack_from("<IBBHQQ", b, sym_off + 24 * k)
                if not sz or not (text_addr <= value < text_addr + text_size):
                    continue
                name = b[str_off + st_name:b.index(b"\0", str_off + st_name)].decode()
                start = text_off + (value - text_addr)
                found[name] = hashlib.sha256(b[start:start + sz]).hexdigest()[:16]
        pos = b.find(magic, pos + 24, fat_off + fat_size)
    return found


def demangle(names) -> dict:
    """{mangled: demangled} through binutils' c++filt (on this image and the GPU box)."""
    names = list(names)
    tool = shutil.which("c++filt") or shutil.which("llvm-cxxfilt") or "/usr/bin/c++filt"
    out = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.splitlines()
    return dict(zip(names, out))


def kernel_family_digest(prefix: str, lib_path: str = None) -> str:
    """One digest over the machine code of every kernel whose demangled name contains
    `prefix` (the PMC reducer's match): a changed kernel changes it."""
    import hashlib
    codes = device_code_digests(lib_path)
    names = demangle(codes)
    hit = sorted(codes[m] for m, d in names.items() if prefix in d)
    return hashlib.sha256(",".join(hit).encode()).hexdigest()[:16] if hit else ""


def compiler_id() -> str:
    """The first line of `hipcc --version` (the machine code depends on it, not only on the
    source): recorded beside every machine-code digest."""
    try:
        out = subprocess.run([hipcc(), "--version"], capture_output=True, text=True, timeout=60)
        lines = (out.stdout or out.stderr).strip().splitlines()
        return "; ".join([lines[0]] + [x.strip() for x in lines if "clang version" in x][:1])
    except Exception as e:  # noqa: BLE001
        return f"unknown ({type(e).__name__})"


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
    build_multi(verbose, force, headers)
    return LIB


def build_multi(verbose: bool = False, force: bool = False, headers=()) -> str:
    """lib/libsks_homography_multi.so: the multi-GPU C ABI (csrc/hg_multi.cpp,
    include/sks_homography_multi.h), host C++ over the product library and librccl -- kept
    apart so the product library has no RCCL dependency."""
    src = os.path.join(CSRC, "hg_multi.cpp")
    if not force and not _stale(MULTI_LIB, [src, LIB, *headers]):
        return MULTI_LIB
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", MULTI_LIB, src,
           "-D__HIP_PLATFORM_AMD__=1", f"-I{os.path.join(ROOT, 'include')}", "-I/opt/rocm/include",
           f"-L{LIB_DIR}", "-lsks_homography_amd", "-L/opt/rocm/lib", "-lamdhip64", "-lrccl",
           "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return MULTI_LIB


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
