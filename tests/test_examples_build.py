"""The native C++ examples compile and link against the in-tree libraries on the build host
(no GPU needed); tests/test_gpu_cpp_api.py runs them on the GPU box."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

LIBDIR = os.path.join(ROOT, "sks-homography_amd", "lib")
EXAMPLES = {
    "dropin_main.cpp": ["-lsks_homography_amd"],
    "runtime_test.cpp": ["-lsks_homography_amd"],
    "multi_gpu.cpp": ["-lsks_homography_multi", "-lsks_homography_amd"],
}


@pytest.mark.parametrize("name", sorted(EXAMPLES))
def test_example_builds(name, tmp_path):
    if shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"):
        pytest.skip("needs g++ and the ROCm headers")
    libs = EXAMPLES[name]
    for lib in libs:
        so = os.path.join(LIBDIR, f"lib{lib[2:]}.so")
        if not os.path.exists(so):
            pytest.skip(f"{so} not built (run __graft_entry__.build())")
    exe = tmp_path / name[:-4]
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", f"-I{ROOT}/include",
                        "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
                        os.path.join(ROOT, "examples", name), f"-L{LIBDIR}", *libs,
                        f"-Wl,-rpath,{LIBDIR}", "-L/opt/rocm/lib", "-lamdhip64",
                        "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert exe.exists()
