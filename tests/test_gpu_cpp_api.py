"""A native C++ program (examples/dropin_main.cpp) calls the reference's sks::
interface against the library on the GPU: single-problem calls on host and device
pointers, the batch overload, and 8 host threads calling at once, all bit-consistent."""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_cpp_dropin_program(pkg, dev, tmp_path):
    libdir = os.path.dirname(pkg._lib.LIB_PATH)
    exe = tmp_path / "dropin"
    subprocess.run(["g++", "-std=c++17", f"-I{ROOT}/include", "-I/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", f"{ROOT}/examples/dropin_main.cpp",
                    f"-L{libdir}", "-lsks_homography_amd", f"-Wl,-rpath,{libdir}",
                    "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-pthread", "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "dropin ok" in r.stdout
