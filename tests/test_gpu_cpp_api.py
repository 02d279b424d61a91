"""A native C++ program (examples/dropin_main.cpp) calls the reference's sks::
interface against the library on the GPU: every problem of a golden file (the reference's
own outputs) through all four single-problem functions and the four batch overloads,
bit for bit; then single-problem calls on host and device pointers, the batch overload,
and 8 host threads calling at once, all bit-consistent."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_golden

pytestmark = pytest.mark.gpu


def write_golden_bin(path, n_uniform=64):
    """int64 n, then src/tar/aca/sks in f32, then the same in f64 (dropin_main.cpp's format):
    the first n_uniform problems of cpp_uniform.npz and all 64 edge cases of cpp_edge.npz
    (duplicates, collinear, +-Inf, NaN, subnormals), outputs of the compiled reference."""
    u = load_golden("cpp_uniform.npz")
    e = load_golden("cpp_edge.npz")
    k = n_uniform
    parts32 = [np.concatenate([u["src_f32"][:k], e["src"]]), np.concatenate([u["tar_f32"][:k], e["tar"]]),
               np.concatenate([u["aca_f32"][:k], e["aca"]]), np.concatenate([u["sks_f32"][:k], e["sks"]])]
    parts64 = [np.concatenate([u["src_f64"][:k], e["src_f64"]]),
               np.concatenate([u["tar_f64"][:k], e["tar_f64"]]),
               np.concatenate([u["aca_f64"][:k], e["aca_f64"]]),
               np.concatenate([u["sks_f64"][:k], e["sks_f64"]])]
    n = parts32[0].shape[0]
    with open(path, "wb") as f:
        f.write(np.int64(n).tobytes())
        for a in parts32:
            f.write(np.ascontiguousarray(a, np.float32).tobytes())
        for a in parts64:
            f.write(np.ascontiguousarray(a, np.float64).tobytes())
    return n


def test_cpp_dropin_program(pkg, dev, tmp_path):
    gold = tmp_path / "golden.bin"
    n = write_golden_bin(gold)
    libdir = os.path.dirname(pkg._lib.LIB_PATH)
    exe = tmp_path / "dropin"
    subprocess.run(["g++", "-std=c++17", f"-I{ROOT}/include", "-I/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", f"{ROOT}/examples/dropin_main.cpp",
                    f"-L{libdir}", "-lsks_homography_amd", f"-Wl,-rpath,{libdir}",
                    "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-pthread", "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe), str(gold)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"golden ok: {n} problems" in r.stdout
    assert "dropin ok" in r.stdout


def test_cpp_runtime_harness(pkg, dev, tmp_path):
    """examples/runtime_test.cpp -- the reference GPU harness's flow in native C++ over the
    C ABI: reads the reference's point-file format (written here from the committed
    orig_pts_wall.txt fixture), draws 4*N MRG32K3A words, gathers the 4-subsets on the device
    (get_rand_list), times ACA/SKS/GPT/GE per N, checks ACA against GE, and the fused gather +
    solve and the one-launch draws + gather + solve against gather-then-solve bit for bit."""
    import numpy as np
    from conftest import load_golden
    g = load_golden("cpp_wall.npz")
    pts = tmp_path / "pts.txt"
    with open(pts, "w") as f:
        f.write(f"{g['pool_src'].shape[0]}\n")
        for a, b in zip(g["pool_src"], g["pool_tar"]):
            f.write(" ".join(np.format_float_positional(v, unique=True)
                             for v in (a[0], a[1], b[0], b[1])) + "\n")
    libdir = os.path.dirname(pkg._lib.LIB_PATH)
    exe = tmp_path / "runtime_test"
    subprocess.run(["g++", "-std=c++17", "-O2", f"-I{ROOT}/include", "-I/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", f"{ROOT}/examples/runtime_test.cpp",
                    f"-L{libdir}", "-lsks_homography_amd", f"-Wl,-rpath,{libdir}",
                    "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe), str(pts), "100000", "0.05"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cal_Homo_ACA N=100000" in r.stdout and "cal_Homo_GE  N=100000" in r.stdout
    assert "0 of 900000 words differ from gather-then-solve" in r.stdout, r.stdout
    assert "one launch: 0 of 900000 words differ" in r.stdout, r.stdout


@pytest.mark.parametrize("shards_per_device", [1, 3])
def test_cpp_multi_gpu(pkg, dev, tmp_path, shards_per_device):
    """examples/multi_gpu.cpp -- one native process over every visible GPU through the
    multi-GPU C ABI: per-device blocks generated and solved on their own streams
    (hg_solve_multi), compute-resident throughput for 1, 2, 4 ... devices, then every block
    gathered on device 0 -- RCCL ncclSend / ncclRecv (hg_gather_multi) with one shard per
    device, copies with several -- and compared with one whole-batch solve, bit for bit.  On
    the one-GPU box that is one RCCL rank, or three shards on one device."""
    libdir = os.path.dirname(pkg._lib.LIB_PATH)
    exe = tmp_path / "multi_gpu"
    subprocess.run(["g++", "-std=c++17", "-O2", f"-I{ROOT}/include", "-I/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", f"{ROOT}/examples/multi_gpu.cpp",
                    f"-L{libdir}", "-lsks_homography_multi", "-lsks_homography_amd",
                    f"-Wl,-rpath,{libdir}", "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "1000003", "5", str(shards_per_device)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "solve_multi devices=1:" in r.stdout, r.stdout
    assert "(RCCL" in r.stdout if shards_per_device == 1 else "(copies)" in r.stdout, r.stdout
    assert " 0 of " in r.stdout and "words differ from one whole-batch solve" in r.stdout, r.stdout
