"""The C-ABI library loads (no GPU needed) and exports every symbol include/*.h
declares; argument validation happens before any HIP call.  CPU only."""
import ctypes
import os
import re
import subprocess
import sys
import tempfile

import pytest

from conftest import ROOT

INCLUDE = os.path.join(ROOT, "include")


def _c_decls(header="sks_homography.h"):
    text = open(os.path.join(INCLUDE, header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hg_\w+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    decls = _c_decls()
    for name in ("hg_aca_f32", "hg_aca_f64", "hg_sks_f32", "hg_sks_f64",
                 "hg_tensor_aca_rect_f32", "hg_fill_uniform_f32", "hg_version"):
        assert name in decls


def test_library_exports_every_c_symbol(pkg):
    lib = pkg.lib()
    for name in _c_decls():
        assert hasattr(lib, name), f"{name} declared in sks_homography.h but not exported"
    assert set(_c_decls()) == set(pkg._lib.SIGNATURES), "ctypes table out of sync with header"


def test_tune_library_exports_its_header(pkg):
    """include/sks_homography_tune.h (kernel-variant sweeps, timing loops) is served by
    lib/libsks_homography_tune.so; the product library carries none of it."""
    tune, lib = pkg._lib.tune(), pkg.lib()
    decls = _c_decls("sks_homography_tune.h")
    assert decls
    for name in decls:
        assert hasattr(tune, name), f"{name} declared in sks_homography_tune.h but not exported"
        assert not hasattr(lib, name), f"{name} leaked into the product library"


def test_cpp_api_links_against_library(pkg):
    """Every declaration of include/sks_aca_sks.hpp (the reference's sks:: interface)
    resolves when a C++ program is linked against the library."""
    prog = r"""
    #include "sks_aca_sks.hpp"
    #include <cstdio>
    int main(int argc, char**) {
        void* f[] = {(void*)&sks::runKernel_ACA, (void*)&sks::runKernel_ACA_double,
                     (void*)&sks::runKernel_SKS, (void*)&sks::runKernel_SKS_double,
                     (void*)&sks::runKernel_ACA_batch, (void*)&sks::runKernel_ACA_double_batch,
                     (void*)&sks::runKernel_SKS_batch, (void*)&sks::runKernel_SKS_double_batch,
                     (void*)&hg_aca_f32, (void*)&hg_sks_f64, (void*)&hg_version};
        if (argc > 5) std::printf("%p", f[0]);
        // argument validation returns before touching the GPU
        return sks::runKernel_ACA_batch(nullptr, nullptr, nullptr, -1) == 1 ? 0 : 3;
    }
    """
    libdir = os.path.dirname(pkg._lib.LIB_PATH)
    with tempfile.TemporaryDirectory() as d:
        cpp = os.path.join(d, "t.cpp")
        exe = os.path.join(d, "t")
        open(cpp, "w").write(prog)
        subprocess.run(["g++", "-std=c++17", f"-I{INCLUDE}", cpp, f"-L{libdir}",
                        "-lsks_homography_amd", f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
        assert subprocess.run([exe]).returncode == 0


@pytest.mark.parametrize("fn", ["hg_aca_f32", "hg_aca_f64", "hg_sks_f32", "hg_sks_f64"])
def test_argument_validation_without_gpu(pkg, fn):
    lib = pkg.lib()
    f = getattr(lib, fn)
    INVALID = 1  # hipErrorInvalidValue
    assert f(None, None, None, -1, 0, 0, None) == INVALID      # n < 0
    assert f(None, None, None, 0, 0, 0, None) == 0             # empty batch: no-op
    assert f(None, None, None, 5, 0, 0, None) == INVALID       # NULL with n > 0
    assert f(None, None, None, 5, 7, 0, None) == INVALID       # unknown layout
    assert f(None, None, None, 5, 0, 6, None) == INVALID       # unknown flag bits
    assert f(None, None, None, 0, 2, 0, None) == INVALID       # layout checked first


def test_other_entry_validation(pkg):
    lib = pkg.lib()
    assert lib.hg_tensor_aca_rect_f32(None, None, None, -1, None, None, None) == 1
    assert lib.hg_tensor_aca_rect_f32(None, None, None, 0, None, None, None) == 0
    assert lib.hg_tensor_aca_rect_f32(None, None, None, 4, None, None, None) == 1
    assert lib.hg_tensor_aca_rect_f32_hostscalar(None, None, None, 4, 1.0, 1.0, None) == 1
    assert lib.hg_fill_uniform_f32(None, -3, 0, 0, 0.0, 1.0, None) == 1
    assert lib.hg_fill_uniform_f32(None, 0, 0, 0, 0.0, 1.0, None) == 0
    assert lib.hg_sample_solve_f32(None, None, 0, None, None, 4, 0, 0, None) == 1  # npool 0
    assert lib.hg_sample_solve_f32(None, None, 5, None, None, 4, 9, 0, None) == 1  # algo
    assert lib.hg_sample_solve_f32(None, None, 5, 8, 16, 4, 0, 0, None) == 1      # unaligned idx
    assert lib.hg_fill_bits_u32(None, -1, 0, 0, None) == 1
    assert lib.hg_sample_solve_seeded_f32(None, None, 0, 1, 0, None, 4, 0, 0, None) == 1  # npool 0
    assert lib.hg_sample_solve_seeded_f32(None, None, 5, 1, 0, None, 4, 2, 0, None) == 1  # algo
    assert lib.hg_sample_solve_seeded_f32(None, None, 5, 1, 0, None, 4, 0, 4, None) == 1  # flags
    assert lib.hg_sample_solve_seeded_f32(None, None, 5, 1, 0, None, -1, 0, 0, None) == 1  # n < 0
    assert lib.hg_sample_solve_seeded_f32(None, None, 5, 1, 0, None, 0, 0, 0, None) == 0  # empty
    assert lib.hg_sample_solve_seeded_f32(None, None, 5, 1, 0, None, 4, 0, 0, None) == 1  # NULL
    assert lib.hg_sample_solve_seeded_f32(8, 8, 5, 1, 0, 8, 4, 0, 0, None) == 1  # H unaligned
    assert lib.hg_fill_bits_u32(None, 0, 0, 0, None) == 0
    assert lib.hg_ransac_score_f32(None, -1, None, None, 0, 1.0, None, None) == 1
    assert lib.hg_ransac_score_f32(None, 0, None, None, 0, 1.0, None, None) == 0
    assert lib.hg_ransac_score_f32(None, 3, None, None, 0, 1.0, None, None) == 1
    assert lib.hg_tensor_aca_offsets_f32(None, None, None, -2, 1.0, 1.0, None) == 1
    assert lib.hg_tensor_aca_offsets_f32(None, None, None, 0, 1.0, 1.0, None) == 0
    assert lib.hg_tensor_aca_offsets_backward_f32(None, None, None, 3, 1.0, 1.0, None, None,
                                                  None) == 1
    # the Table-8 pipeline entry points (hg_table8.hip)
    assert lib.hg_rand_mrg32k3a_u32(None, -1, 11, None) == 1
    assert lib.hg_rand_mrg32k3a_u32(None, 0, 11, None) == 0
    assert lib.hg_rand_mrg32k3a_u32(None, 4, 11, None) == 1                       # NULL
    assert lib.hg_rand_mrg32k3a_u32(2, 4, 11, None) == 1                          # unaligned
    assert lib.hg_get_rand_list_f64(None, 0, None, None, None, None, 4, None) == 1  # size 0
    assert lib.hg_get_rand_list_f64(None, 5, None, None, None, None, -1, None) == 1
    assert lib.hg_get_rand_list_f64(None, 5, None, None, None, None, 0, None) == 0
    assert lib.hg_get_rand_list_f64(None, 5, None, None, None, None, 4, None) == 1
    assert lib.hg_get_rand_list_f64(16, 5, 8, 16, 16, 16, 4, None) == 1            # pool not 16-B
    for algo, flags, n, want in ((4, 0, 4, 1), (-1, 0, 4, 1), (0, 2, 4, 1), (0, 0, -1, 1),
                                 (3, 1, 0, 0), (0, 0, 4, 1)):
        assert lib.hg_gather_solve_f64(algo, None, None, 5, None, None, n, flags, None) == want
    assert lib.hg_gather_solve_f64(0, None, None, 0, None, None, 4, 0, None) == 1  # size 0
    assert lib.hg_gather_solve_f64(0, 16, 16, 5, 16, 4, 4, 0, None) == 1           # H unaligned
    for algo, flags, n, want in ((4, 0, 4, 1), (-1, 0, 4, 1), (0, 2, 4, 1), (0, 0, -1, 1),
                                 (3, 1, 0, 0), (0, 0, 4, 1), (0, 0, (1 << 61) + 1, 1)):
        assert lib.hg_rand_gather_solve_f64(algo, None, None, 5, 11, None, n, flags, None) == want
    assert lib.hg_rand_gather_solve_f64(0, None, None, 0, 11, None, 4, 0, None) == 1  # size 0
    assert lib.hg_rand_gather_solve_f64(0, 16, 8, 5, 11, 16, 4, 0, None) == 1  # pool not 16-B
    assert lib.hg_rand_gather_solve_f64(0, 16, 16, 5, 11, 4, 4, 0, None) == 1  # H unaligned
    assert lib.hg_mrg32k3a_state(11, 0, 0, None) == 1                             # NULL state
    assert lib.hg_tensor_aca_rect_bcast_f32(None, None, None, -1, None, 0, 0, None, 0, 0, None) == 1
    assert lib.hg_tensor_aca_rect_bcast_f32(None, None, None, 0, None, 0, 0, None, 0, 0, None) == 0
    assert lib.hg_tensor_aca_rect_bcast_f32(None, None, None, 4, None, 0, 0, None, 0, 0, None) == 1
    assert lib.hg_tensor_aca_rect_bcast_backward_f32(None, None, None, 3, None, 0, 0, None, 0, 0,
                                                     None, None, None, 0, None, 0, None) == 1
    for fn in (lib.hg_tensor_aca_rect_backward_f32, lib.hg_tensor_aca_rect_backward_terms_f32):
        assert fn(None, None, None, 3, None, None, None, None, None, None) == 1
        assert fn(None, None, None, 0, None, None, None, None, None, None) == 0
        assert fn(None, None, None, -1, None, None, None, None, None, None) == 1
    # the evaluation-order entry points: HG_ORDER_ATEN_CPU (0) is the bcast form, ROCM (1) its
    # own launch; anything else is refused before a pointer is looked at
    for order in (0, 1):
        assert lib.hg_tensor_aca_rect_order_f32(None, None, None, 0, None, 0, 0, None, 0, 0, order,
                                                None) == 0
        assert lib.hg_tensor_aca_rect_order_f32(None, None, None, -1, None, 0, 0, None, 0, 0, order,
                                                None) == 1
        assert lib.hg_tensor_aca_rect_order_f32(None, None, None, 4, None, 0, 0, None, 0, 0, order,
                                                None) == 1
        assert lib.hg_tensor_aca_rect_backward_order_f32(
            None, None, None, 0, None, 0, 0, None, 0, 0, None, None, None, 0, None, 0, order, None) == 0
        assert lib.hg_tensor_aca_rect_backward_order_f32(
            None, None, None, 3, None, 0, 0, None, 0, 0, None, None, None, 0, None, 0, order, None) == 1
        assert lib.hg_tensor_aca_rect_backward_order_f32(                           # scale mode 3
            8, 8, 8, 3, 8, 0, 0, 8, 0, 0, None, 8, 8, 3, 8, 0, order, None) == 1
    for order in (2, -1):
        assert lib.hg_tensor_aca_rect_order_f32(16, 16, 16, 4, 16, 0, 0, 16, 0, 0, order, None) == 1
        assert lib.hg_tensor_aca_rect_backward_order_f32(
            16, 16, 16, 3, 16, 0, 0, 16, 0, 0, None, 16, None, 0, None, 0, order, None) == 1
    assert lib.hg_solve_one_f32(0, None, None, None, 1, None) == 1               # NULL points
    assert lib.hg_solve_one_f64(2, None, None, None, 1, None) == 1               # algo 2
    assert lib.hg_sum_rows_f32(None, -1, 5, None, None) == 1                      # rows < 0
    assert lib.hg_sum_rows_f32(None, 0, 5, None, None) == 0                       # nothing to do
    assert lib.hg_sum_rows_f32(None, 2, 5, None, None) == 1                       # NULL x / out
    assert lib.hg_sum_rows_f32(None, 70000, 5, None, None) == 1                   # rows > 65535
    assert lib.hg_sum_aten_f32(None, 0, 5, 5, 1, 8, 1, None, None) == 0           # no rows
    assert lib.hg_sum_aten_f32(None, 1, 5, 5, 1, 8, 1, None, None) == 1           # NULL x / out
    assert lib.hg_sum_aten_f32(None, 1, 5, 5, 1, 0, 1, None, None) == 1           # lanes 0
    assert lib.hg_sum_aten_f32(None, 1, 5, 5, 1, 17, 1, None, None) == 1          # lanes > 16
    assert lib.hg_sum_aten_f32(None, 1, 5, 5, 1, 8, 1025, None, None) == 1        # threads
    assert lib.hg_sum_aten_f32(None, 1, 5, 5, 1, 1, 2, None, None) == 1           # chunked 1 lane
    assert lib.hg_sum_aten_f32(None, 70000, 5, 5, 1, 8, 1, None, None) == 1       # runs > 65535
    assert lib.hg_sample_solve_f32(None, None, 0, None, None, 5, 0, 1, None) == 1  # npool 0
    assert lib.hg_sample_solve_f32(None, None, 9, None, None, 5, 7, 1, None) == 1  # algo 7
    assert lib.hg_ransac_score_f32(None, -1, None, None, 9, 1.0, None, None) == 1
    assert lib.hg_fill_bits_u32(None, 5, 0, 0, None) == 1
    assert lib.hg_fill_bits_u32(None, 0, 0, 0, None) == 0
    assert lib.hg_stream_copy(None, None, 17, None) == 1                          # not x16
    assert lib.hg_stream_copy(None, None, 0, None) == 0
    # host-resident batches: every check before the first HIP call
    for f in (lib.hg_solve_host_f32, lib.hg_solve_host_f64):
        assert f(0, None, None, None, -1, 0, 1, None) == 1                      # n < 0
        assert f(0, None, None, None, 0, 0, 1, None) == 0                       # empty
        assert f(0, None, None, None, 5, 0, 1, None) == 1                       # NULL
        assert f(-1, None, None, None, 0, 0, 1, None) == 1                      # algo
        assert f(0, None, None, None, 0, 2, 1, None) == 1                       # layout
        assert f(0, None, None, None, 0, 0, 4, None) == 1                       # flags
        assert f(0, None, None, None, 0, 0, 1 | 2, None) == 0                   # HOST_REGISTER ok
    assert lib.hg_solve_host_f32(3, None, None, None, 0, 0, 1, None) == 1       # GPT: f64 only
    assert lib.hg_solve_host_f64(3, None, None, None, 0, 0, 1, None) == 0
    assert lib.hg_solve_host_f64(4, None, None, None, 0, 0, 1, None) == 1
    for f in (lib.hg_solve_grouped_f32, lib.hg_solve_grouped_f64):  # grouped: checks first
        assert f(0, None, None, None, None, 0, 0, 1, None) == 0                 # no batches
        assert f(0, None, None, None, None, -1, 0, 1, None) == 1                # count < 0
        assert f(0, None, None, None, None, 3, 0, 1, None) == 1                 # NULL arrays
        assert f(9, None, None, None, None, 0, 0, 1, None) == 1                 # algo
        assert f(0, None, None, None, None, 0, 5, 1, None) == 1                 # layout
        assert f(0, None, None, None, None, 0, 0, 4, None) == 1                 # flags
        P = ctypes.c_void_p * 2
        n = (ctypes.c_int64 * 2)(4, -1)
        assert f(0, P(1, 1), P(1, 1), P(1, 1), n, 2, 0, 1, None) == 1           # n < 0
        n = (ctypes.c_int64 * 2)(4, 2)
        assert f(0, P(1, None), P(1, 1), P(1, 1), n, 2, 0, 1, None) == 1        # NULL batch
    assert lib.hg_solve_grouped_f32(3, None, None, None, None, 0, 0, 1, None) == 1  # GPT: f64
    assert pkg.version().startswith("sks-homography-amd")


def test_solve_host_argument_checks(pkg):
    """ops.solve_host validates shapes, dtypes and contiguity before the C call."""
    import torch
    x = torch.zeros(4, 8)
    with pytest.raises(ValueError, match="contiguous"):
        pkg.solve_host("aca", torch.zeros(8, 4).t(), x)
    with pytest.raises(ValueError, match="equal"):
        pkg.solve_host("aca", x, torch.zeros(5, 8))
    with pytest.raises(ValueError, match="out must be"):
        pkg.solve_host("aca", x, x, out=torch.zeros(4, 8))
    with pytest.raises(TypeError, match="float64 only"):
        pkg.solve_host("gpt", x, x)
    with pytest.raises(ValueError, match="algo"):
        pkg.solve_host("dlt", x, x)
    with pytest.raises(ValueError, match=r"\(8,n\)"):
        pkg.solve_host("aca", x, x, layout="soa")


def test_product_rejects_cpu_tensors(pkg):
    """No CPU fallback: host tensors are refused loudly."""
    import torch
    x = torch.zeros(4, 8)
    with pytest.raises(ValueError, match="GPU only"):
        pkg.aca(x, x)
    with pytest.raises(ValueError, match="GPU only"):
        pkg.tensor_aca_rect(torch.zeros(2, 3, 4), torch.zeros(2, 3, 4), 1.0, 1.0)
    # the generators take a device, not a tensor: a host device (or host `out`) must be
    # refused before any kernel could be handed host memory
    with pytest.raises(ValueError, match="GPU only"):
        pkg.fill_bits(16, 1, 0, device="cpu")
    with pytest.raises(ValueError, match="GPU only"):
        pkg.fill_uniform(16, 1, device="cpu")
    with pytest.raises(ValueError, match="GPU only"):
        pkg.fill_uniform(16, 1, out=torch.empty(16))
    with pytest.raises(ValueError, match="count"):
        pkg.fill_bits(-1, 1, 0)
    with pytest.raises(ValueError, match="count"):
        pkg.fill_uniform(-1, 1)
    with pytest.raises(ValueError, match="GPU only"):
        pkg.stream_copy(torch.zeros(4), torch.zeros(4))


def test_missing_library_fails_loudly(pkg, monkeypatch):
    monkeypatch.setattr(pkg._lib, "_lib", None)
    monkeypatch.setattr(pkg._lib, "LIB_PATH", "/nonexistent/libsks_homography_amd.so")
    with pytest.raises(ImportError, match="no CPU fallback"):
        pkg._lib.lib()


def test_product_never_imports_oracle():
    """The product package must not reach the checker."""
    pkg_dir = os.path.join(ROOT, "sks-homography_amd")
    forbidden = re.compile(r"import\s+oracle|from\s+oracle|load_oracle|libhg_oracle|libsks_ref|"
                           r"oracle_\w+\(|ref_batch_f")
    for dirpath, _, files in os.walk(pkg_dir):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".hpp", ".h")):
                text = open(os.path.join(dirpath, f)).read()
                assert not forbidden.search(text), f"{f} reaches the oracle"


def test_native_torch_ops_registered(pkg):
    """torch.ops.sks_amd.* come from lib/libsks_homography_torch.so (C++ dispatcher
    registrations): every schema is there, Meta kernels give the shapes, and there is no
    CPU kernel."""
    import torch
    ops = torch.ops.sks_amd
    want = {
        "solve": ["default", "out"], "aca": ["default", "out"], "sks": ["default", "out"],
        "tensor_aca_rect": ["default", "out", "scalar", "scalar_out"],
        "tensor_aca_rect_backward": ["default"],
        "tensor_aca_offsets": ["default", "out"], "tensor_aca_offsets_backward": ["default"],
    }
    for name, overloads in want.items():
        assert sorted(getattr(ops, name).overloads()) == sorted(overloads), name
    m = lambda *s: torch.empty(*s, device="meta")  # noqa: E731
    assert ops.tensor_aca_rect(m(5, 3, 4), m(5, 3, 4), m(1), m(1)).shape == (5, 3, 3)
    assert ops.tensor_aca_offsets(m(5, 2), m(5, 4, 2), 1.0, 2.0).shape == (5, 3, 3)
    assert ops.aca(m(5, 4, 2), m(5, 4, 2), True).shape == (5, 3, 3)
    assert ops.solve(m(5, 8), m(5, 8), 1, True, 0).shape == (5, 9)
    assert ops.solve(m(8, 7), m(8, 7), 2, False, 1).shape == (9, 7)
    g = ops.tensor_aca_rect_backward(m(5, 3, 4), m(5, 3, 4), m(5, 3, 3), m(1), m(1), True, False)
    assert [tuple(x.shape) for x in g] == [(5, 3, 4), (5, 3, 4), (0,), (0,)]
    with pytest.raises(NotImplementedError):
        ops.tensor_aca_offsets(torch.zeros(2, 2), torch.zeros(2, 4, 2), 1.0, 1.0)
    with open("/proc/self/maps") as f:
        assert "libsks_homography_torch.so" in f.read()


def test_read_points_matches_reference_format(pkg, tmp_path):
    """read_points parses the reference's correspondence-file format (utils.cpp:6-21:
    count line, then "x1 y1 x2 y2" rows) to the same float32 pools as the committed
    orig_pts_wall.txt fixture."""
    import numpy as np
    from conftest import load_golden
    g = load_golden("cpp_wall.npz")
    ps, pt = g["pool_src"], g["pool_tar"]
    path = tmp_path / "pts.txt"
    with open(path, "w") as f:
        f.write(f"{ps.shape[0]}\n")
        for a, b in zip(ps, pt):  # shortest decimals that round-trip (the file's own style)
            f.write(" ".join(np.format_float_positional(v, unique=True)
                             for v in (a[0], a[1], b[0], b[1])) + "\n")
    rs, rt = pkg.read_points(str(path))
    assert rs.dtype == np.float32 and rs.shape == ps.shape
    assert np.array_equal(rs, ps) and np.array_equal(rt, pt)
    fs, ft = pkg.read_points(os.path.join(ROOT, "tests", "golden", "orig_pts_wall_restated.txt"))
    assert np.array_equal(fs, ps) and np.array_equal(ft, pt)
    bad = tmp_path / "short.txt"
    bad.write_text("3\n1 2 3 4\n")
    with pytest.raises(ValueError):
        pkg.read_points(str(bad))


def test_read_points_rounds_once_like_sscanf(pkg, tmp_path):
    """Values are converted the way the reference's sscanf("%f", &float) converts them (one
    correct rounding to binary32), not through binary64 first: a decimal just above the
    midpoint between 1 and 1 + 2^-23 must give 1 + 2^-23 (binary64 first lands on the
    midpoint, and ties-to-even then gives 1).  Checked against the C library's strtof and
    exact rational rounding."""
    import ctypes
    import ctypes.util
    from fractions import Fraction

    import numpy as np
    tricky = ["1.00000005960464477539062500000001", "0.99999997019767761230468749999999",
              "16777217.0000000000000001", "3.4028235677973366e38", "1e-46", "-0.0", "356.39"]
    path = tmp_path / "tricky.txt"
    path.write_text("2\n" + " ".join(tricky[:4]) + "\n" + " ".join(tricky[3:7]) + "\n")
    rs, rt = pkg.read_points(str(path))
    got = np.concatenate([rs, rt], axis=1).ravel()
    strtof = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6").strtof
    strtof.restype, strtof.argtypes = ctypes.c_float, [ctypes.c_char_p, ctypes.c_void_p]
    want = np.array([strtof(t.encode(), None) for t in tricky[:4] + tricky[3:7]], np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert got[0].view(np.uint32) == np.float32(1.0).view(np.uint32) + 1
    # the first value by exact rounding of the rational: above the midpoint -> the upper neighbour
    lo, hi = Fraction(1), Fraction(1) + Fraction(1, 2**23)
    assert Fraction(tricky[0]) > (lo + hi) / 2 and Fraction(float(got[0])) == hi


def test_pmc_traffic_matches_the_kernel_code():
    """profiles/pmc_traffic.json's PMC figures were measured on headline kernels whose gfx950
    machine code digest it records (build_lib.kernel_code_digest, read from the library that
    ran); bench.py reports them as `roofline.traffic` only while the built library still holds
    that code.  A change to the headline kernels fails here until the PMC passes are re-run
    (tools/gpu_round.sh pmc, tools/pmc_traffic.py) -- the committed figure is never silently
    reused for a different kernel.  The machine code is a function of
    the compiler too: when the recorded hipcc differs from this one, the comparison says
    nothing about the kernels and is skipped (bench.py still reports null on a mismatch)."""
    import json
    import bench
    sys.path.insert(0, os.path.join(ROOT, "sks-homography_amd"))
    try:
        import build_lib as bl
    finally:
        sys.path.pop(0)
    with open(bench.PMC_TRAFFIC) as f:
        measured_with = json.load(f).get("provenance", {}).get("compiler")
    if measured_with and measured_with != bl.compiler_id():
        pytest.skip(f"PMC figures measured with another compiler ({measured_with})")
    src = bench.traffic_source()
    assert src["kernel_code_measured"], "profiles/pmc_traffic.json has no kernel code digest"
    assert src["kernel_code_match"], (f"headline kernel code changed since the PMC run "
                                      f"({src['kernel_code_measured']} -> "
                                      f"{src['kernel_code_now']}): re-measure the traffic")
    assert bench.pmc_traffic("aca_f32_aos_norm") is not None


def test_pmc_families_name_built_kernels_and_match_their_code():
    """Every kernel family tools/pmc_traffic.py reduces names kernels the built library holds
    (a changed template signature -- a new parameter -- would otherwise drop the family from
    the PMC summary without a word), and each family's recorded machine-code digest is the
    built code's, so every `traffic` figure bench.py quotes belongs to the kernel it times."""
    import json
    import bench
    sys.path.insert(0, os.path.join(ROOT, "sks-homography_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import build_lib as bl
        import pmc_traffic as pt
    finally:
        sys.path.pop(0)
        sys.path.pop(0)
    now = {k: bl.kernel_family_digest(prefix) for k, (prefix, _) in pt.KEYS.items()}
    assert all(now.values()), [k for k, v in now.items() if not v]
    with open(bench.PMC_TRAFFIC) as f:
        rec = json.load(f)
    measured_with = rec.get("provenance", {}).get("compiler")
    if measured_with and measured_with != bl.compiler_id():
        pytest.skip(f"PMC figures measured with another compiler ({measured_with})")
    assert set(rec["detail"]) == set(pt.KEYS), set(pt.KEYS) ^ set(rec["detail"])
    stale = {k: (rec["detail"][k].get("code"), now[k]) for k in pt.KEYS
             if rec["detail"][k].get("code") != now[k]}
    assert not stale, f"kernel code changed since the PMC run: {stale}"
    # bench.py matches a record by the prefix stored IN it (a record whose
    # stored prefix no longer named the kernel printed `traffic_bytes: null` on the box)
    moved = {k: (rec["detail"][k].get("prefix"), prefix) for k, (prefix, _) in pt.KEYS.items()
             if rec["detail"][k].get("prefix") != prefix}
    assert not moved, f"recorded prefixes differ from tools/pmc_traffic.py's: {moved}"


def test_every_quoted_pmc_figure_is_current():
    """Every family bench.py quotes a `traffic` for (pmc_detail / pmc_traffic) has a record in
    profiles/pmc_traffic.json whose machine code is the built library's: pmc_detail, run here
    on the CPU, returns a figure for each -- never `traffic_bytes: null`."""
    import json
    import re
    import bench
    sys.path.insert(0, os.path.join(ROOT, "sks-homography_amd"))
    try:
        import build_lib as bl
    finally:
        sys.path.pop(0)
    with open(bench.PMC_TRAFFIC) as f:
        measured_with = json.load(f).get("provenance", {}).get("compiler")
    if measured_with and measured_with != bl.compiler_id():
        pytest.skip(f"PMC figures measured with another compiler ({measured_with})")
    with open(os.path.join(ROOT, "bench.py")) as f:
        text = f.read()
    keys = sorted(set(re.findall(r'pmc_detail\(\s*"([a-z0-9_]+)"', text)))
    assert len(keys) >= 10, keys
    bench._FAMILY_CODE.clear()
    missing = {k: bench.pmc_detail(k).get("reason") for k in keys
               if bench.pmc_detail(k).get("traffic_bytes") is None}
    assert not missing, missing
    for k in ("aca_f32_aos_norm", "sks_f32_aos_norm"):  # the headline's roofline.traffic
        assert bench.pmc_traffic(k) is not None, k


def test_kernel_code_digest_reads_the_headline_entry_points(pkg):
    """The digest finds exactly the two headline kernels' code in the gfx950 code objects of
    the built library, and it is a function of the code alone (stable across reads)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sks-homography_amd"))
    try:
        import build_lib as bl
    finally:
        sys.path.pop(0)
    d1, d2 = bl.kernel_code_digest(), bl.kernel_code_digest()
    assert d1 == d2 and set(d1) == set(bl.TRAFFIC_KERNELS)
    assert d1["aca_f32_aos_norm"] != d1["sks_f32_aos_norm"]
