"""The CPU-side code under AddressSanitizer + UndefinedBehaviorSanitizer.

* oracle/hg_oracle.c and the reference-side shim oracle/ref_batch.cpp (with the reference's
  own ACA_SKS.cpp / GE.cpp where /root/reference is present) are rebuilt instrumented
  (oracle/build.sh with SKS_ORACLE_SANITIZE) and tests/test_oracle_golden.py +
  tests/test_properties.py run against those builds, the sanitizer runtimes preloaded into
  Python; the pinned multi-thread timing path and the f64 same-points timing run too.
* A negative control: an out-of-bounds oracle call in the same setup must be caught, which
  shows the instrumented libraries are the ones loaded.
* hg_host_ranges.hpp -- the page-range merge and registration plan of hg_solve_host_*
  (csrc/hg_host.cpp) -- and hg_host_stage.hpp -- the staged ring of its pageable path and the
  copy thread pool -- in a pure C++ unit check (tests/host_ranges_check.cpp), also under
  ThreadSanitizer.
"""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

HERE = os.path.dirname(os.path.abspath(__file__))


def _runtime(name):
    path = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True,
                          text=True).stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


@pytest.fixture(scope="module")
def san_build(tmp_path_factory):
    if not shutil.which("gcc") or not shutil.which("g++"):
        pytest.skip("gcc/g++ not available")
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("sanitizer runtimes not installed")
    out = tmp_path_factory.mktemp("san")
    subprocess.run(["bash", os.path.join(ROOT, "oracle", "build.sh")], check=True,
                   env=dict(os.environ, SKS_ORACLE_SANITIZE=str(out)), capture_output=True)
    env = dict(os.environ,
               SKS_ORACLE_SO=str(out / "libhg_oracle.so"),
               LD_PRELOAD=f"{asan} {ubsan}",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               PYTHONDONTWRITEBYTECODE="1")
    if (out / "libsks_ref.so").exists():
        env["SKS_REF_SO"] = str(out / "libsks_ref.so")
    return out, env


def test_sanitized_builds_are_instrumented(san_build):
    out, _ = san_build
    syms = subprocess.run(["nm", "-D", str(out / "libhg_oracle.so")], capture_output=True,
                          text=True).stdout
    assert "__asan_" in syms and "__ubsan_" in syms


def test_oracle_tests_under_asan_ubsan(san_build):
    _, env = san_build
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p",
                        "no:cacheprovider", os.path.join(HERE, "test_oracle_golden.py"),
                        os.path.join(HERE, "test_properties.py")],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "passed" in r.stdout


TIMING = r"""
import sys, numpy as np
sys.path.insert(0, "oracle")
import oracle as o
g = o.Oracle()
n = 5000
s = g.fill_uniform(n * 8, 11, 0).reshape(n, 8); t = g.fill_uniform(n * 8, 11, n * 8).reshape(n, 8)
H = np.empty((n, 9), np.float32)
for algo in ("aca", "sks"):
    assert g.time_batch(algo, s, t, H, 3, 2) > 0
if o.RefOracle.available():
    r = o.RefOracle()
    for algo in ("aca", "sks", "ge"):
        assert r.time_pinned(algo, s, t, [0, 0, 0], 2, H) > 0
        assert np.array_equal(H.view(np.uint32), r.solve(algo, s, t).view(np.uint32))
    for algo in ("aca", "sks"):
        assert r.time_repeat(algo, s[0].astype(np.float64), t[0].astype(np.float64), 1000) > 0
        assert r.time_repeat(algo, s[0], t[0], 1000) > 0
print("timing ok")
"""


def test_timing_paths_under_asan_ubsan(san_build):
    _, env = san_build
    r = subprocess.run([sys.executable, "-c", TIMING], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "timing ok" in r.stdout, r.stdout + r.stderr[-4000:]


OOB = r"""
import sys, numpy as np
sys.path.insert(0, "oracle")
import oracle as o
g = o.Oracle()
s = np.zeros((2, 8), np.float32); t = np.zeros((2, 8), np.float32); H = np.zeros((2, 9), np.float32)
fp = o._f32p
g.lib.oracle_aca_f32(s.ctypes.data_as(fp), t.ctypes.data_as(fp), H.ctypes.data_as(fp), 64, 0, 1)
print("not caught")
"""


def test_negative_control_is_caught(san_build):
    _, env = san_build
    r = subprocess.run([sys.executable, "-c", OOB], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "not caught" not in r.stdout
    assert "AddressSanitizer" in r.stderr


def test_host_ranges_under_asan_ubsan(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = tmp_path / "host_ranges_check"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
                    f"-I{ROOT}/sks-homography_amd/csrc", os.path.join(HERE, "host_ranges_check.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0 and "host ranges ok" in r.stdout, r.stdout + r.stderr


def test_host_stage_under_tsan(tmp_path):
    """The copy thread pool and the staged ring (hg_host_stage.hpp) under ThreadSanitizer:
    several callers sharing one pool's helpers, lists handed over and retired while helpers
    still hold them."""
    if not shutil.which("g++") or not _runtime("libtsan.so"):
        pytest.skip("g++ or the ThreadSanitizer runtime not available")
    exe = tmp_path / "host_stage_tsan"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread",
                    f"-I{ROOT}/sks-homography_amd/csrc", os.path.join(HERE, "host_ranges_check.cpp"),
                    "-o", str(exe), "-lpthread"], check=True)
    r = subprocess.run([str(exe), "30"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0 and "host ranges ok" in r.stdout, r.stdout + r.stderr[-4000:]
