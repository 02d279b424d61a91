import ctypes
import glob
import os
import sys

import numpy as np
import pytest

# HIP's runtime logs the address and reason of a GPU memory fault at level 1 (errors only):
# with it set before HIP starts, a fault's own report lands in the failing test's captured
# stderr, which the driver's log tail shows.
os.environ.setdefault("AMD_LOG_LEVEL", "1")
# HIP copies a pageable host buffer of >= 2 MB by mapping the user's pages into the GPU's
# address space in place (KFD shared-virtual-memory ranges over the heap) and keeps those
# mappings after the copy; every GPU fault this suite ever had was such a copy writing a heap
# page.  The tests' own .cpu() / .to() copies go through HIP's staging
# buffers instead (the runtime reads this before it starts): no heap page of the test process
# is mapped for the GPU except by the library's HG_FLAG_HOST_REGISTER calls under test (its
# default host path maps none -- tests/test_gpu_host_nomap.py checks that in a child process
# that runs WITHOUT this setting).
os.environ.setdefault("GPU_PINNED_MIN_XFER_SIZE", "65536")  # MiB

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size (10M) parity checks")


# ----------------------------------------------------------------------------- GPU test order
# The oracle / golden / reference parity files run first, the BASELINE configs at their full
# sizes among the very first, so that a late failure under -x cannot erase the evidence that
# matters most; then the subprocess programs; then the plumbing and stress tests (threads,
# host-page registration, pending-error probes, graphs); the >2^31 (~200 GB) tests last.
# Within a tier the files keep their order and every test its place in its file.  Nothing
# is dropped or skipped by this.
_FIRST = [  # (file, test name prefix): BASELINE configs and the reference's own outputs
    ("test_gpu_parity.py", "test_config2_full_batch_equals_compiled_reference"),  # configs[1], [2]
    ("test_gpu_parity.py", "test_rect_close_to_torch_composed_on_gpu"),          # configs[3]
    ("test_gpu_parity.py", "test_config1_gpu_equals_compiled_reference"),        # configs[0]
    ("test_gpu_config5.py", "test_config5_rank_blocks"),                          # configs[4]
    ("test_gpu_parity.py", "test_golden_"),
    ("test_gpu_parity.py", "test_full_size_10m_bit_exact"),
    ("test_gpu_copies.py", ""),  # before any library host call maps heap pages
    ("test_gpu_parity.py", "test_rect_backward_kernel_vs_oracle"),
]
_PARITY_FILES = [
    "test_gpu_parity.py", "test_gpu_refcpp_bits.py", "test_gpu_kat.py", "test_gpu_vanilla_grad.py",
    "test_gpu_rect_grad.py", "test_gpu_rect_bcast.py", "test_gpu_rect_aten_bits.py",
    "test_gpu_rect_rocm_order.py", "test_gpu_offsets.py", "test_gpu_table8.py",
    "test_gpu_ransac.py", "test_gpu_mrg32k3a.py", "test_gpu_aten_sum.py", "test_gpu_rocm_sum.py",
    "test_gpu_refcu.py", "test_gpu_config5.py", "test_gpu_multi.py",
]
_PROGRAM_FILES = ["test_gpu_bench_contract.py", "test_gpu_cpp_api.py", "test_gpu_host_nomap.py"]
_STRESS_FILES = ["test_gpu_grouped.py", "test_gpu_errors.py", "test_gpu_host.py"]
_STRESS_TESTS = [  # plumbing tests inside the parity file: threads, host pointers, graphs
    ("test_gpu_parity.py", "test_cpp_api_single_problem_host_and_device"),
    ("test_gpu_parity.py", "test_cpp_api_mixed_pointers_and_edge_cases"),
    ("test_gpu_parity.py", "test_solve_one_c_abi"),
    ("test_gpu_parity.py", "test_stream_and_graph_capture"),
    ("test_gpu_parity.py", "test_concurrent_streams"),
    ("test_gpu_parity.py", "test_c_abi_from_many_threads"),
]
_LAST = [("test_gpu_large.py", ""), ("test_gpu_parity.py", "test_beyond_int32_problem_count")]


def gpu_tier(fname, name):
    """(tier, rank within the tier) of a GPU test: lower runs first."""
    for i, (f, p) in enumerate(_FIRST):
        if fname == f and name.startswith(p):
            return 0, i
    for i, (f, p) in enumerate(_LAST):
        if fname == f and name.startswith(p):
            return 4, i
    for i, (f, p) in enumerate(_STRESS_TESTS):
        if fname == f and name.startswith(p):
            return 3, len(_STRESS_FILES) + i
    for tier, files in ((1, _PARITY_FILES), (2, _PROGRAM_FILES), (3, _STRESS_FILES)):
        if fname in files:
            return tier, files.index(fname)
    return 1, len(_PARITY_FILES)  # a GPU file not listed yet: with the parity files


def pytest_collection_modifyitems(session, config, items):
    gpu = [(i, it) for i, it in enumerate(items) if it.get_closest_marker("gpu") is not None]
    if not gpu:
        return
    slots = [i for i, _ in gpu]
    ordered = sorted(gpu, key=lambda e: (gpu_tier(os.path.basename(str(e[1].fspath)),
                                                  e[1].name), e[0]))
    for slot, (_, it) in zip(slots, ordered):
        items[slot] = it


# ------------------------------------------------------------------- GPU fault attribution
_FAULTS = {"checked": 0, "first": None}
_HIP = None


def _hip():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so.7")
        _HIP.hipGetErrorName.restype = ctypes.c_char_p
    return _HIP


_PROBE = {"lib": None, "tried": False}


def _fault_probe():
    """tests/_build/libfault_probe.so (tests/fault_probe.c): a ROCr system-event handler that
    prints a GPU memory fault's virtual address and reason the moment it happens.  Installed
    once HIP is up; None when it is not built or cannot register."""
    if not _PROBE["tried"]:
        _PROBE["tried"] = True
        path = os.path.join(ROOT, "tests", "_build", "libfault_probe.so")
        if os.path.exists(path):
            lib = ctypes.CDLL(path)
            lib.hg_fault_probe_read.argtypes = [ctypes.POINTER(ctypes.c_int),
                                                ctypes.POINTER(ctypes.c_uint64),
                                                ctypes.POINTER(ctypes.c_uint32)]
            if lib.hg_fault_probe_install() == 0:
                _PROBE["lib"] = lib
    return _PROBE["lib"]


def _where(va):
    """What holds virtual address `va` in this process: its /proc/self/maps line, and the
    torch caching-allocator segment (device memory) containing it, if any."""
    out = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                lo, hi = (int(x, 16) for x in line.split()[0].split("-"))
                if lo <= va < hi:
                    out.append(f"maps: {line.strip()} (+0x{va - lo:x})")
                    break
            else:
                out.append("maps: no mapping holds it")
    except OSError:
        pass
    try:  # what HIP itself takes the address for (a registered or pinned host range?)
        hip = _hip()
        attrs = (ctypes.c_uint64 * 8)()
        rc = hip.hipPointerGetAttributes(attrs, ctypes.c_void_p(va))
        hip.hipGetLastError()
        raw = ctypes.string_at(attrs, 40)
        mtype = int.from_bytes(raw[0:4], "little")
        out.append(f"hipPointerGetAttributes rc {rc} type {mtype} (0 unregistered, 1 host, 2 device, 3 "
                   f"managed) device ptr 0x{int.from_bytes(raw[8:16], 'little'):x} host ptr "
                   f"0x{int.from_bytes(raw[16:24], 'little'):x}")
    except Exception as e:  # noqa: BLE001 -- diagnostics only
        out.append(f"hipPointerGetAttributes unavailable: {e!r}"[:120])
    try:  # KFD's view of the page: HIP's in-place copies and registrations live here
        probe = _fault_probe()
        if probe is not None:
            u64 = ctypes.c_uint64
            probe.hg_fault_probe_svm.argtypes = [u64, u64] + [ctypes.POINTER(u64)] * 3
            acc, ro, gf = u64(), u64(), u64()
            rc = probe.hg_fault_probe_svm(va // 4096 * 4096, 4096, ctypes.byref(acc), ctypes.byref(ro),
                                          ctypes.byref(gf))
            out.append(f"SVM attributes rc {rc} access 0x{acc.value:x} (0x200 accessible, 0x201 in "
                       f"place, 0x202 none) read-only {ro.value} global flag {gf.value}")
    except Exception as e:  # noqa: BLE001 -- diagnostics only
        out.append(f"SVM attributes unavailable: {e!r}"[:120])
    try:  # the library's own page registrations (hg_host.cpp history)
        lib = ctypes.CDLL(os.path.join(ROOT, "sks-homography_amd", "lib", "libsks_homography_amd.so"))
        lo, hi, seq = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        st = lib.hg_internal_host_registry_find(ctypes.c_uint64(va), ctypes.byref(lo), ctypes.byref(hi),
                                                ctypes.byref(seq))
        stats = (ctypes.c_int64 * 4)()
        lib.hg_internal_host_registry_stats(stats)
        state = {0: "never registered by the library (last 4096)", 1: "LIVE library registration",
                 2: "library registration, released", 3: "library registration, RELEASE FAILED"}[st]
        out.append(f"{state}" + (f" [0x{lo.value:x}, 0x{hi.value:x}) #{seq.value}" if st else "")
                   + f"; registry: {stats[0]} live, {stats[1]} made, {stats[2]} unregister failures")
    except Exception as e:  # noqa: BLE001 -- diagnostics only
        out.append(f"registry history unavailable: {e!r}"[:120])
    try:
        import torch
        for seg in torch.cuda.memory_snapshot():
            a, n = seg["address"], seg["total_size"]
            if a <= va < a + n:
                out.append(f"torch segment 0x{a:x} + {n} ({seg.get('segment_type')}, offset 0x{va - a:x})")
                break
        else:
            out.append("not in any torch caching-allocator segment")
    except Exception as e:  # noqa: BLE001 -- diagnostics only
        out.append(f"torch snapshot unavailable: {e!r}"[:200])
    return "; ".join(out)


@pytest.fixture(autouse=True)
def _gpu_fault_check(request):
    """After every GPU test: a device-wide synchronisation, so that a kernel fault (an illegal
    address, an aborted queue) is reported against the test whose launches caused it, by
    name, instead of surfacing at some later test's first copy -- with the faulting address
    and what holds it (tests/fault_probe.c).  A test that never touched the GPU in this
    process (the subprocess programs) is not checked here."""
    gpu = request.node.get_closest_marker("gpu") is not None
    if gpu:
        import torch
        if torch.cuda.is_initialized():
            _fault_probe()
    yield
    if not gpu:
        return
    import torch
    if not torch.cuda.is_initialized():
        return
    probe = _fault_probe()
    hip = _hip()
    rc = hip.hipDeviceSynchronize()
    _FAULTS["checked"] += 1
    seen = 0
    if probe is not None:
        t, va, why = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint32()
        seen = probe.hg_fault_probe_read(ctypes.byref(t), ctypes.byref(va), ctypes.byref(why))
    if rc != 0 or seen:
        name = hip.hipGetErrorName(rc).decode() if rc else "no HIP error yet"
        detail = ""
        if seen:
            detail = (f"; fault probe: {seen} event(s), first type {t.value}, VA 0x{va.value:x}, "
                      f"reason 0x{why.value:x}; {_where(va.value)}")
        if _FAULTS["first"] is None:
            _FAULTS["first"] = (request.node.nodeid, name + detail)
        pytest.fail(f"GPU error {name} ({rc}) pending at the end of {request.node.nodeid}: a "
                    "kernel launched during this test (or by a thread it started) faulted"
                    + detail, pytrace=False)


def _cards_used_gb():
    """{PCI address: card-wide VRAM in use by every process, GB} (amdgpu's
    mem_info_vram_used) for every card the host shows -- read without touching HIP."""
    vals = {}
    for p in glob.glob("/sys/class/drm/card*/device/mem_info_vram_used"):
        try:
            with open(p) as f:
                vals[os.path.basename(os.path.realpath(os.path.dirname(p)))] = int(f.read()) / 1e9
        except (OSError, ValueError):
            pass
    return vals


def _our_card_gb(cards):
    """The entry of `cards` for cuda:0 (the PCI address from HIP, which the tests started)."""
    try:
        import torch
        if not torch.cuda.is_initialized():
            return None
        pr = torch.cuda.get_device_properties(0)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
    except Exception:  # noqa: BLE001 -- a summary line must not fail the session
        return None
    for addr, gb in cards.items():
        if addr.startswith(bdf):
            return gb
    return None


def pytest_sessionstart(session):
    session.config._cards_at_start = _cards_used_gb()


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """One line for the driver's log tail: how many GPU tests were fault-checked, the first
    fault if any, and what the card held (all processes) when the session began."""
    if not _FAULTS["checked"] and _FAULTS["first"] is None:
        return
    first = _FAULTS["first"]
    card = _our_card_gb(getattr(config, "_cards_at_start", {}))
    probe = "fault probe on" if _PROBE["lib"] is not None else "fault probe off"
    terminalreporter.write_line(
        f"gpu fault check ({probe}): {_FAULTS['checked']} GPU tests synchronised after running; "
        + (f"FIRST FAULT {first[1]} after {first[0]}" if first else "no fault")
        + "; this card's VRAM in use at session start (all processes): "
        + (f"{card:.1f} GB" if card is not None else "n/a"))
    large = [r for r in terminalreporter.stats.get("passed", []) + terminalreporter.stats.get("skipped", [])
             if "test_gpu_large.py" in r.nodeid and r.when in ("call", "setup")]
    if large:
        terminalreporter.write_line(
            "beyond-2^31 parity: " + "; ".join(f"{r.nodeid.split('::')[-1]} {r.outcome}"
                                                for r in large))


# ----------------------------------------------------------------------------- fixtures
@pytest.fixture(scope="session")
def orc():
    """Oracle module (test infrastructure)."""
    return ge.load_oracle()


@pytest.fixture(scope="session")
def oracle(orc):
    return orc.Oracle()


@pytest.fixture(scope="session")
def pkg():
    return ge.load_package()


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def load_golden(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.fail(f"golden fixture {path} missing (run tools/make_golden.py here)")
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


class default_dtype:
    """torch's default dtype set for a block (the reference's statements allocate H with it:
    torch.zeros / torch.ones without a dtype, Modules_Runtime_Test.py:296, :372)."""

    def __init__(self, dt):
        import torch
        self.dt, self.torch = dt, torch

    def __enter__(self):
        self.prev = self.torch.get_default_dtype()
        self.torch.set_default_dtype(self.dt)

    def __exit__(self, *exc):
        self.torch.set_default_dtype(self.prev)
