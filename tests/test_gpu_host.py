"""Host-resident batches (hg_solve_host_f32/_f64, ops.solve_host): pinned buffers are read and
written by the kernel in place; pageable ones go through the library's ring of pinned stages
(the default) or, with HG_FLAG_HOST_REGISTER (register=True), are registered for the call.
Pinned and pageable buffers, every solver, both layouts, one chunk and many (a small ring
configured through hg_internal_host_stage_config), pinned, device and pageable buffers mixed,
buffers cut from one allocation (sharing pages), misaligned views, threads at once -- each
bit-identical to the device-resident solve, which tests/test_gpu_parity.py pins to the
oracle; a small batch is also checked against the oracle directly.  That the staged path
leaves the caller's pages unmapped is tests/test_gpu_host_nomap.py."""
import ctypes
import os
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SEED = 5


@pytest.fixture(autouse=True)
def _registrations_released(pkg):
    """After every host-memory test: no page registration of the library's is left, and none
    failed to be released (hg_host.cpp; a leftover would map pages the caller frees or reuses)."""
    yield
    lib = pkg.lib()
    stats = (ctypes.c_int64 * 4)()
    assert lib.hg_internal_host_registry_stats(stats) == 0
    assert stats[0] == 0, f"{stats[0]} registrations still live"
    assert stats[2] == 0, f"{stats[2]} unregistrations failed (last hipError {stats[3]})"


def _inputs(pkg, dev, n, dtype, layout, off=0):
    s = pkg.fill_uniform(n * 8, SEED, off, device=dev)
    t = pkg.fill_uniform(n * 8, SEED, off + n * 8, device=dev)
    shape = (n, 8) if layout == "aos" else (8, n)
    return s.view(shape).to(dtype), t.view(shape).to(dtype)


def _bits(x):
    return x.view(torch.int32 if x.dtype is torch.float32 else torch.int64)


def _internal(lib):
    """Signatures of the library-internal stage hooks (hg_host.cpp; not in the header)."""
    p64 = ctypes.POINTER(ctypes.c_int64)
    lib.hg_internal_host_stage_config.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, p64]
    lib.hg_internal_host_stage_config.restype = ctypes.c_int
    lib.hg_internal_host_stage_stats.argtypes = [p64]
    lib.hg_internal_host_stage_stats.restype = ctypes.c_int
    return lib


def _stage_stats(lib):
    _internal(lib)
    st = (ctypes.c_int64 * 8)()
    assert lib.hg_internal_host_stage_stats(st) == 0
    return list(st)


@pytest.fixture
def small_ring(pkg):
    """A 64 KiB ring stage, 3 deep, 4 copy threads: every batch below of more than a few
    hundred problems runs in many chunks.  The library's settings are restored after."""
    lib = _internal(pkg.lib())
    prev = (ctypes.c_int64 * 3)()
    assert lib.hg_internal_host_stage_config(64 << 10, 3, 4, prev) == 0
    yield lib
    assert lib.hg_internal_host_stage_config(prev[0], prev[1], prev[2], None) == 0


def _hip():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipPointerGetAttributes.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return hip


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("layout", ["aos", "soa"])
@pytest.mark.parametrize("pinned", [False, True])
def test_host_batch_matches_device(pkg, dev, dtype, layout, pinned):
    n = 70001  # ragged: not a multiple of any tile
    algos = ["aca", "sks", "ge"] + (["gpt"] if dtype is torch.float64 else [])
    ds, dt = _inputs(pkg, dev, n, dtype, layout)
    hs, ht = ds.cpu(), dt.cpu()
    if pinned:
        hs, ht = hs.pin_memory(), ht.pin_memory()
    for algo in algos:
        for norm in (True, False):
            want = pkg.solve(algo, ds, dt, normalize=norm, layout=layout).cpu()
            out = torch.full(want.shape, float("nan"), dtype=dtype)
            if pinned:
                out = out.pin_memory()
            got = pkg.solve_host(algo, hs, ht, normalize=norm, layout=layout, out=out)
            assert got is out
            assert torch.equal(_bits(got), _bits(want)), (algo, norm)


def test_host_batch_vs_oracle(pkg, dev, oracle):
    n = 4099
    ds, dt = _inputs(pkg, dev, n, torch.float32, "aos", off=123)
    hs, ht = ds.cpu(), dt.cpu()
    for algo in ("aca", "sks"):
        got = pkg.solve_host(algo, hs, ht, normalize=True)
        want = oracle.solve(algo, hs.numpy(), ht.numpy(), normalize=True)
        assert np.array_equal(got.numpy().view(np.uint32), want.view(np.uint32)), algo


@pytest.mark.parametrize("register", [False, True])
def test_host_buffers_sharing_pages_and_misaligned(pkg, dev, register):
    """src, tar and H carved out of ONE pageable allocation (neighbours share pages, so
    registrations must merge), H at a 4-B offset (not 16-B aligned: the generic
    kernel), and no registration left afterwards -- staged and registered."""
    n = 30011
    ds, dt = _inputs(pkg, dev, n, torch.float32, "aos", off=77)
    want = pkg.solve("aca", ds, dt, normalize=True).cpu()
    buf = torch.zeros(n * 8 * 2 + 1 + n * 9, dtype=torch.float32)
    s = buf[:n * 8].view(n, 8)
    t = buf[n * 8:n * 16].view(n, 8)
    h = buf[n * 16 + 1:].view(n, 9)  # 4 B past a 16-B boundary
    s.copy_(ds.cpu())
    t.copy_(dt.cpu())
    pkg.solve_host("aca", s, t, out=h, register=register)
    assert torch.equal(_bits(h), _bits(want))
    assert torch.equal(_bits(s), _bits(ds.cpu()))  # inputs untouched
    # unregistered again: a second registration of the same pages succeeds
    hip = _hip()
    attrs = ctypes.create_string_buffer(256)
    rc = hip.hipPointerGetAttributes(attrs, ctypes.c_void_p(buf.data_ptr()))
    hip.hipGetLastError()
    assert rc != 0 or attrs.raw[:4] == b"\0\0\0\0", "pages still registered after the call"
    pkg.solve_host("aca", s, t, out=h, register=register)
    assert torch.equal(_bits(h), _bits(want))


def test_host_entry_accepts_device_and_mixed(pkg, dev):
    n = 5000
    ds, dt = _inputs(pkg, dev, n, torch.float64, "aos", off=9)
    want = pkg.solve("sks", ds, dt, normalize=True)
    lib = pkg.lib()
    dH = torch.empty_like(want)
    assert lib.hg_solve_host_f64(1, ds.data_ptr(), dt.data_ptr(), dH.data_ptr(), n, 0, 1, None) == 0
    assert torch.equal(_bits(dH), _bits(want))
    hH = torch.empty((n, 9), dtype=torch.float64)  # host H, device inputs
    assert lib.hg_solve_host_f64(1, ds.data_ptr(), dt.data_ptr(), hH.data_ptr(), n, 0, 1, None) == 0
    assert torch.equal(_bits(hH), _bits(want.cpu()))


def test_host_threads_at_once(pkg, dev):
    """Eight threads, each its own pageable batch (registrations serialised), plus one
    pinned caller that never takes the registration lock."""
    n = 20000
    jobs = []
    for k in range(8):
        ds, dt = _inputs(pkg, dev, n, torch.float32, "aos", off=k * 1_000_000)
        jobs.append((ds.cpu(), dt.cpu(), pkg.solve("aca", ds, dt).cpu()))
    ds, dt = _inputs(pkg, dev, n, torch.float32, "aos", off=99_000_000)
    jobs.append((ds.cpu().pin_memory(), dt.cpu().pin_memory(), pkg.solve("aca", ds, dt).cpu()))
    bad = []

    def work(k):
        s, t, want = jobs[k]
        for _ in range(5):
            got = pkg.solve_host("aca", s, t)
            if not torch.equal(_bits(got), _bits(want)):
                bad.append(k)

    th = [threading.Thread(target=work, args=(k,)) for k in range(len(jobs))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not bad


@pytest.mark.parametrize("register", [False, True])
def test_host_threads_share_one_pageable_allocation(pkg, dev, register):
    """threads solving slices of ONE pageable allocation.  Neighbouring
    slices share the pages at their boundaries, so one call finds pages another call
    registered (they read as pinned memory); the library must treat them as its own
    registration -- shared, reference-counted, unregistered only after the last kernel that
    uses them has finished -- and never as user-pinned memory.  Each thread also checks its
    neighbours' rows stay untouched, and the pages are unregistered at the end."""
    k, n = 8, 20011  # 20011 * 32 B and * 36 B: slice edges fall inside pages
    ds, dt = _inputs(pkg, dev, k * n, torch.float32, "aos", off=555)
    want = pkg.solve("aca", ds, dt).cpu()
    src, tar = ds.cpu(), dt.cpu()  # one pageable allocation each
    H = torch.full((k * n, 9), float("nan"))
    bad = []
    start = threading.Barrier(k)

    def work(i):
        lo, hi = i * n, (i + 1) * n
        start.wait()
        for it in range(12):
            # alternate the slice shape so registrations overlap in changing ways: the
            # whole slice, then its two halves in turn
            if it % 3 == 0:
                pkg.solve_host("aca", src[lo:hi], tar[lo:hi], out=H[lo:hi], register=register)
            else:
                mid = lo + n // 2 + (it % 2)
                pkg.solve_host("aca", src[lo:mid], tar[lo:mid], out=H[lo:mid], register=register)
                pkg.solve_host("aca", src[mid:hi], tar[mid:hi], out=H[mid:hi], register=register)
            if not torch.equal(_bits(H[lo:hi]), _bits(want[lo:hi])):
                bad.append((i, it))

    th = [threading.Thread(target=work, args=(i,)) for i in range(k)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not bad, bad
    assert torch.equal(_bits(H), _bits(want))
    hip = _hip()
    attrs = ctypes.create_string_buffer(256)
    for p in (src.data_ptr(), tar.data_ptr() + 4096 * 7, H.data_ptr() + 36 * n):
        rc = hip.hipPointerGetAttributes(attrs, ctypes.c_void_p(p))
        hip.hipGetLastError()
        assert rc != 0 or attrs.raw[:4] == b"\0\0\0\0", "pages still registered after the calls"


@pytest.mark.parametrize("register", [False, True])
def test_host_threads_random_overlapping_slices(pkg, dev, register):
    """Stress of the shared registrations: 6 threads, each solving 40 random (possibly
    overlapping in pages, never in rows) slices of one pageable allocation, sizes from 1
    problem to 40 K, f32 AoS; every row written equals the device solve, untouched rows
    stay NaN, and no registration survives."""
    import random
    n = 300_007
    ds, dt = _inputs(pkg, dev, n, torch.float32, "aos", off=4242)
    want = pkg.solve("aca", ds, dt).cpu()
    src, tar = ds.cpu(), dt.cpu()
    H = torch.full((n, 9), float("nan"))
    k = 6
    per = n // k
    bad = []

    def work(i):
        rng = random.Random(i)
        lo0, hi0 = i * per, (i + 1) * per if i < k - 1 else n
        for _ in range(40):
            a = rng.randrange(lo0, hi0)
            b = min(hi0, a + rng.choice((1, 7, 100, 4096, 40_000)))
            pkg.solve_host("aca", src[a:b], tar[a:b], out=H[a:b], register=register)
            if not torch.equal(_bits(H[a:b]), _bits(want[a:b])):
                bad.append((i, a, b))

    th = [threading.Thread(target=work, args=(i,)) for i in range(k)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not bad, bad[:5]
    done = ~torch.isnan(H[:, 0])
    assert torch.equal(_bits(H[done]), _bits(want[done]))
    assert done.sum() > 0
    hip = _hip()
    attrs = ctypes.create_string_buffer(256)
    for p in (src.data_ptr(), tar.data_ptr() + 4096 * 100, H.data_ptr() + 36 * (n // 2)):
        rc = hip.hipPointerGetAttributes(attrs, ctypes.c_void_p(p))
        hip.hipGetLastError()
        assert rc != 0 or attrs.raw[:4] == b"\0\0\0\0", "pages still registered after the calls"


def test_host_full_size(pkg, dev):
    """BASELINE configs[1] size, 10 M problems, from pageable memory."""
    n = 10_000_000
    ds, dt = _inputs(pkg, dev, n, torch.float32, "aos")
    want = pkg.solve("aca", ds, dt).cpu()
    got = pkg.solve_host("aca", ds.cpu(), dt.cpu())
    assert torch.equal(_bits(got), _bits(want))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("layout", ["aos", "soa"])
def test_pageable_batches_are_staged_never_registered(pkg, dev, dtype, layout):
    """Pageable batches go through library-owned pinned stages and are never registered: bits
    equal the device solve for every solver, ragged sizes up to the 128 KiB small stage's
    edge, just past it (a ring stage) and well past it, H at a 4-B offset; no call makes a
    page registration, and batches past the small stage's edge take ring stages."""
    lib = pkg.lib()
    stats = (ctypes.c_int64 * 4)()
    algos = ["aca", "sks", "ge"] + (["gpt"] if dtype is torch.float64 else [])
    per = 100 if dtype is torch.float32 else 200  # bytes a problem stages (src + tar + H)
    edge = (128 << 10) // per - 16
    for n in (1, 2, 7, 64, 100, 1000 if dtype is torch.float32 else 500, edge, edge + 40, 200_003):
        ds, dt = _inputs(pkg, dev, n, dtype, layout, off=n)
        hs, ht = ds.cpu(), dt.cpu()
        for algo in algos:
            want = pkg.solve(algo, ds, dt, normalize=True, layout=layout).cpu()
            buf = torch.full((want.numel() + 1,), float("nan"), dtype=dtype)
            out = buf[1:].view(want.shape)  # one element past the allocation's start
            assert lib.hg_internal_host_registry_stats(stats) == 0
            made = stats[1]
            ring = _stage_stats(lib)[4]
            got = pkg.solve_host(algo, hs, ht, normalize=True, layout=layout, out=out)
            assert got is out
            assert torch.equal(_bits(got), _bits(want)), (n, algo)
            assert lib.hg_internal_host_registry_stats(stats) == 0
            assert stats[1] == made, (n, "registered")
            assert (_stage_stats(lib)[4] > ring) == (n > edge), (n, "ring stage use")
            assert torch.equal(_bits(hs), _bits(ds.cpu()))  # inputs untouched


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("layout", ["aos", "soa"])
def test_staged_ring_many_chunks(pkg, dev, small_ring, dtype, layout):
    """The ring at work: a 64 KiB stage, 3 deep, so a ragged 70001-problem batch runs in
    about 110 chunks (the last one short) -- every solver, normalised and not, bits equal to
    the device solve; pageable inputs untouched; no registration."""
    lib = small_ring
    n = 70001
    algos = ["aca", "sks", "ge"] + (["gpt"] if dtype is torch.float64 else [])
    ds, dt = _inputs(pkg, dev, n, dtype, layout, off=31)
    hs, ht = ds.cpu(), dt.cpu()
    stats = (ctypes.c_int64 * 4)()
    assert lib.hg_internal_host_registry_stats(stats) == 0
    made = stats[1]
    for algo in algos:
        for norm in (True, False):
            want = pkg.solve(algo, ds, dt, normalize=norm, layout=layout).cpu()
            out = torch.full(want.shape, float("nan"), dtype=dtype)
            c0 = _stage_stats(lib)[2]
            pkg.solve_host(algo, hs, ht, normalize=norm, layout=layout, out=out)
            assert torch.equal(_bits(out), _bits(want)), (algo, norm)
            assert _stage_stats(lib)[2] - c0 > 50, "expected many chunks"
    assert torch.equal(_bits(hs), _bits(ds.cpu())) and torch.equal(_bits(ht), _bits(dt.cpu()))
    assert lib.hg_internal_host_registry_stats(stats) == 0 and stats[1] == made


@pytest.mark.parametrize("layout", ["aos", "soa"])
def test_staged_ring_mixed_memory(pkg, dev, small_ring, layout):
    """Pageable buffers beside pinned and device ones, in many chunks: in AoS the pinned and
    device buffers are used in place at each chunk's offset; in SoA a chunk is C-wide rows,
    so the pinned ones are copied by the host threads and the device ones by the DMA engines
    (hipMemcpy2DAsync) through the stage too.  Every combination, f64 SKS, bits equal."""
    lib = small_ring
    n = 40007
    ds, dt = _inputs(pkg, dev, n, torch.float64, layout, off=5)
    want = pkg.solve("sks", ds, dt, normalize=True, layout=layout)
    kinds = {"pageable": lambda x: x.cpu(), "pinned": lambda x: x.cpu().pin_memory(),
             "device": lambda x: x.clone()}
    combos = [("pageable", "pinned", "pageable"), ("pinned", "pageable", "pinned"),
              ("device", "pageable", "pageable"), ("pageable", "device", "device"),
              ("pinned", "device", "pageable"), ("device", "device", "pageable")]
    for ks, kt, kh in combos:
        s, t = kinds[ks](ds), kinds[kt](dt)
        h = kinds[kh](torch.full(want.shape, float("nan"), dtype=torch.float64, device=dev))
        rc = lib.hg_solve_host_f64(1, s.data_ptr(), t.data_ptr(), h.data_ptr(), n,
                                   0 if layout == "aos" else 1, 1, None)
        assert rc == 0, (ks, kt, kh, rc)
        assert torch.equal(_bits(h.cpu()), _bits(want.cpu())), (ks, kt, kh)


def test_staged_ring_settings_validated(pkg, dev):
    lib = _internal(pkg.lib())
    prev = (ctypes.c_int64 * 3)()
    assert lib.hg_internal_host_stage_config(0, 0, 0, prev) == 0  # a query
    assert prev[0] >= 64 << 10 and 1 <= prev[1] <= 16 and 1 <= prev[2] <= 64
    assert lib.hg_internal_host_stage_config(1024, 0, 0, None) == 1
    assert lib.hg_internal_host_stage_config(0, 17, 0, None) == 1
    assert lib.hg_internal_host_stage_config(0, 0, 65, None) == 1
    now = (ctypes.c_int64 * 3)()
    assert lib.hg_internal_host_stage_config(0, 0, 0, now) == 0
    assert list(now) == list(prev)


def test_small_pageable_batches_from_threads(pkg, dev):
    """Eight threads, each 60 small pageable calls (staged through pooled stages), one of them
    with pinned inputs and a pageable H: every result bit-exact, no registration made, no
    stage withheld."""
    lib = pkg.lib()
    stats = (ctypes.c_int64 * 4)()
    jobs = []
    for k in range(8):
        n = 37 + 113 * k
        ds, dt = _inputs(pkg, dev, n, torch.float32, "aos", off=7 * k)
        hs, ht = ds.cpu(), dt.cpu()
        if k == 3:
            hs, ht = hs.pin_memory(), ht.pin_memory()
        jobs.append((hs, ht, pkg.solve("sks", ds, dt).cpu()))
    assert lib.hg_internal_host_registry_stats(stats) == 0
    made = stats[1]
    bad = []

    def work(k):
        s, t, want = jobs[k]
        for _ in range(60):
            got = pkg.solve_host("sks", s, t)
            if not torch.equal(_bits(got), _bits(want)):
                bad.append(k)

    th = [threading.Thread(target=work, args=(k,)) for k in range(len(jobs))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not bad, bad
    assert lib.hg_internal_host_registry_stats(stats) == 0
    assert stats[1] == made, f"{stats[1] - made} registrations made by staged calls"
    assert _stage_stats(lib)[3] == 0


def test_host_entry_errors(pkg, dev):
    lib = pkg.lib()
    s = torch.zeros((4, 8))
    h = torch.zeros((4, 9))
    assert lib.hg_solve_host_f32(3, s.data_ptr(), s.data_ptr(), h.data_ptr(), 4, 0, 1, None) == 1
    assert lib.hg_solve_host_f32(0, s.data_ptr(), s.data_ptr(), h.data_ptr(), 4, 3, 1, None) == 1
    assert lib.hg_solve_host_f32(0, s.data_ptr(), s.data_ptr(), h.data_ptr(), 0, 0, 1, None) == 0
    with pytest.raises(ValueError):
        pkg.solve_host("aca", s.cuda(), s.cuda())


def test_ctypes_numpy_binding_as_documented(pkg, dev):
    """INTEGRATION.md section 4's plain-ctypes binding on numpy arrays (pageable memory)."""
    lib = pkg.lib()
    n = 12345
    ds, dt = _inputs(pkg, dev, n, torch.float32, "aos", off=321)
    want = pkg.solve("aca", ds, dt).cpu().numpy()
    src = np.ascontiguousarray(ds.cpu().numpy(), np.float32)
    tar = np.ascontiguousarray(dt.cpu().numpy(), np.float32)
    H = np.empty((len(src), 9), np.float32)
    rc = lib.hg_solve_host_f32(0, src.ctypes.data, tar.ctypes.data, H.ctypes.data, len(src), 0, 1, None)
    assert rc == 0
    assert np.array_equal(H.view(np.uint32), want.view(np.uint32))


def test_shared_host_batch_solve_block(pkg, dev):
    """shard.SharedHostBatch in one process (world 1 and a 3-way split solved block by
    block): the GPU reads and writes the /dev/shm pages, bits equal the device solve."""
    from sks_homography_amd.shard import SharedHostBatch
    n = 50001
    ds, dt = _inputs(pkg, dev, n, torch.float32, "aos", off=777)
    want = pkg.solve("aca", ds, dt).cpu()
    b = SharedHostBatch(f"sks_hg_gpu_test_{os.getpid()}", n, 0, lambda: None)
    try:
        b.src.copy_(ds.cpu())
        b.tar.copy_(dt.cpu())
        assert b.solve_block(1) == (0, n)
        assert torch.equal(b.H.view(torch.int32), want.view(torch.int32))
        b.H.zero_()
        for r in range(3):  # what three ranks would each do for their own rows
            b.rank = r
            lo, hi = b.solve_block(3)
            assert (lo, hi) == pkg.shard_range(n, 3, r)
        b.rank = 0
        assert torch.equal(b.H.view(torch.int32), want.view(torch.int32))
    finally:
        b.rank = 0
        b.close()
    assert not os.path.exists(f"/dev/shm/sks_hg_gpu_test_{os.getpid()}")


def test_staged_calls_alternate_devices(pkg, dev, small_ring):
    """the stage pool is shared by every device of the process -- stages are
    portable pinned memory, their device address looked up per device, ring streams pooled per
    device.  Small (one stage) and ring (many chunks) calls alternate between cuda:0 and cuda:1,
    every result bit-exact.  Needs two GPUs (skipped on the one-GPU boxes)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU: the cross-device stage reuse needs two")
    for n in (500, 70001):
        ds, dt = _inputs(pkg, dev, n, torch.float32, "aos", off=n)
        want = pkg.solve("aca", ds, dt).cpu()
        hs, ht = ds.cpu(), dt.cpu()
        for d in (0, 1, 0, 1):
            got = pkg.solve_host("aca", hs, ht, device=d)
            assert torch.equal(_bits(got), _bits(want)), (n, d)


def test_staged_rings_from_threads(pkg, dev, small_ring):
    """Four threads, each running many-chunk rings at once (64 KiB stages, 3 deep: every call
    takes 3 stages, 3 device buffers and 3 ring streams from the shared pools), AoS and SoA,
    f32 and f64, 6 calls each: every H bit-exact, no stage withheld, no registration made."""
    lib = small_ring
    stats = (ctypes.c_int64 * 4)()
    assert lib.hg_internal_host_registry_stats(stats) == 0
    made = stats[1]
    jobs = []
    for k, (dtype, layout) in enumerate([(torch.float32, "aos"), (torch.float64, "soa"),
                                         (torch.float64, "aos"), (torch.float32, "soa")]):
        n = 30011 + 977 * k
        ds, dt = _inputs(pkg, dev, n, dtype, layout, off=17 * k)
        jobs.append((ds.cpu(), dt.cpu(), layout, pkg.solve("sks", ds, dt, layout=layout).cpu()))
    bad = []

    def work(k):
        s, t, layout, want = jobs[k]
        for _ in range(6):
            got = pkg.solve_host("sks", s, t, layout=layout)
            if not torch.equal(_bits(got), _bits(want)):
                bad.append(k)

    th = [threading.Thread(target=work, args=(k,)) for k in range(len(jobs))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not bad, bad
    assert _stage_stats(lib)[3] == 0
    assert lib.hg_internal_host_registry_stats(stats) == 0 and stats[1] == made
