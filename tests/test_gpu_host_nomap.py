"""The library's host entry leaves no GPU mapping of the caller's pages.

hg_solve_host_* on pageable memory copies through library-owned pinned stages (hg_host.cpp)
and never registers the caller's pages, so KFD's attribute of every page of src, tar and H is
still 0x202 (no GPU access) when the call returns -- an attribute query, not a fault
reproduction.  The check runs in a fresh process with HIP's default copy policy
(GPU_PINNED_MIN_XFER_SIZE unset, unlike this process, tests/conftest.py) that touches the GPU
only through the library: tests/host_nomap_child.py, which also replays ADVICE r05's sequence
(free, reallocate, a >= 2 MB in-place HIP copy into the reused pages) and records a positive
control (an HG_FLAG_HOST_REGISTER call, whose pages stay mapped)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(290)
def test_host_entry_leaves_no_gpu_mapping_under_default_runtime(dev, record_property):
    if not os.path.exists(os.path.join(ROOT, "tests", "_build", "libfault_probe.so")):
        pytest.fail("tests/_build/libfault_probe.so not built (__graft_entry__.build())")
    env = {k: v for k, v in os.environ.items() if k != "GPU_PINNED_MIN_XFER_SIZE"}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "host_nomap_child.py")],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines, f"child printed no result (rc {r.returncode}): {r.stdout[-2000:]} {r.stderr[-3000:]}"
    res = json.loads(lines[-1])
    record_property("host_nomap", res)
    print(json.dumps({"control_register": res.get("control_register"),
                      "reuse_copies": res.get("reuse_copies")}))
    assert res["knob"] is None
    bad = [c for c in res["cases"] if not c["bits"] or any(c["mapped_after"])]
    assert not bad, f"cases with wrong bits or GPU-mapped pages after the call: {bad}"
    assert len(res["cases"]) == 16
    assert all(not any(c["mapped_before"]) for c in res["cases"])
    assert all(x["data"] for x in res["reuse_copies"]), res["reuse_copies"]
    assert res["sync_rc"] == 0 and res["fault_events"] == 0
    assert res["control_register"]["rc"] == 0
    assert r.returncode == 0 and res["ok"], r.stderr[-3000:]
