"""bench.py's --gpus contract (CPU): the launch decision, the child command, and the
pass-through of a spawned job's stdout and exit status.

The driver runs `python bench.py --gpus N` either under torch.distributed.run (WORLD_SIZE set)
or bare.  Bare with N > 1, bench.py starts the N ranks itself as a child process; a
WORLD_SIZE that disagrees with --gpus is refused before any GPU call.
"""
import os
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("gpus,env,plan", [
    (1, {}, "self"),
    (1, {"WORLD_SIZE": ""}, "self"),
    (2, {}, "spawn"),
    (8, {}, "spawn"),
    (1, {"WORLD_SIZE": "1"}, "self"),
    (8, {"WORLD_SIZE": "8"}, "self"),
    (8, {"WORLD_SIZE": "1"}, "refuse"),
    (1, {"WORLD_SIZE": "8"}, "refuse"),
    (2, {"WORLD_SIZE": "x"}, "refuse"),
    (0, {}, "refuse"),
])
def test_launch_plan(gpus, env, plan):
    got, why = bench.launch_plan(gpus, env)
    assert got == plan
    assert (why == "") == (plan == "self")


def test_torchrun_cmd():
    cmd = bench.torchrun_cmd(4, ["--gpus", "4", "--steps", "3"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert cmd[-5] == os.path.join(ROOT, "bench.py")


def test_spawn_passes_rank0_line_and_status(tmp_path, monkeypatch, capfd):
    """The spawn path end to end with gloo ranks standing in for bench's GPU ranks: the
    children see WORLD_SIZE = N, rank 0's line reaches our stdout, the status is returned."""
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent("""
        import json, os, sys
        import torch.distributed as dist
        dist.init_process_group("gloo")
        if dist.get_rank() == 0:
            print(json.dumps({"n_gpus": dist.get_world_size(), "argv": sys.argv[1:]}), flush=True)
        dist.barrier()
        dist.destroy_process_group()
        sys.exit(int(os.environ.get("RANK_EXIT", "0")))
    """))
    real = bench.torchrun_cmd
    monkeypatch.setattr(bench, "torchrun_cmd",
                        lambda n, argv, port: real(n, argv, port)[:-len(argv) - 1] + [str(script), *argv])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.spawn_ranks(2, ["--gpus", "2"]) == 0
    out = capfd.readouterr().out
    line = [t for t in out.splitlines() if t.startswith("{")]
    assert len(line) == 1 and '"n_gpus": 2' in line[0] and '"--gpus", "2"' in line[0]
    monkeypatch.setenv("RANK_EXIT", "3")
    assert bench.spawn_ranks(2, ["--gpus", "2"]) != 0


def test_refusal_exits_before_gpu(monkeypatch):
    """A WORLD_SIZE that disagrees with --gpus ends main() with status 2 (no device opened)."""
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 2


def test_spawn_forwards_termination_to_the_ranks(tmp_path):
    """A SIGTERM sent to bench.py's process alone (a driver's time limit) reaches the ranks it
    started: they end instead of running on without a parent, and bench.py exits non-zero."""
    import signal
    import subprocess
    import time
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(f"""
        import os, time
        open(os.path.join({str(tmp_path)!r}, "rank%s.pid" % os.environ["RANK"]), "w").write(str(os.getpid()))
        time.sleep(120)
    """))
    driver = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {ROOT!r})
        import bench
        real = bench.torchrun_cmd
        bench.torchrun_cmd = lambda n, argv, port: real(n, argv, port)[:-len(argv) - 1] + [{str(script)!r}, *argv]
        sys.exit(bench.spawn_ranks(2, ["--gpus", "2"]))
    """)
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    parent = subprocess.Popen([sys.executable, "-c", driver], env=env, stdout=subprocess.DEVNULL,
                              stderr=subprocess.DEVNULL)
    pids = []
    try:
        deadline = time.time() + 90
        while time.time() < deadline and len(pids) < 2:
            pids = [int(p.read_text()) for p in tmp_path.glob("rank*.pid") if p.read_text()]
            time.sleep(0.2)
        assert len(pids) == 2, "the ranks did not start"
        parent.send_signal(signal.SIGTERM)
        rc = parent.wait(timeout=60)
        assert rc != 0
        deadline = time.time() + 30
        alive = pids
        while time.time() < deadline and alive:
            alive = [p for p in pids if os.path.exists(f"/proc/{p}") and
                     "Z" not in open(f"/proc/{p}/stat").read().split(")")[-1].split()[:1]]
            time.sleep(0.2)
        assert not alive, f"ranks {alive} outlived bench.py"
    finally:
        if parent.poll() is None:
            parent.kill()
            parent.wait()
        for p in pids:
            try:
                os.kill(p, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
