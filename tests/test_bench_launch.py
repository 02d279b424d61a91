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
