"""`bench.py --gpus N` starts N ranks itself (torch.distributed.run as a child process,
127.0.0.1 rendezvous) and rejects a --gpus that disagrees with the launcher's WORLD_SIZE.
The ranks run bench.py's --dry-run leg (gloo, no GPU), so this runs on the CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, timeout=300, env=e, cwd=ROOT)


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_2_launches_two_ranks():
    p = _run(["--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = _json_line(p.stdout)
    assert d["n_gpus"] == 2 and sorted(d["ranks"]) == [0, 1]


@pytest.mark.parametrize("renderer,res", [("dos", 2048), ("ebs", 1024)])
def test_gpus_2_dry_run_shaded_configs(renderer, res):
    """Configs 4 and 5 over two gloo ranks: every pixel of the 2048^2 / 1024^2 viewport
    travels through pack -> gather -> unpack exactly once."""
    p = _run(["--gpus", "2", "--dry-run", "--renderer", renderer])
    assert p.returncode == 0, p.stderr[-2000:]
    d = _json_line(p.stdout)
    assert d["viewport"] == [res, res] and d["renderer"] == renderer
    assert d["gather_exact"] is True
    assert sum(d["tiles_per_rank"]) == (res // d["tile"]) ** 2


def test_gpus_1_stays_in_process():
    p = _run(["--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert _json_line(p.stdout)["n_gpus"] == 1


def test_gpus_disagreeing_with_world_size_fails():
    p = _run(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0",
                                                "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr


@pytest.mark.parametrize("args,want", [([], 8), (["--hw-queues", "16"], 16), (["--hw-queues=12"], 12)])
def test_hw_queues_both_forms(args, want):
    """GPU_MAX_HW_QUEUES is set before HIP initialises from either spelling of the flag."""
    p = _run(["--dry-run", *args])
    assert p.returncode == 0, p.stderr[-2000:]
    assert _json_line(p.stdout)["hw_queues"] == want


@pytest.mark.parametrize("bad", [["--hw-queues=40"], ["--hw-queues", "33"], ["--hw-queues"]])
def test_hw_queues_rejects_bad_values(bad):
    """Outside 1..32 (the box refuses more than 32) or without a value: a clear exit."""
    p = _run(["--dry-run", *bad])
    assert p.returncode != 0
    assert "hw-queues" in p.stderr


def test_split_defaults_frames_per_launch_follow_the_run_length():
    """bench.split_defaults: at N > 1 the rc1pass launch groups grow with the run (two
    launches per render stream at least: 4 frames for the driver's 20-step runs, 16
    from 128 steps on); one GPU keeps 4; other renderers 1."""
    import bench
    want = {20: 4, 50: 4, 64: 8, 100: 8, 128: 16, 200: 16}
    for steps, fpl in want.items():
        for world in (2, 4, 8):
            a = bench.parse(["--gpus", str(world), "--steps", str(steps)])
            kw = bench.split_defaults(a, world)
            assert kw["frames_per_launch"] == fpl == kw["frames_per_exchange"], (steps, world, kw)
            assert kw["streams"] == 4 and kw["root_renders"] == (world < 8)
        assert bench.split_defaults(bench.parse(["--steps", str(steps)]), 1)["frames_per_launch"] == 4
    a = bench.parse(["--gpus", "8"])                 # the default run (200 steps)
    assert bench.split_defaults(a, 8)["frames_per_launch"] == 16
    a = bench.parse(["--gpus", "8", "--renderer", "dos", "--steps", "200"])
    assert bench.split_defaults(a, 8)["frames_per_launch"] == 1
    a = bench.parse(["--gpus", "8", "--frames-per-launch", "8", "--steps", "20"])
    assert bench.split_defaults(a, 8)["frames_per_launch"] == 8
