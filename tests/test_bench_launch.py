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
