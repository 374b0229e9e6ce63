"""bench.py's own N-rank launch (the driver's `python bench.py --gpus N`).

Without WORLD_SIZE in the environment, `--gpus N` (N > 1) must start N ranks
itself (torch.distributed.run, one per GPU) and relay ONE JSON line from
rank 0; with WORLD_SIZE set (an external launcher) a different --gpus is an
error.  `--dry-run` exercises exactly that launch path on CPU: the ranks join
a gloo group and report (rank, local rank, pid) without touching a GPU.
"""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def _json_lines(out):
    return [json.loads(s) for s in out.splitlines() if s.strip().startswith("{")]


def test_gpus_2_launches_two_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=300, env=_env())
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout           # rank 0 only, relayed once
    r = lines[0]
    assert r["dry_run"] and r["world_size"] == 2 and r["n_gpus"] == 2 and r["gpus_arg"] == 2
    assert r["backend"] == "gloo"
    assert sorted(x["rank"] for x in r["ranks"]) == [0, 1]
    assert sorted(x["local_rank"] for x in r["ranks"]) == [0, 1]
    pids = {x["pid"] for x in r["ranks"]}
    assert len(pids) == 2                       # two processes, one per rank


def test_gpus_1_stays_single_process():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--dry-run"], capture_output=True, text=True,
                       timeout=300, env=_env())
    assert p.returncode == 0, p.stderr[-2000:]
    (r,) = _json_lines(p.stdout)
    assert r["world_size"] == 1 and [x["rank"] for x in r["ranks"]] == [0]


def test_world_size_mismatch_is_an_error():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"))
    assert p.returncode != 0
    assert "WORLD_SIZE=3" in p.stderr
    assert _json_lines(p.stdout) == []
