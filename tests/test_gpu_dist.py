"""The RCCL code paths on device tensors, on a one-GPU box.

RCCL refuses two ranks on one device, so the N-rank path runs here as ONE
rank in an "nccl" process group of world size 1: the collectives still
execute (pdht_amd.dist runs them in any initialised group), through RCCL, on
HIP tensors.  Each case starts a fresh child process (before any GPU call in
it) and reads its one JSON line."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> str:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return str(p)


def _child(cmd, timeout):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [s for s in p.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_rccl_world1_exchange_and_reductions():
    """exchange_buckets / exchange_records (all_to_all_single), allreduce_max,
    allreduce_fold, allreduce_min_int and per_rank_report through RCCL on
    device tensors; RCCL is mapped in the child."""
    r = _child([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_child.py"), _port()], 110)
    assert r["backend"] == "nccl" and r["world"] == 1
    for k in ("exchange_buckets", "exchange_records", "allreduce_max", "allreduce_fold", "allreduce_min_int",
              "per_rank_report", "rccl_mapped", "product_mapped"):
        assert r[k] is True, (k, r)


def test_bench_nccl_world1_xrecords():
    """bench.py's nccl branch at N = 1: the xrecords step buckets 1M keys by
    the world size into wire records and ships them with one all-to-all(v)
    through RCCL inside every timed step; the line's parity check verifies
    the received records."""
    r = _child([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--config", "xrecords", "--dist-backend",
                "nccl", "--steps", "3", "--warmup", "1", "--keys-per-gpu", str(1 << 20), "--no-cpu-baseline"], 110)
    assert r["per_rank"]["backend"] == "nccl" and r["n_gpus"] == 1
    assert "exchange:" in r["parity"] and "FAILED" not in r["parity"], r["parity"]
