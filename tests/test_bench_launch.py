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
    # the default N > 1 run also times BASELINE configs[4]: 1B x 64 B keys split
    # over the ranks (strong scaling), beside the cfg2 weak-scaling value
    c4 = r["plan"]["config4"]
    assert r["plan"]["config"] == "cfg2" and r["plan"]["value_scaling"] == "weak"
    assert c4["keys_total"] == 1 << 30 and c4["keys_per_rank"] == [1 << 29, 1 << 29]


def test_config4_split_is_whole_reference_chunks():
    """Every world size the driver runs (1/2/4/8) splits the 1B keys into
    whole 16M-key chunks, so every rank's slice has a reference fold."""
    sys.path.insert(0, ROOT)
    import bench
    folds = bench.golden_folds()
    for world in (1, 2, 4, 8):
        a = type("A", (), {"config": "cfg2", "no_config4": False, "keys_per_gpu": 0, "dist_backend": "nccl"})
        per = bench.plan(a, world)["config4"]["keys_per_rank"]
        assert sum(per) == 1 << 30
        first = 0
        for n in per:
            assert bench.city64_chunk_fold(folds, first, n) is not None
            first += n
    # the folds of the 8 shards of 1B, summed from chunks, equal the shard folds
    c5 = folds["cfg5_city64_1B_x64"]
    for s in range(8):
        assert bench.city64_chunk_fold(folds, s << 27, 1 << 27) == int(c5["shards"][s], 16)
    assert bench.city64_chunk_fold(folds, 0, 1 << 30) == int(c5["total"], 16)
    assert bench.city64_chunk_fold(folds, 5, 1 << 24) is None      # not whole chunks
    assert bench.city64_chunk_fold(folds, 0, (1 << 30) + (1 << 24)) is None


def test_config4_block_only_on_default_workload():
    sys.path.insert(0, ROOT)
    import bench
    mk = lambda **kw: type("A", (), {"config": "cfg2", "no_config4": False, "keys_per_gpu": 0,  # noqa: E731
                                     "dist_backend": "nccl", **kw})
    assert "config4" in bench.plan(mk(), 1)
    assert "config4" not in bench.plan(mk(config="cfg3"), 2)
    assert "config4" not in bench.plan(mk(no_config4=True), 2)
    assert "config4" not in bench.plan(mk(keys_per_gpu=1000), 2)


def test_config4_line_is_strong_scaling_and_rejects_keys_per_gpu():
    sys.path.insert(0, ROOT)
    import bench
    a = type("A", (), {"config": "config4", "no_config4": False, "keys_per_gpu": 0, "dist_backend": None})
    assert bench.plan(a, 8)["value_scaling"] == "strong"
    p = subprocess.run([sys.executable, BENCH, "--config", "config4", "--keys-per-gpu", "1000", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=_env())
    assert p.returncode == 2 and "--keys-per-gpu" in p.stderr
    assert _json_lines(p.stdout) == []


def test_gloo_rehearsal_flag_accepted():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert p.returncode == 0, p.stderr[-2000:]
    (r,) = _json_lines(p.stdout)
    assert r["plan"]["backend"] == "gloo" and r["world_size"] == 2


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


def test_cache_sized_inputs_rotate_past_the_infinity_cache():
    """Inputs that fit the 256 MiB Infinity Cache are cycled through enough
    identical copies that >= 512 MiB pass between two reads of one copy
    (bench.rot_copies); larger inputs are used alone."""
    sys.path.insert(0, ROOT)
    import bench

    class T:  # stands in for a tensor: size and clone only
        def __init__(self, nbytes):
            self.nbytes = nbytes

        def numel(self):
            return self.nbytes

        def element_size(self):
            return 1

        def clone(self):
            return T(self.nbytes)

    M = 1 << 20
    for nbytes, copies in ((64 * M, 8), (128 * M, 4), (256 * M, 2), (1 << 30, 1), (8 << 30, 1), (1 * M, 8)):
        ks = bench.rot_copies(None, T(nbytes))
        assert len(ks) == copies
        assert all(k.nbytes == nbytes for k in ks)
        assert copies == 8 or copies * nbytes >= bench.ROT_BYTES
