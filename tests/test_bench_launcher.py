"""bench.py's own multi-rank launcher (`--gpus N` without WORLD_SIZE), on the CPU: the
parent spawns N workers with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, they meet over the
host channel (token-checked rendezvous), time their steps between barriers, all-gather
their rewards in the RCCL path's padded block layout (uneven shards included) and check
the whole vector; the parent relays rank 0's line. `--dry-host` uses the CPU oracle's
rewards and never loads HIP. Failures must give a non-zero exit: a corrupted gathered
vector, WORLD_SIZE != --gpus, more ranks than GPUs."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")
SMALL = ["--n-agents", "16", "--n-envs", "2", "--steps", "3", "--warmup", "1"]


def run(args, env=None, timeout=150):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "GYMFLOCK_HOST_TOKEN",
              "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, timeout=timeout)


@pytest.mark.timeout(200)
@pytest.mark.parametrize("world", [2, 8])
def test_launcher_dry_host(world):
    p = run(["--gpus", str(world), "--dry-host"] + SMALL)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    lines = p.stdout.decode().strip().splitlines()
    assert len(lines) == 1  # the parent relays rank 0's JSON line only
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["dry_host"] is True
    assert len(d["per_rank_ms_per_step"]) == world
    assert d["ms_per_step"] == max(d["per_rank_ms_per_step"])
    assert d["gathered_rewards_ok"] is True
    assert d["gathered_stats_ok"] is True
    assert d["config"]["global_envs"] == 2 * world
    assert "torch" not in p.stderr.decode()


@pytest.mark.timeout(200)
def test_launcher_uneven_shards_padded():
    """The last rank holds one env more (shard_range's split of 3 * 2 + 1 envs): the
    gathers ship every rank's block padded to the largest shard, and the unpadded vector
    equals every rank's local values."""
    p = run(["--gpus", "3", "--dry-host", "--dry-host-uneven"] + SMALL)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    d = json.loads(p.stdout.decode().strip().splitlines()[0])
    assert d["shard_sizes"] == [2, 2, 3] and d["config"]["global_envs"] == 7
    assert d["gathered_rewards_ok"] is True and d["gathered_stats_ok"] is True


@pytest.mark.timeout(200)
def test_launcher_fails_loudly():
    p = run(["--gpus", "3", "--dry-host", "--dry-host-corrupt"] + SMALL)
    assert p.returncode != 0
    assert p.stdout.decode().strip() == ""
    assert "run failed" in p.stderr.decode()


@pytest.mark.timeout(60)
def test_world_size_must_match_gpus():
    p = run(["--gpus", "4", "--dry-host"] + SMALL, env={"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 4" in p.stderr.decode()


@pytest.mark.timeout(60)
def test_more_ranks_than_visible_gpus_is_refused(tmp_path):
    """The parent counts GPUs from the KFD topology (no HIP call): a fake topology with one
    GPU node (and one CPU node) refuses --gpus 2 before anything is spawned."""
    for i, simd in enumerate((0, 256)):
        d = tmp_path / "nodes" / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text("cpu_cores_count 8\nsimd_count %d\n" % simd)
    p = run(["--gpus", "2"] + SMALL, env={"GYMFLOCK_KFD_TOPOLOGY": str(tmp_path)})
    assert p.returncode == 2
    assert "only 1 GPU(s) are visible" in p.stderr.decode()
