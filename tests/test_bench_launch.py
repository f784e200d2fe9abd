"""bench.py's multi-GPU entry point (CPU): `--gpus N` must start and check N
ranks itself, and never print a smaller run than it was asked for.

The N-rank path is exercised with --dry-plan (gloo on the CPU, each rank plans
its SPI-hash share of the config's packets, key.c:293-299 key_u32hash); the
driver's 8-GPU scaling run uses the same launcher with the GPU work."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                        "LOCAL_WORLD_SIZE", "GROUP_RANK", "TORCHELASTIC_RUN_ID")}
    env.update(extra)
    return env


def _run(args, **extra):
    return subprocess.run([sys.executable, BENCH] + args, env=_env(**extra), capture_output=True,
                          text=True, timeout=240, cwd=ROOT)


def _json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_gpus2_launches_two_ranks_itself():
    p = _run(["--gpus", "2", "--dry-plan", "--config", "cfg4", "--packets", "4096"])
    assert p.returncode == 0, p.stderr[-3000:]
    res = _json(p.stdout)
    assert res["n_gpus"] == 2 and res["config"]["world"] == 2
    ppr = res["config"]["packets_per_rank"]
    assert len(ppr) == 2 and sum(ppr) == 2 * 4096 and min(ppr) > 0     # cfg4: one global batch, hash-split
    assert res["config"]["device_per_rank"] == [0, 1]
    assert sum(res["config"]["sas_per_rank"]) == 2 * 1024


def test_gpus2_weak_scaling_configs_plan_full_batches():
    p = _run(["--gpus", "2", "--dry-plan", "--config", "cfg1", "--packets", "1000"])
    assert p.returncode == 0, p.stderr[-3000:]
    res = _json(p.stdout)
    assert res["config"]["packets_per_rank"] == [1000, 1000]


def test_gpus_more_than_the_node_has_fails_loudly():
    # more GPUs than any node has (this host has none, a GPU node at most 8):
    # a real (not dry) run must refuse, not report a smaller one
    p = _run(["--gpus", "64", "--steps", "1", "--warmup", "0"])
    assert p.returncode != 0
    assert not any(ln.startswith("{") for ln in p.stdout.splitlines())
    assert "refusing" in p.stderr


def test_world_size_mismatch_exits_nonzero():
    p = _run(["--gpus", "2", "--dry-plan"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert p.returncode == 2
    assert "WORLD_SIZE=1 but --gpus 2" in p.stderr


def test_single_rank_dry_plan():
    p = _run(["--dry-plan", "--packets", "64"])
    assert p.returncode == 0, p.stderr[-3000:]
    res = _json(p.stdout)
    assert res["n_gpus"] == 1 and res["config"]["packets_per_rank"] == [64]
