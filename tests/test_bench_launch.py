"""`python bench.py --gpus N` without torchrun launches its own N ranks (one fresh child
process per GPU with the torchrun environment) and relays rank 0's JSON line.  CPU: the
dry-run hook stops every child before any device work and prints its environment; a
child that fails makes the launcher fail.  GPU: two ranks of the real bench on the box's
one GPU (gloo rehearsal: RCCL refuses two ranks on one device) report n_gpus 2."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def test_launcher_spawns_n_ranks_with_torchrun_env():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-dry-run"], capture_output=True, text=True,
                       env=_env(BGCN_DIST_BACKEND="gloo"), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.strip().splitlines()]
    assert [d["RANK"] for d in lines] == ["0", "1", "2"]
    assert [d["LOCAL_RANK"] for d in lines] == ["0", "1", "2"]
    assert {d["WORLD_SIZE"] for d in lines} == {"3"}
    assert {d["MASTER_ADDR"] for d in lines} == {"127.0.0.1"}
    assert len({d["MASTER_PORT"] for d in lines}) == 1 and int(lines[0]["MASTER_PORT"]) > 0
    assert {d["BGCN_DIST_BACKEND"] for d in lines} == {"gloo"}


def test_launcher_under_torchrun_env_does_not_respawn():
    # WORLD_SIZE present (torchrun launched us): the process is one rank, not a launcher
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-dry-run"], capture_output=True, text=True,
                       env=_env(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1"), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1 and json.loads(lines[0])["RANK"] == "1"


def test_launcher_fails_when_a_rank_fails():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--workload", "no_such_workload"],
                       capture_output=True, text=True, env=_env(), timeout=120)
    assert r.returncode != 0
    assert "exited with status" in r.stderr


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--steps", "2", "--warmup", "1", "--pool", "2",
                        "--no-cpu-baseline"], capture_output=True, text=True,
                       env=_env(BGCN_DIST_BACKEND="gloo"), timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "dp2"
    assert line["invalid_steps"] == 0 and line["status"] == 0
    assert line["value"] > 0
