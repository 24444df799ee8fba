"""bench.py's launcher and batch plan, without a GPU (STE_BENCH_PLAN_ONLY=1 stops each rank after
a gloo rendezvous and prints its plan).  `--gpus N` alone must start N ranks; under torchrun
WORLD_SIZE must match --gpus; the default global batch is c2's 64 at N=1 and c3's 256 at N>1,
split 256/N per rank in micro-batches of at most 64 (BASELINE configs)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(args, extra_env=None):
    env = dict(os.environ, STE_BENCH_PLAN_ONLY="1", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True, env=env,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]


@pytest.mark.parametrize("n,local,micro,acc", [(1, 64, 64, 1), (2, 128, 64, 2), (4, 64, 64, 1)])
def test_launcher_spawns_ranks_and_plans_c3(n, local, micro, acc):
    plans = _run(["--gpus", str(n)])
    assert sorted(p["rank"] for p in plans) == list(range(n))
    for p in plans:
        assert p["world"] == n and p["local_rank"] == p["rank"]
        assert (p["local_batch"], p["micro_batch"], p["accumulation_steps"]) == (local, micro, acc)
        assert p["global_batch"] == (64 if n == 1 else 256)
        assert p["scaling"] == "strong"


def test_plan_c3_eight_ranks_and_overrides():
    from importlib import util
    spec = util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    b = util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b.batch_plan(b.parse(["--gpus", "8"]), 8) == (256, 32, 32, 1, "strong")       # c3: 8 x 32
    assert b.batch_plan(b.parse(["--global-batch", "256"]), 1) == (256, 256, 64, 4, "strong")
    assert b.batch_plan(b.parse(["--batch", "64", "--gpus", "8"]), 8) == (512, 64, 64, 1, "weak")
    with pytest.raises(SystemExit):
        b.batch_plan(b.parse(["--global-batch", "100"]), 8)


def test_world_size_must_match_gpus():
    env = dict(os.environ, STE_BENCH_PLAN_ONLY="1", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4"], capture_output=True, text=True,
                       env=env, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
