"""bench.py's own multi-GPU launcher (CPU): ``python bench.py --gpus N`` starts N ranks itself when
no outer launcher set WORLD_SIZE, and a --gpus / WORLD_SIZE mismatch aborts (the replacement of
the reference's sequential chunk loop, run.py:136-151, must really run N processes)."""
import os
import subprocess
import sys
import time

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_arg_forms():
    assert bench.gpus_arg(["--steps", "3"]) is None
    assert bench.gpus_arg(["--gpus", "4", "--steps", "3"]) == 4
    assert bench.gpus_arg(["--steps", "3", "--gpus=8"]) == 8


def test_check_world():
    assert bench.check_world(None, {}) == 1
    assert bench.check_world(None, {"WORLD_SIZE": "4"}) == 4
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == 4
    assert bench.check_world(1, {}) == 1
    with pytest.raises(SystemExit):
        bench.check_world(8, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        bench.check_world(2, {})   # --gpus 2 inside a process that is not one of 2 ranks


def test_rank_envs():
    envs = bench.rank_envs(3, 29555, {"HSA_ENABLE_IPC_MODE_LEGACY": "0", "X": "y"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    for e in envs:
        assert e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["X"] == "y"


def test_spawn_ranks_runs_every_rank(tmp_path):
    code = ("import os; open(os.path.join(%r, 'r' + os.environ['RANK']), 'w').write("
            "os.environ['WORLD_SIZE'] + ' ' + os.environ['LOCAL_RANK'] + ' ' + os.environ['MASTER_PORT'])" % str(tmp_path))
    rc = bench.spawn_ranks(4, [sys.executable, "-c", code], base_env=dict(os.environ))
    assert rc == 0
    got = [open(tmp_path / f"r{r}").read().split() for r in range(4)]
    assert [g[1] for g in got] == ["0", "1", "2", "3"]
    assert all(g[0] == "4" for g in got) and len({g[2] for g in got}) == 1


def test_spawn_ranks_failure_stops_the_others():
    # rank 1 fails at once; rank 0 would block (as in a collective) -- the launcher must stop it
    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(3) if r == 1 else time.sleep(120)"
    t0 = time.time()
    rc = bench.spawn_ranks(2, [sys.executable, "-c", code], base_env=dict(os.environ))
    assert rc == 3
    assert time.time() - t0 < 60


def test_bench_aborts_on_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "WORLD_SIZE=3" in p.stderr
    assert p.stdout.strip() == ""
