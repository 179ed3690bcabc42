"""bench.py --gpus N without an external launcher: the launch plan (the
environment of every rank), exit-code propagation, the rank timeout, rank 0's stdout relayed, and
the WORLD_SIZE / --gpus consistency check.  CPU only: the children here are small Python
programs standing in for the ranks; the GPU rehearsal is `bench.py --gpus 2 --backend gloo`."""
import importlib.util
import json
import os
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_launch_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_argv_gpus(bench):
    assert bench.argv_gpus([]) == 1
    assert bench.argv_gpus(["--steps", "5", "--gpus", "8"]) == 8
    assert bench.argv_gpus(["--gpus=4"]) == 4


def test_launch_plan_env_per_rank(bench):
    argv = ["bench.py", "--gpus", "4", "--steps", "20"]
    plan = bench.launch_plan(4, argv, {"KEEP": "x", "RANK": "stale"}, 29511)
    assert len(plan) == 4
    for r, (cmd, env) in enumerate(plan):
        assert cmd[-len(argv):] == argv                 # the same command line for every rank
        assert cmd[0] == sys.executable
        assert env["RANK"] == env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1"
        assert env["MASTER_PORT"] == "29511"
        assert env["KEEP"] == "x"


def _child(code):
    return [sys.executable, "-c", code]


def test_run_ranks_all_ok_and_rank0_stdout(bench):
    plan = bench.launch_plan(3, [], dict(os.environ), 1)
    code = ("import os, json; r = int(os.environ['RANK']); "
            "print(json.dumps({'rank': r, 'world': int(os.environ['WORLD_SIZE'])}))")
    plan = [(_child(code), env) for _, env in plan]
    with tempfile.TemporaryFile("w+") as out, tempfile.TemporaryFile("w+") as err:
        rc = bench.run_ranks(plan, timeout_s=60, out=out, err=err)
        out.seek(0)
        err.seek(0)
        lines = out.read().splitlines()
        other = err.read()
    assert rc == 0
    assert [json.loads(x) for x in lines] == [{"rank": 0, "world": 3}]     # only rank 0's line
    assert '"rank": 1' in other and '"rank": 2' in other


def test_run_ranks_failure_propagates_and_stops_others(bench):
    env = dict(os.environ)
    plan = [(_child("import time; time.sleep(60)"), env),
            (_child("import sys; sys.exit(3)"), env)]
    with tempfile.TemporaryFile("w+") as out, tempfile.TemporaryFile("w+") as err:
        rc = bench.run_ranks(plan, timeout_s=60, out=out, err=err)
        err.seek(0)
        msg = err.read()
    assert rc == 3
    assert "rank 1 exited with 3" in msg


def test_run_ranks_signal_is_failure(bench):
    env = dict(os.environ)
    plan = [(_child("import os, signal; os.kill(os.getpid(), signal.SIGABRT)"), env)]
    with tempfile.TemporaryFile("w+") as out, tempfile.TemporaryFile("w+") as err:
        assert bench.run_ranks(plan, timeout_s=60, out=out, err=err) == 128 + 6


def test_run_ranks_timeout(bench):
    env = dict(os.environ)
    plan = [(_child("import time; time.sleep(60)"), env)] * 2
    with tempfile.TemporaryFile("w+") as out, tempfile.TemporaryFile("w+") as err:
        assert bench.run_ranks(plan, timeout_s=1.0, out=out, err=err) == 124


def test_world_size_mismatch_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 4" in r.stderr
