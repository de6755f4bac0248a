"""Single-node rank launcher (parallel/launch.py) used by `bench.py --gpus N`
without torchrun: per-rank environment, exit-code propagation, kill-on-failure,
distinct-device counting, and bench.py's own argument handling (CPU)."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rank_envs_contract():
    envs = launch.rank_envs(4, 29555, base={"FOO": "1"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555" for e in envs)
    assert all(e["LOCAL_RANK"] == e["RANK"] and e["FOO"] == "1" for e in envs)
    assert all(e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)
    with pytest.raises(ValueError):
        launch.rank_envs(0, 1)


def test_launched_by_torchrun():
    assert launch.launched_by_torchrun({"WORLD_SIZE": "2", "RANK": "1"})
    assert not launch.launched_by_torchrun({"WORLD_SIZE": "2"})
    assert not launch.launched_by_torchrun({})


def test_distinct_devices():
    assert launch.distinct_devices([("h", 0), ("h", 0)]) == 1
    assert launch.distinct_devices([("h", 0), ("h", 1), ("h", 2), ("h", 3)]) == 4
    assert launch.distinct_devices([("a", 0), ("b", 0)]) == 2


def _script(tmp_path, body):
    p = tmp_path / "child.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_launch_local_runs_every_rank(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    s = _script(tmp_path, f"""
        import json, os, sys
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        json.dump({{k: os.environ[k] for k in keys}} | {{"argv": sys.argv[1:]}},
                  open(os.path.join({str(out)!r}, os.environ["RANK"] + ".json"), "w"))
    """)
    rc = launch.launch_local(["--steps", "3"], 3, script=s, timeout_s=60)
    assert rc == 0
    recs = [json.load(open(out / f"{r}.json")) for r in range(3)]
    assert [r["RANK"] for r in recs] == ["0", "1", "2"]
    assert len({r["MASTER_PORT"] for r in recs}) == 1
    assert all(r["argv"] == ["--steps", "3"] and r["WORLD_SIZE"] == "3" for r in recs)


def test_launch_local_failure_kills_job(tmp_path):
    """Rank 1 fails: the job exits with its code and rank 0 (blocked, as on a
    dead RCCL peer) is terminated instead of hanging."""
    s = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)
    """)
    t0 = time.monotonic()
    rc = launch.launch_local([], 2, script=s, timeout_s=100)
    assert rc == 3
    assert time.monotonic() - t0 < 30


def test_launch_local_timeout(tmp_path):
    s = _script(tmp_path, "import time\ntime.sleep(60)\n")
    assert launch.launch_local([], 2, script=s, timeout_s=1.0) == 124


def test_bench_self_launches_without_torchrun(tmp_path):
    """`bench.py --gpus 2` outside torchrun re-runs itself as 2 ranks: with the
    GPU call stubbed out by a sitecustomize, the children see the launcher env."""
    stub = tmp_path / "stub"
    stub.mkdir()
    (stub / "sitecustomize.py").write_text(textwrap.dedent(f"""
        import os, sys
        if os.environ.get("RANK") is not None and sys.argv and sys.argv[0].endswith("bench.py"):
            open(os.path.join({str(tmp_path)!r}, "rank" + os.environ["RANK"]), "w").write(
                os.environ["WORLD_SIZE"] + " " + " ".join(sys.argv[1:]))
            os._exit(0)
    """))
    env = {k: v for k, v in os.environ.items() if k not in launch.RANK_ENV}
    env["PYTHONPATH"] = str(stub) + os.pathsep + ROOT
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    for k in range(2):
        assert (tmp_path / f"rank{k}").read_text() == "2 --gpus 2 --steps 1"


def test_rank_envs_drop_torchrun_agent_vars():
    """A job started from inside a torchrun rank (bench.py's sub-runs) must host
    its own store, not join the agent's."""
    base = {"TORCHELASTIC_USE_AGENT_STORE": "True", "TORCHELASTIC_RUN_ID": "x", "GROUP_WORLD_SIZE": "1",
            "ROLE_WORLD_SIZE": "8", "RANK": "5", "WORLD_SIZE": "8", "KEEP": "1"}
    envs = launch.rank_envs(2, 29600, base=base)
    for e in envs:
        assert not any(k.startswith("TORCHELASTIC_") for k in e)
        assert "GROUP_WORLD_SIZE" not in e and "ROLE_WORLD_SIZE" not in e and e["KEEP"] == "1"
        assert e["WORLD_SIZE"] == "2"
