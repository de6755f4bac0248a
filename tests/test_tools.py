"""Sanitizer builds of the native host runtime, typed config resolution, CLI
planner, telemetry (CPU)."""
import os
import subprocess
import sys

import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import build_resnet
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.utils.config import AdaptConfig
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.utils.telemetry import Metrics, Tracer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd"


@pytest.mark.slow
@pytest.mark.parametrize("mode", ["asan", "tsan"])
def test_native_runtime_under_sanitizers(mode):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh"), mode], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "selftest passed" in r.stdout


def test_config_layers(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("model: resnet152\nbatch: 8\npart_at: [conv4_block1_out]\ntransport: rccl\n")
    cfg = AdaptConfig.load(str(p), env={"ADAPT_BATCH": "16", "ADAPT_ORDERED": "true"}, overrides={"codec": "zvc"})
    assert cfg.model == "resnet152" and cfg.batch == 16 and cfg.ordered and cfg.codec == "zvc"
    assert cfg.transport == "rccl" and cfg.cuts() == ["conv4_block1_out"]
    auto = AdaptConfig(part_at="auto:4", batch=32).cuts(build_resnet("resnet50"))
    assert len(auto) == 3
    assert AdaptConfig(part_at="a,b").cuts() == ["a", "b"]
    with pytest.raises(KeyError):
        AdaptConfig().replace(nope=1)


def test_cli_plan_and_summary():
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", PKG, "plan", "--stages", "4", "--batch", "32"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 0 and "part_at" in r.stdout and "part4" in r.stdout
    r = subprocess.run([sys.executable, "-m", PKG, "summary", "--model", "resnet_tiny"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 0 and "conv5_block1_out" in r.stdout


def test_tracer_and_metrics(tmp_path):
    t = Tracer(path=str(tmp_path / "trace.jsonl"))
    with t.span("stage", stage=1):
        pass
    t.event("complete", req=3)
    t.flush()
    lines = (tmp_path / "trace.jsonl").read_text().splitlines()
    assert len(lines) == 2 and '"stage"' in lines[0] and "dur_ms" in lines[0]
    m = Metrics()
    for v in range(100):
        m.observe("lat", float(v))
    m.inc("n", 3)
    s = m.summary()
    assert s["lat"]["n"] == 100 and 40 < s["lat"]["p50"] < 60 and s["counters"]["n"] == 3


def test_reference_demo_driver_runs_on_cpu():
    """examples/test.py = the reference's distributed demo (`test/test.py`): DEFER +
    two local CPU workers, multi-tensor cut, prints results and req/s."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "examples", "test.py"), "--devices", "cpu,cpu",
                        "--model", "resnet_tiny", "--task-size", "3", "--part-at", "conv3_block1_1_conv"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("(1, 10)") == 3 and "3 results in" in r.stdout and "Throughput:" in r.stdout
