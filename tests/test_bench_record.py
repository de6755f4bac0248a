"""bench.py's JSON contract (CPU): the headline line, the bf16 companion and the
pipeline sub-object the multi-GPU run adds (reference topology:
`src/dispatcher.py:39-53`)."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_defaults_are_reference_precision():
    b = _bench()
    a = b.parse([])
    assert a.dtype == "fp32" and a.gpus >= 1 and a.mode == "dp" and not a.no_bf16 and not a.no_pp


def test_record_fields_and_pp_subobject():
    b = _bench()
    a = b.parse(["--steps", "20", "--warmup", "5"])
    pp = b.make_pp_record(value=80000.0, elapsed=0.8, steps=20, stages=8, part_at=["conv2_block2_out"] * 7,
                          dtype="fp32", ok=True, max_logit_rel=2.5e-5, top1_agree=1.0, p2p_gbps=48.2,
                          rccl_ranks=8, backend="rccl-native")
    job = {"global_batch": 256, "parallelism": "dp8", "part_at": []}
    rec = b.make_record(a, world=8, n_gpus=8, backend="nccl", value=100000.0, elapsed=0.6, image=(224, 224, 3),
                        job=job, bf16={"value": 300000.0, "elapsed": 0.2}, pp=pp)
    line = json.loads(json.dumps(rec))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line, k
    assert line["dtype"] == "fp32" and line["value"] == 100000.0 and line["ms_per_step"] == 30.0
    assert line["value_bf16"] == 300000.0 and line["ms_per_step_bf16"] == 10.0
    assert line["config"]["parallelism"] == "dp8" and line["config"]["global_batch"] == 256
    assert line["scaling"] == "weak" and line["higher_is_better"] is True
    p = line["pp"]
    assert p["ok"] is True and p["stages"] == 8 and p["rccl_ranks"] == 8 and p["p2p_GBps"] == 48.2
    assert p["max_logit_rel"] == 2.5e-5 and p["ms_per_step"] == 40.0 and len(p["part_at"]) == 7


def test_record_single_gpu_has_no_pp():
    b = _bench()
    a = b.parse([])
    rec = b.make_record(a, world=1, n_gpus=1, backend="nccl", value=10000.0, elapsed=0.1, image=(224, 224, 3),
                        job={"global_batch": 32, "parallelism": "dp1", "part_at": []})
    assert "pp" not in rec and rec["config"]["backend"] is None and "value_bf16" not in rec


def test_pp_tolerances():
    b = _bench()
    assert b.PP_LOGIT_RTOL["bf16"] == 5e-2 and b.PP_LOGIT_RTOL["fp32"] <= 1e-3
