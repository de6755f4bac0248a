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


def _names(subs):
    return {s[0]: s for s in subs}


def test_subrun_plan_covers_every_baseline_config():
    """N=2: config 2's multi-tensor cut; N=4: config 5 (R152 4-stage bf16);
    N=8: config 3 (lz4 on the links); N>=2: config 4 (kill + recovery)."""
    b = _bench()
    a = b.parse(["--steps", "20", "--warmup", "5"])
    assert b.plan_subruns(a, 1, "nccl") == []
    s2 = _names(b.plan_subruns(a, 2, "nccl"))
    assert set(s2) == {"pp", "fault"}
    pp = s2["pp"][2]
    assert pp[pp.index("--part-at") + 1] == "conv3_block1_1_conv" and "--codec" not in pp
    assert s2["pp"][3] == 2 and "config 2" in s2["pp"][5]
    s4 = _names(b.plan_subruns(a, 4, "nccl"))
    assert set(s4) == {"pp", "pp_r152", "fault"}
    r152 = s4["pp_r152"][2]
    assert r152[r152.index("--model") + 1] == "resnet152" and r152[r152.index("--pp-dtype") + 1] == "bf16"
    assert s4["pp_r152"][3] == 4
    s8 = _names(b.plan_subruns(a, 8, "nccl"))
    pp8 = s8["pp"][2]
    assert pp8[pp8.index("--codec") + 1] == "lz4" and "--part-at" not in pp8 and s8["pp"][3] == 8
    f = s8["fault"][2]
    assert f[f.index("--workers") + 1] == "8" and f[f.index("--devices") + 1] == "each"
    assert "--hb-timeout" not in f and "--precision" not in f and "--transport" not in f   # DEFER defaults
    assert s8["fault"][1] == "fault" and s8["fault"][3] == 1
    # the steps / warmup / backend of the headline reach the pipeline sub-runs
    assert pp8[pp8.index("--steps") + 1] == "20" and pp8[pp8.index("--backend") + 1] == "nccl"
    assert b.plan_subruns(b.parse(["--no-subruns"]), 8, "nccl") == []
    assert set(_names(b.plan_subruns(b.parse(["--no-fault"]), 8, "nccl"))) == {"pp"}
    assert b.plan_subruns(b.parse(["--mode", "pp"]), 8, "nccl") == []


def test_subrun_time_limits_fit_the_driver():
    """Worst case (every sub-run of N hits its limit) stays under the budget, and the fault sub-run
    (last) keeps its whole limit even when the pipeline sub-runs before it hit theirs."""
    b = _bench()
    a = b.parse([])
    assert a.sub_budget <= 420
    assert all(v <= a.sub_budget for v in b.SUB_LIMIT_S.values())
    for world in (2, 4, 8):
        plan = b.plan_subruns(a, world, "nccl")
        assert plan[-1][0] == "fault"
        left, total = a.sub_budget, 0.0
        for i in range(len(plan)):
            lim = b.subrun_limit(plan, i, left)
            if plan[i][0] == "fault":
                assert lim == min(b.SUB_LIMIT_S["fault"], a.sub_budget)
                # fault_run's own phases fit its limit: ready wait + settle + window + drain
                assert b.fault_ready_timeout(lim, a.fault_duration) + a.fault_duration + 70.0 <= lim + 1e-9
            left -= lim                      # every sub-run takes its whole limit
            total += lim
        assert total <= a.sub_budget + 1e-9


class _FakeLaunch:
    def __init__(self, rc, write=None, sleep=0.0):
        self.rc, self.write, self.sleep = rc, write, sleep
        self.calls = []

    def launch_local(self, argv, nprocs, script=None, timeout_s=None, stdout=None, module=None):
        import time
        self.calls.append((list(argv), nprocs, script, module, timeout_s))
        out = argv[argv.index("--out" if "--out" in argv else "--json") + 1]
        if self.write is not None:
            with open(out, "w") as f:
                json.dump(self.write, f)
        if self.rc not in (0, 124):
            with open(out + ".rank1.err", "w") as f:
                f.write("rank 1: LinkError: pp8/job1/link1-2: communicator aborted")
        time.sleep(self.sleep)
        return self.rc


def test_subrun_failure_is_recorded_not_raised():
    b = _bench()
    ok = b.run_subrun("pp", "bench", ["--sub", "pp"], 2, 60, "x", _FakeLaunch(0, write={"value": 5.0, "ok": True}))
    assert ok["ok"] is True and ok["value"] == 5.0 and ok["label"] == "x" and "wall_s" in ok
    bad = b.run_subrun("pp", "bench", ["--sub", "pp"], 8, 60, "x", _FakeLaunch(3))
    assert bad["ok"] is False and "LinkError" in bad["error"] and bad["rc"] == 3
    hung = b.run_subrun("fault", "fault", ["--workers", "8"], 1, 60, "y", _FakeLaunch(124))
    assert hung["ok"] is False and hung["error"] == "time limit reached"
    # a record written before the job failed keeps its fields but is marked failed
    part = b.run_subrun("pp", "bench", [], 2, 60, "z", _FakeLaunch(3, write={"value": 1.0}))
    assert part["ok"] is False and part["value"] == 1.0

    class Boom:
        def launch_local(self, *a, **k):
            raise OSError("fork failed")
    boom = b.run_subrun("pp", "bench", [], 2, 60, "w", Boom())
    assert boom["ok"] is False and "fork failed" in boom["error"]


def test_headline_record_carries_failed_subruns():
    b = _bench()
    a = b.parse(["--steps", "20", "--warmup", "5"])
    subs = {"pp": {"ok": False, "error": "time limit reached"}, "fault": {"ok": True, "value": 150.0}}
    rec = b.make_record(a, world=8, n_gpus=8, backend="nccl", value=100000.0, elapsed=0.6, image=(224, 224, 3),
                        job={"global_batch": 256, "parallelism": "dp8", "part_at": []}, subs=subs)
    line = json.loads(json.dumps(rec))
    assert line["value"] == 100000.0 and line["pp"]["ok"] is False and line["fault"]["value"] == 150.0
    assert line["config"]["control"] == "gloo"


def test_subrun_of_a_real_job_fails_cleanly_without_gpu(tmp_path):
    """The real launcher + `bench.py --sub pp` on a machine without a GPU: every
    rank fails at device selection, and the parent records ok: false with the
    rank's error instead of raising."""
    import torch
    if torch.cuda.is_available():
        import pytest
        pytest.skip("needs a GPU-less host")
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel import launch
    b = _bench()
    rec = b.run_subrun("pp", "bench", ["--sub", "pp", "--steps", "1", "--warmup", "0"], 2, 120, "cpu", launch)
    assert rec["ok"] is False and rec["rc"] != 0 and "rank" in rec["error"]


def test_fault_subrun_through_the_launcher_on_cpu():
    """bench.py's config-4 sub-run path end to end on CPU workers: the fault run
    started as `python -m <pkg>.parallel.fault_run` by the rank launcher (the
    module-run package name once resolved to `__main__` and no worker started)."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel import launch
    b = _bench()
    argv = ["--workers", "2", "--devices", "cpu", "--model", "resnet_tiny", "--image", "32", "--batch", "1",
            "--duration", "4", "--kill-at", "2", "--ready-timeout", "60"]
    rec = b.run_subrun("fault", "fault", argv, 1, 150, "cpu twin", launch)
    assert rec["rc"] if not rec["ok"] else True, rec
    assert rec["ok"] is True and rec["exactly_once"] is True, rec
    assert rec["workers"] == 2 and rec["devices"] == ["cpu", "cpu"] and rec["precision"] == "fp32"
    assert rec["epoch_transport"] == "tcp" and rec["hb_timeout"] == 0.25 and rec["victim"] == "w1"
    # per-phase stamps of the fault run travel in its record (the 8-GPU node's first run must say where it was)
    for ph in ("dispatcher_up", "workers_spawned", "pipeline_up", "feeding", "kill", "drained", "teardown"):
        assert ph in rec["phases"], (ph, rec["phases"])
    assert rec["phases"]["kill"] >= rec["phases"]["feeding"] >= rec["phases"]["pipeline_up"]


def test_fault_run_expects_rccl_with_one_gpu_per_worker():
    """`--devices each` on enough GPUs at transport "auto" must run the hops over
    RCCL p2p; a tcp fallback there is recorded as a failure, not a success."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.parallel import fault_run
    assert fault_run.expected_transport("auto", ["cuda:0", "cuda:1", "cuda:2"]) == "rccl"
    assert fault_run.expected_transport("auto", ["cuda:0", "cuda:0"]) is None        # shared GPU: tcp links
    assert fault_run.expected_transport("auto", ["cpu", "cpu"]) is None
    assert fault_run.expected_transport("tcp", ["cuda:0", "cuda:1"]) is None
    assert fault_run.expected_transport("auto", ["cuda:0"]) is None


def test_phase_stamps_print_and_record(capsys):
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.utils.telemetry import (
        PhaseStamps)
    import sys
    st = PhaseStamps("bench r3", stream=sys.stderr)
    st.stamp("build_job", stage=3, link_init_ms={"2-3": 41.5})
    st.stamp("first_step")
    err = capsys.readouterr().err.splitlines()
    assert err[0].startswith("[bench r3 +") and "] build_job stage=3 link_init_ms={'2-3': 41.5}" in err[0]
    assert list(st.phases) == ["build_job", "first_step"] and st.phases["first_step"] >= st.phases["build_job"]
    assert PhaseStamps.arm_faulthandler(5.0) is None           # a limit inside the margin arms nothing


def test_pp_record_carries_pair_rates_and_phases():
    """The N > 1 pipeline record: rccl_ranks, the stage0 -> 1 rate, every pair's
    rate, each pair's link init and the per-phase stamps (bench.py run_pp)."""
    b = _bench()
    pp = b.make_pp_record(1000.0, 1.0, 20, 4, ["a", "b", "c"], "fp32", True, 1e-6, 1.0, 120.0, 4, "rccl-native")
    pp["p2p_GBps_pairs"] = {"0-1": 120.0, "1-2": 118.2, "2-3": 121.4}
    pp["link_init_ms"] = {"0-1": 40.0, "1-2": 38.0, "2-3": 44.0}
    pp["phases"] = {"init_process_group": 10.0, "build_job": 900.0, "first_step": 950.0, "teardown": 2000.0}
    line = json.loads(json.dumps(pp))
    assert line["rccl_ranks"] == 4 and line["p2p_GBps"] == 120.0 and len(line["p2p_GBps_pairs"]) == 3
    src = open(b.__file__).read()
    for key in ("p2p_GBps_pairs", "link_init_ms", '"phases"', "first_step", "arm_faulthandler", "ADAPT_SUB_LIMIT_S"):
        assert key in src


def test_every_planned_subrun_gets_time_at_n4():
    """Round 6's N=4 rehearsal skipped the plain pipeline sub-run ("budget spent"):
    the later sub-runs' reserved limits exceeded the budget.  Every planned
    sub-run now starts with at least 60 s even when the ones before it used
    their whole limits."""
    b = _bench()
    a = b.parse([])
    for world in (2, 4, 8):
        plan = b.plan_subruns(a, world, "nccl")
        left = a.sub_budget
        for i in range(len(plan)):
            lim = b.subrun_limit(plan, i, left)
            assert lim >= 60.0, (world, plan[i][0], lim)
            left -= lim
