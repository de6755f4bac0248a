"""Graph IR, ResNet builders, slicer, planner and plan compiler (CPU)."""
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.ir import Graph
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.planner import (
    articulation_points, balance_ratio, default_candidates, plan_cuts)
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph.slicer import (
    is_single_tensor_cut, partition, subgraph, validate_slices)
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import build_resnet
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.plan import compile_plan


@pytest.fixture(autouse=True)
def _no_pair_fusion(monkeypatch):
    """The step-count assertions below describe the plan without the stage-3
    1x1 pair fusion; test_plan_fused_pairs turns it back on."""
    monkeypatch.setenv("ADAPT_FUSED_PAIR", "0")


@pytest.fixture(scope="module")
def r50():
    return build_resnet("resnet50")


def test_resnet_param_counts_match_keras():
    # Keras applications totals
    assert build_resnet("resnet50").count_params() == 25_636_712
    assert build_resnet("resnet152").count_params() == 60_419_944


def test_resnet50_structure(r50):
    assert len(r50) == 177
    assert len(r50.weight_specs()) == 320          # get_weights() list length
    assert abs(r50.total_macs() / 1e9 - 3.858) < 0.01
    assert r50.order[:7] == ["input_1", "conv1_pad", "conv1_conv", "conv1_bn", "conv1_relu", "pool1_pad", "pool1_pool"]
    assert r50["conv3_block1_0_conv"].attrs["stride"] == 2 and r50["conv3_block1_1_conv"].attrs["stride"] == 2
    assert r50["conv5_block3_out"].out_shape == (7, 7, 2048)
    assert r50["predictions"].out_shape == (1000,)
    # shortcut conv exists only in block 1 of each stage
    assert "conv2_block2_0_conv" not in r50.layers and "conv4_block1_0_conv" in r50.layers


def test_graph_json_roundtrip(r50):
    g2 = Graph.from_json(r50.to_json())
    assert g2.order == r50.order
    assert g2["conv2_block1_2_conv"].attrs["kernel"] == (3, 3)
    assert g2.count_params() == r50.count_params()


def test_single_tensor_cut_matches_reference_semantics(r50):
    s = partition(r50, ["conv4_block1_out"])
    validate_slices(r50, s)
    assert s[0].outputs == ["conv4_block1_out"] and s[1].inputs == ["conv4_block1_out"]
    assert s[0].layers[-1] == "conv4_block1_out"
    assert s[0].name == "part1" and s[1].name == "part2"
    assert len(s[0].layers) + len(s[1].layers) == len(r50)


def test_multi_tensor_frontier_config2(r50):
    # BASELINE config 2: part_at=['conv3_block1_1_conv'] is not a single-tensor cut
    s = partition(r50, ["conv3_block1_1_conv"])
    validate_slices(r50, s)
    assert s[0].outputs == ["conv2_block3_out", "conv3_block1_1_conv"]
    assert not is_single_tensor_cut(r50, "conv3_block1_1_conv")
    assert is_single_tensor_cut(r50, "conv3_block1_out")
    assert "conv3_block1_0_conv" in s[1].layers


def test_relay_through_middle_stage(r50):
    # a tensor produced in part 1 and consumed in part 3 must be relayed by part 2
    s = partition(r50, ["conv3_block1_1_conv", "conv3_block1_2_conv"])
    validate_slices(r50, s)
    assert "conv2_block3_out" in s[1].relay


def test_bad_cuts(r50):
    with pytest.raises(KeyError):
        partition(r50, ["nope"])
    with pytest.raises(ValueError):
        partition(r50, ["conv4_block1_out", "conv3_block1_out"])   # out of order


def test_subgraph_inputs(r50):
    s = partition(r50, ["conv3_block1_1_conv"])
    sg = subgraph(r50, s[1])
    assert sg.input_names == ["conv2_block3_out", "conv3_block1_1_conv"]
    assert sg["conv3_block1_1_conv"].op == "input"
    assert sg.output_names == ["predictions"]


def test_planner_balanced(r50):
    cuts, per = plan_cuts(r50, 4)
    assert len(cuts) == 3 and balance_ratio(per) < 1.4
    assert all(c in default_candidates(r50) for c in cuts)
    cuts8, per8 = plan_cuts(r50, 8)
    assert len(cuts8) == 7
    assert plan_cuts(r50, 1)[0] == []
    r152 = build_resnet("resnet152")
    c, p = plan_cuts(r152, 4)
    assert balance_ratio(p) < 1.15
    assert "conv4_block1_out" in articulation_points(r50)
    assert "conv3_block1_1_conv" not in articulation_points(r50)


def test_planner_precision_model(r50):
    """fp32 jobs (DEFER's default) charge 4-byte frontiers on the links and the fp32 matrix rate; the cuts
    stay valid candidates and the link terms double against bf16 (verdict r4: the link-cost model assumed
    bf16 frontiers)."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.graph import planner as P
    hw = P.HwModel(link_bw=50e9)
    f32, b16 = P.for_precision(hw, "fp32"), P.for_precision(hw, "bf16")
    assert f32.act_bytes == 4 and b16.act_bytes == 2 and f32.mfma_flops <= P.FP32_MFMA_FLOPS
    cut = "conv3_block4_out"
    assert P.crossing_bytes(r50, cut, f32.act_bytes) == 2 * P.crossing_bytes(r50, cut, b16.act_bytes)
    c32, per32 = plan_cuts(r50, 4, hw=hw, precision="fp32", calibrated=False)
    c16, per16 = plan_cuts(r50, 4, hw=hw, precision="bf16", calibrated=False)
    assert all(c in default_candidates(r50) for c in c32 + c16)
    assert sum(per32) > 2 * sum(per16)          # fp32 stages are slower in the analytic model too


def test_plan_fuses_resnet(r50, monkeypatch):
    monkeypatch.setenv("ADAPT_FUSED_BOTTLENECK", "0")      # per-conv plan; the fused blocks are tested below
    steps = compile_plan(r50)
    kinds = [s.kind for s in steps]
    assert kinds.count("bn") == 0 and kinds.count("add") == 0
    # 52 convs: the 4 projection shortcuts share a GEMM with their block's first 1x1 conv
    assert kinds.count("conv") == 48 and kinds[0] == "stem" and kinds[-2:] == ["gap", "dense"]
    dual = [s for s in steps if s.p.get("out2")]
    assert [(s.out, s.p["out2"]) for s in dual] == [(f"conv{k}_block1_0_bn", f"conv{k}_block1_1_relu")
                                                    for k in (2, 3, 4, 5)]
    assert all(s.p["relu2"] and not s.p["relu"] for s in dual)
    st = steps[0]
    assert st.p["pads"] == ((3, 3), (3, 3)) and st.p["pool"] and st.out == "pool1_pool" and st.ins == ["input_1"]
    assert st.covers == ["conv1_pad", "conv1_conv", "conv1_bn", "conv1_relu", "pool1_pad", "pool1_pool"]
    res = [s for s in steps if s.kind == "conv" and s.p["residual"]]
    assert len(res) == 16 and all(s.out.endswith("_out") for s in res)


def test_plan_siblings_respect_cuts(r50):
    # a cut that exposes conv3_block1_1_conv leaves that conv unfused: no merge with the shortcut
    s = partition(r50, ["conv3_block1_1_conv"])
    st0 = compile_plan(subgraph(r50, s[0]))
    assert not any(x.p.get("out2", "").startswith("conv3") for x in st0)
    st1 = compile_plan(subgraph(r50, s[1]))
    assert all(x.p.get("out2") is None or x.out.startswith(("conv4", "conv5")) for x in st1)


def test_plan_stem_respects_cuts(r50, monkeypatch):
    # cut right after conv1_relu: the stem keeps the conv (fused pack) but not the pool
    s = partition(r50, ["conv1_relu"])
    st1 = compile_plan(subgraph(r50, s[0]))
    assert [x.kind for x in st1] == ["stem"] and not st1[0].p["pool"] and st1[0].out == "conv1_relu"
    st2 = compile_plan(subgraph(r50, s[1]))
    assert st2[0].kind == "maxpool"
    # cut inside the stem (raw conv output exposed): no stem kernel, generic path
    s = partition(r50, ["conv1_conv"])
    assert [x.kind for x in compile_plan(subgraph(r50, s[0]))] == ["pack", "conv"]
    monkeypatch.setenv("ADAPT_NO_STEM", "1")
    kinds = [x.kind for x in compile_plan(r50)]
    # 53 convs, 4 sibling pairs merged, the 3 stage-2 blocks (9 conv steps) fused into bottleneck steps
    assert kinds[:3] == ["pack", "conv", "maxpool"] and kinds.count("conv") == 40 and kinds.count("bottleneck") == 3


def test_plan_fused_bottlenecks(r50):
    steps = compile_plan(r50)
    kinds = [s.kind for s in steps]
    assert kinds[:4] == ["stem", "bottleneck", "bottleneck", "bottleneck"] and kinds.count("conv") == 39
    b = [s for s in steps if s.kind == "bottleneck"]
    assert [s.out for s in b] == [f"conv2_block{i}_out" for i in (1, 2, 3)]
    assert b[0].p["proj"] and not b[1].p["proj"] and not b[2].p["proj"]
    assert b[0].ins == ["pool1_pool"] and b[1].ins == ["conv2_block1_out"]
    # a cut inside block 2 leaves that block on the per-conv path
    s = partition(r50, ["conv2_block2_2_relu"])
    k0 = [x.kind for x in compile_plan(subgraph(r50, s[0]))]
    assert k0.count("bottleneck") == 1 and k0.count("conv") == 2


def test_plan_fused_pairs(r50, monkeypatch):
    """ADAPT_FUSED_PAIR=1: each stride-1 `_out` -> next `_1` pair of stage 3 becomes
    one two-output `pair` step (3 in ResNet-50); stages 4 and 5 have no kernel
    instance and stay unfused; a slice cut at the second conv's output still
    produces it (as the pair's second output)."""
    monkeypatch.setenv("ADAPT_FUSED_PAIR", "1")
    steps = compile_plan(r50)
    pairs = [s for s in steps if s.kind == "pair"]
    assert [s.out for s in pairs] == [f"conv3_block{i}_out" for i in (1, 2, 3)]
    assert [s.p["out2"] for s in pairs[:2]] == ["conv3_block2_1_relu", "conv3_block3_1_relu"]
    assert pairs[0].ins == ["conv3_block1_2_relu", "conv3_block1_0_bn"]
    assert (pairs[0].p["cin"], pairs[0].p["co"], pairs[0].p["cm"]) == (128, 512, 128)
    outs = {s.out for s in steps} | {s.p.get("out2") for s in steps}
    assert "conv3_block2_1_relu" in outs and "conv4_block2_1_relu" in outs
    s = partition(r50, ["conv3_block2_1_relu"])
    k0 = compile_plan(subgraph(r50, s[0]))
    assert k0[-1].kind == "pair" and k0[-1].p["out2"] == "conv3_block2_1_relu"
    monkeypatch.setenv("ADAPT_FUSED_PAIR", "0")
    assert not any(x.kind == "pair" for x in compile_plan(r50))


def test_plan_unfused_at_cut(r50):
    s = partition(r50, ["conv3_block1_1_conv"])
    st2 = compile_plan(subgraph(r50, s[1]))
    bn = [s for s in st2 if s.kind == "bn"]
    assert len(bn) == 1 and bn[0].p["relu"] and bn[0].out == "conv3_block1_1_relu"   # BN + ReLU standalone
    st1 = compile_plan(subgraph(r50, s[0]))
    assert st1[-1].kind == "conv" and st1[-1].out == "conv3_block1_1_conv" and not st1[-1].p["bn"]


def test_fp32_plan_fuses_stem_and_pool():
    """fp32 path (the reference's precision): conv1 7x7/s2 + BN + ReLU + pool1 become one stem_f32 step."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import build_resnet
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.plan import compile_plan
    g = build_resnet("resnet50")
    steps = compile_plan(g, fp32=True)
    assert steps[0].kind == "stem_f32" and steps[0].out == "pool1_pool"
    assert "conv1_conv" in steps[0].covers and "pool1_pool" in steps[0].covers
    assert not any(s.kind == "maxpool" for s in steps)


def test_fp32_plan_fuses_stage2_pairs_and_merges_siblings():
    """fp32 ResNet-50 plan: the two stride-1 stage-2 1x1 pairs (block k `_out` + block k+1 `_1`) become
    fp32 pair steps (pw_pair_f32.hip), and each stage's projection shortcut shares one GEMM with that
    block's `_1` conv (dual output)."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import build_resnet
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.plan import compile_plan
    g = build_resnet("resnet50")
    steps = compile_plan(g, fp32=True)
    pairs = [s for s in steps if s.kind == "pair"]
    assert [s.out for s in pairs] == ["conv2_block1_out", "conv2_block2_out"]
    assert [s.p["out2"] for s in pairs] == ["conv2_block2_1_relu", "conv2_block3_1_relu"]
    merged = [s for s in steps if s.kind == "conv" and s.p.get("out2")]
    assert len(merged) == 4 and all(s.p["kernel"] == (1, 1) for s in merged)
    covered = [c for s in steps for c in s.covers]
    assert len(covered) == len(set(covered))


@pytest.mark.parametrize("cut", ["conv2_block1_out", "conv2_block2_1_relu", "conv2_block2_out",
                                 "conv3_block1_1_conv", "conv4_block1_out"])
def test_fp32_plan_slices_cover_every_layer_once(cut):
    """fp32 plans of a 2-stage cut (including cuts that expose one output of a stage-2 pair, or the
    block-1 conv of a merged sibling GEMM) still compute every layer exactly once across the slices."""
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.resnet import build_resnet
    g = build_resnet("resnet50")
    s = partition(g, [cut])
    covered = []
    for sl in s:
        sg = subgraph(g, sl)
        for st in compile_plan(sg, fp32=True):
            covered += [c for c in st.covers if sg.layers[c].op != "input"]
    layers = [n for n in g.order if g.layers[n].op != "input"]
    assert sorted(covered) == sorted(layers)
