"""Launch-plan compiler: graph (slice) -> fused kernel steps.

The reference re-creates each slice as a Keras model on the worker
(`src/node.py:40-45,77-78`) and calls `model.predict` per request
(`src/node.py:177`), i.e. one TF op per Keras layer.  Here a slice is
compiled once into a short list of fused steps that map 1:1 onto our HIP
kernels:

* ``conv``     Conv2D [+BN folded] [+Add residual] [+ReLU / ReLU6, or the
               Conv2D's own activation='relu']; a preceding ZeroPadding2D or
               'same' padding (any stride, TF placement) becomes explicit pads
* ``maxpool``  [ZeroPadding2D +] MaxPooling2D ('same' padding excluded from the max)
* ``avgpool``  AveragePooling2D (padding excluded from the mean)
* ``dwconv``   DepthwiseConv2D [+BN folded] [+ReLU/ReLU6], explicit pads
* ``concat``   Concatenate along channels (one copy launch per input)
* ``copy``     a Flatten/Dropout that the slice emits under its own name
               (otherwise they alias their input: Dropout everywhere,
               Flatten when a Dense consumes it)
* ``bn``       standalone BN [+ReLU] (only when a cut exposes the raw conv output)
* ``add``      standalone Add [+ReLU]
* ``relu``, ``pad`` (materialised ZeroPadding2D), ``gap``,
* ``dense``    Dense (+softmax) as a GEMM on the conv kernel + row softmax
* ``pack``     fp32 image -> bf16 NHWC padded to 8 channels (stem input)
* ``stem``     fp32 image -> conv1 7x7/s2 (+BN, ReLU) [-> pool1 3x3/s2] in one
               launch (csrc/kernels/stem.hip); replaces pack+conv[+maxpool]
               when the cut allows it

Fusion never hides a tensor that the slice must emit or that another layer
consumes, so any cut (including the multi-tensor frontier of BASELINE
config 2) is executable.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set

from ..graph.ir import ACT_MODE, Graph, _pair, same_pads


@dataclass
class Step:
    kind: str
    out: str                       # tensor name produced (name of the last covered layer)
    ins: List[str]                 # tensor names consumed (physical names)
    covers: List[str]              # graph layers executed by this step
    p: Dict = field(default_factory=dict)


def _phys(name: str, packed: Set[str]) -> str:
    return name + "#packed" if name in packed else name


def compile_plan(g: Graph, outputs: Optional[List[str]] = None, fp32: bool = False,
                 device_fusions: bool = True) -> List[Step]:
    """fp32=True: the fp32 execution path (csrc/kernels/conv_f32.hip) keeps the
    image as it is (no bf16 pack, so no stem fusion) and runs sibling convs as
    separate GEMMs.  device_fusions=False (with fp32): only the per-layer
    fusions (BN folding, conv epilogues, folded pads) -- the plan of the native
    CPU path (runtime/cpu_executor.py), which has no stem / pair / merged
    sibling kernels."""
    outputs = list(outputs or g.output_names)
    outset = set(outputs)
    cons = g.consumers()
    done: Set[str] = set()
    produced: Set[str] = set()
    steps: List[Step] = []
    packed: Set[str] = set()
    pad_fold: Dict[str, tuple] = {}     # consumer layer -> (source tensor, pad)

    def single(n: str) -> Optional[str]:
        """The unique consumer of n, if n may be fused into it."""
        if n in outset:
            return None
        c = cons.get(n, [])
        return c[0] if len(c) == 1 else None

    for n in g.order:
        L = g.layers[n]
        if L.op != "input":
            continue
        produced.add(n)
        done.add(n)
        c = L.out_shape[-1] if L.out_shape else 0
        # the user's fp32 image becomes bf16 NHWC with channels padded to 8 (a pure cast when C % 8 == 0)
        if len(L.out_shape) == 3 and L.attrs.get("stands_for", "input") == "input" and not fp32:
            packed.add(n)
            steps.append(Step("pack", n + "#packed", [n], [], {"cin": c, "cpad": ((c + 7) // 8) * 8}))

    alias: Dict[str, str] = {}          # identity / flatten-into-dense layers -> the tensor they pass on

    def R(t: str) -> str:
        return _phys(alias.get(t, t), packed)

    def same(n: str, L, k) -> tuple:
        """Explicit pads of a 'same' conv / pool (TF: the odd pixel after)."""
        h, w = g.layers[L.inputs[0]].out_shape[:2]
        kh, kw = _pair(k)
        s = L.attrs.get("stride", 1)
        return same_pads(h, kh, s), same_pads(w, kw, s)

    def act_mode(c: Optional[str]) -> int:
        """Kernel ActMode of a fusible activation layer (ReLU, ReLU6, swish, sigmoid, ...), 0 if `c`
        is not one (LeakyReLU needs its slope: it runs as its own step)."""
        if c is None:
            return 0
        Lc = g.layers[c]
        if Lc.op == "act":
            return 0 if Lc.attrs["fn"] == "leaky_relu" else ACT_MODE[Lc.attrs["fn"]]
        if Lc.op != "relu":
            return 0
        mv = Lc.attrs.get("max_value")
        if mv is None:
            return 1
        if float(mv) == 6.0:
            return 2
        raise NotImplementedError(f"ReLU(max_value={mv}) ({c})")

    def own_act(n: str, L) -> int:
        """ActMode of a conv / dense layer's own `activation` argument."""
        act = L.attrs.get("activation")
        if act in (None, "linear"):
            return 0
        if act not in ACT_MODE or act == "leaky_relu":
            raise NotImplementedError(f"{L.op} activation {act!r} ({n})")
        return ACT_MODE[act]

    for n in g.order:
        if n in done:
            continue
        L = g.layers[n]
        a = L.attrs
        if L.op == "zeropad":
            c = single(n)
            if (c is not None and g.layers[c].op in ("conv", "dwconv", "maxpool", "avgpool")
                    and g.layers[c].attrs.get("padding", "valid") == "valid"):
                pad_fold[c] = (L.inputs[0], a["pad"])
                done.add(n)
                continue
            steps.append(Step("pad", n, [R(L.inputs[0])], [n], {"pad": a["pad"]}))
        elif L.op in ("conv", "dwconv"):
            src = L.inputs[0]
            pads = ((0, 0), (0, 0))
            cover = [n]
            if n in pad_fold:
                src, pads = pad_fold[n]
                cover = [g.layers[n].inputs[0], n]
            if a.get("padding", "valid") == "same":
                pads = same(n, L, a["kernel"])
            bn = None
            relu = 0
            res = None
            out = n
            post_act = 0                        # an activation the MFMA epilogue does not take (swish, ...)
            if own_act(n, L):
                relu = own_act(n, L)            # Conv2D(activation=...): nothing after it fuses
                if L.op == "conv" and relu > 2:
                    post_act, relu = relu, 0
            else:
                c1 = single(n)
                if c1 is not None and g.layers[c1].op == "bn":
                    bn = c1
                    cover.append(c1)
                    out = c1
                    c2 = single(c1)
                    feed = c1                       # the tensor the residual Add sees from this branch
                    while (c2 is not None and g.layers[c2].op == "identity"
                           and single(c2) is not None and g.layers[single(c2)].op == "add"):
                        cover.append(c2)            # drop-connect Dropout between the BN and the residual Add
                        feed, c2 = c2, single(c2)
                    if act_mode(c2) and (L.op == "dwconv" or act_mode(c2) <= 2):
                        relu = act_mode(c2)
                        cover.append(c2)
                        out = c2
                    elif (L.op == "conv" and c2 is not None and g.layers[c2].op == "add"
                          and len(g.layers[c2].inputs) == 2):
                        other = [i for i in g.layers[c2].inputs if i != feed]
                        if len(other) == 1 and alias.get(other[0], other[0]) in produced:
                            res = alias.get(other[0], other[0])
                            cover.append(c2)
                            out = c2
                            c3 = single(c2)
                            if 0 < act_mode(c3) <= 2:
                                relu = act_mode(c3)
                                cover.append(c3)
                                out = c3
                elif act_mode(c1) and (L.op == "dwconv" or act_mode(c1) <= 2):
                    relu = act_mode(c1)
                    cover.append(c1)
                    out = c1
            kernel = tuple(_pair(a["kernel"]))
            if L.op == "dwconv":
                steps.append(Step("dwconv", out, [R(src)], cover,
                                  {"conv": n, "bn": bn, "relu": relu, "pads": pads, "stride": a.get("stride", 1),
                                   "kernel": kernel}))
            else:
                cv_out = out if not post_act else n + "#preact"
                steps.append(Step("conv", cv_out, [R(src)] + ([res] if res else []), cover,
                                  {"conv": n, "bn": bn, "relu": relu, "residual": res, "pads": pads,
                                   "stride": a.get("stride", 1), "kernel": kernel,
                                   "filters": a["filters"], "packed_input": src in packed}))
                if post_act:
                    steps.append(Step("act", out, [cv_out], [], {"mode": post_act, "alpha": 0.3}))
            done.update(cover)
        elif L.op in ("maxpool", "avgpool"):
            src = L.inputs[0]
            pads = ((0, 0), (0, 0))
            cover = [n]
            pad_zero = True                     # a folded ZeroPadding2D: the zeros take part
            if n in pad_fold:
                src, pads = pad_fold[n]
                cover = [L.inputs[0], n]
            if a.get("padding", "valid") == "same":
                pads = same(n, L, a["pool"])
                pad_zero = False                # Keras 'same' pooling ignores the padding
            if L.op == "avgpool" and n in pad_fold:
                raise NotImplementedError(f"ZeroPadding2D before AveragePooling2D ({n})")
            steps.append(Step(L.op, n, [R(src)], cover,
                              {"pool": a["pool"], "stride": a["stride"], "pads": pads, "pad_zero": pad_zero}))
            done.update(cover)
        elif L.op == "bn":
            cover = [n]
            relu = 0
            out = n
            c = single(n)
            if act_mode(c):
                relu = act_mode(c)
                cover.append(c)
                out = c
            steps.append(Step("bn", out, [R(L.inputs[0])], cover, {"bn": n, "relu": relu}))
            done.update(cover)
        elif L.op == "add":
            cover = [n]
            relu = 0
            out = n
            c = single(n)
            if act_mode(c):
                relu = act_mode(c)
                cover.append(c)
                out = c
            if len(L.inputs) != 2:
                raise NotImplementedError("add with != 2 inputs")
            steps.append(Step("add", out, [R(i) for i in L.inputs], cover, {"relu": relu}))
            done.update(cover)
        elif L.op == "relu":
            steps.append(Step("relu", n, [R(L.inputs[0])], [n], {"mode": act_mode(n)}))
            done.add(n)
        elif L.op == "act":
            steps.append(Step("act", n, [R(L.inputs[0])], [n],
                              {"mode": ACT_MODE[a["fn"]], "alpha": float(a.get("alpha", 0.3))}))
            done.add(n)
        elif L.op == "binary":
            cover = [n]
            out = n
            mode = 0
            c = single(n)
            if act_mode(c):
                mode = act_mode(c)
                cover.append(c)
                out = c
            steps.append(Step("binary", out, [R(i) for i in L.inputs], cover, {"fn": a["fn"], "act": mode}))
            done.update(cover)
        elif L.op in ("rescale", "normalization"):
            steps.append(Step("affine", n, [R(L.inputs[0])], [n], {"layer": n}))
            done.add(n)
        elif L.op == "gmp":
            steps.append(Step("gmp", n, [R(L.inputs[0])], [n]))
            done.add(n)
        elif L.op == "reshape":
            src_shape = g.layers[L.inputs[0]].out_shape
            if device_fusions and src_shape[-1] != L.out_shape[-1] and (src_shape[-1] % 8 or L.out_shape[-1] % 8):
                raise NotImplementedError(f"Reshape {src_shape} -> {L.out_shape} ({n}): channels are padded to 8")
            if n in outset:
                steps.append(Step("copy", n, [R(L.inputs[0])], [n]))
                done.add(n)
            else:
                alias[n] = alias.get(L.inputs[0], L.inputs[0])
                done.add(n)
                continue
        elif L.op == "concat":
            steps.append(Step("concat", n, [R(i) for i in L.inputs], [n],
                              {"channels": [g.layers[i].out_shape[-1] for i in L.inputs]}))
            done.add(n)
        elif L.op in ("identity", "flatten"):
            c = single(n)
            src_shape = g.layers[L.inputs[0]].out_shape
            if L.op == "identity" or (c is not None and g.layers[c].op == "dense"):
                if n in outset:                 # the slice must emit it under its own name
                    steps.append(Step("copy", n, [R(L.inputs[0])], [n]))
                else:
                    alias[n] = alias.get(L.inputs[0], L.inputs[0])
                    done.add(n)
                    continue
            else:
                steps.append(Step("copy", n, [R(L.inputs[0])], [n]))
            if device_fusions and L.op == "flatten" and len(src_shape) == 3 and src_shape[-1] % 8:
                raise NotImplementedError(f"Flatten of a {src_shape[-1]}-channel tensor ({n}): channels are padded to 8")
            done.add(n)
        elif L.op == "gap":
            steps.append(Step("gap", n, [R(L.inputs[0])], [n]))
            done.add(n)
        elif L.op == "dense":
            act = a.get("activation")
            mode = 0 if act == "softmax" else own_act(n, L)
            if mode > 2:                        # not an MFMA-epilogue activation: its own step
                steps.append(Step("dense", n + "#preact", [R(L.inputs[0])], [n],
                                  {"units": a["units"], "softmax": False, "relu": 0, "layer": n}))
                steps.append(Step("act", n, [n + "#preact"], [], {"mode": mode, "alpha": 0.3}))
            else:
                steps.append(Step("dense", n, [R(L.inputs[0])], [n],
                                  {"units": a["units"], "softmax": act == "softmax", "relu": mode, "layer": n}))
            done.add(n)
        elif L.op == "softmax":
            steps.append(Step("softmax", n, [R(L.inputs[0])], [n]))
            done.add(n)
        else:
            raise NotImplementedError(f"op {L.op}")
        produced.add(steps[-1].out)
    missing = [o for o in outputs if o not in produced]
    if missing:
        raise RuntimeError(f"plan does not produce outputs {missing}")
    if fp32 and not device_fusions:
        return steps
    if fp32:
        if os.environ.get("ADAPT_NO_STEM", "0") != "1":
            steps = _fuse_stem_f32(g, steps, outset)
        if os.environ.get("ADAPT_FUSED_PAIR_F32", "1") == "1":
            steps = fuse_pairs(g, steps, outset, fp32=True)
        if os.environ.get("ADAPT_NO_SIBLINGS", "0") != "1":
            steps = merge_siblings(steps)
        return steps
    if os.environ.get("ADAPT_FUSED_BOTTLENECK", "1") == "1":
        steps = fuse_bottlenecks(g, steps, outset)
    # ADAPT_FUSED_PAIR=0 keeps the two launches (A/B: profiles/r2/experiments/pair/)
    if os.environ.get("ADAPT_FUSED_PAIR", "1") == "1":
        steps = fuse_pairs(g, steps, outset)
    if os.environ.get("ADAPT_NO_STEM", "0") != "1":
        steps = _fuse_stem(g, steps, outset)
    if os.environ.get("ADAPT_NO_SIBLINGS", "0") != "1":
        steps = merge_siblings(steps)
    return steps


def fuse_bottlenecks(g: Graph, steps: List[Step], outset: Set[str]) -> List[Step]:
    """1x1 (->64, ReLU) -> 3x3 s1 p1 (64->64, ReLU) -> 1x1 (64->256) + shortcut + ReLU
    ==> one ``bottleneck`` step (csrc/kernels/bottleneck.hip) when the block's
    input is H x W x 256 (identity shortcut) or H x W x 64 with a stride-1 1x1
    projection shortcut, H and W multiples of 8, and no intermediate tensor is
    needed elsewhere (a cut inside the block keeps it unfused).  ResNet
    stage 2: three launches and two 51 MB round trips per block become one."""
    def users(t: str) -> List[int]:
        return [j for j, st in enumerate(steps) if t in st.ins]

    def conv(j, k, filters, relu, res):
        st = steps[j]
        p = st.p
        return (st.kind == "conv" and p.get("kernel") == k and p.get("stride") == 1 and p.get("filters") == filters
                and p.get("relu") == relu and bool(p.get("residual")) == res and not p.get("packed_input")
                and not p.get("sibling"))

    drop: Set[int] = set()
    repl: Dict[int, Step] = {}
    for j3, s3 in enumerate(steps):
        if j3 in drop or not conv(j3, (1, 1), 256, 1, True):
            continue
        y2, sc = s3.ins[0], s3.ins[1]
        u2 = [j for j, st in enumerate(steps) if st.out == y2]
        if len(u2) != 1 or y2 in outset or users(y2) != [j3] or not conv(u2[0], (3, 3), 64, 1, False):
            continue
        j2 = u2[0]
        if steps[j2].p["pads"] != ((1, 1), (1, 1)):
            continue
        y1 = steps[j2].ins[0]
        u1 = [j for j, st in enumerate(steps) if st.out == y1]
        if len(u1) != 1 or y1 in outset or users(y1) != [j2] or not conv(u1[0], (1, 1), 64, 1, False):
            continue
        j1 = u1[0]
        x = steps[j1].ins[0]
        xl = g.layers[x.split("#")[0]]
        if len(xl.out_shape) != 3 or xl.out_shape[0] % 8 or xl.out_shape[1] % 8:
            continue
        proj = None
        if sc == x and xl.out_shape[2] == 256:
            pass                                          # identity shortcut
        elif xl.out_shape[2] == 64:
            up = [j for j, st in enumerate(steps) if st.out == sc]
            if (len(up) != 1 or sc in outset or users(sc) != [j3] or not conv(up[0], (1, 1), 256, 0, False)
                    or steps[up[0]].ins[0] != x):
                continue
            proj = up[0]
        else:
            continue
        group = [j1, j2, j3] + ([proj] if proj is not None else [])
        covers = [c for jj in sorted(group) for c in steps[jj].covers]
        p = {"c1": steps[j1].p, "c2": steps[j2].p, "c3": steps[j3].p,
             "proj": steps[proj].p if proj is not None else None, "cin": xl.out_shape[2]}
        repl[j3] = Step("bottleneck", s3.out, [x], covers, p)
        drop.update(jj for jj in group if jj != j3)
    return [repl.get(j, st) for j, st in enumerate(steps) if j not in drop]


def fuse_pairs(g: Graph, steps: List[Step], outset: Set[str], fp32: bool = False) -> List[Step]:
    """1x1 (CIN -> CO) + BN + residual + ReLU (block k's ``_out``) followed by the
    1x1 (CO -> CM) + BN + ReLU that is the next block's ``_1`` ==> one ``pair``
    step with two outputs (csrc/kernels/pw_pair.hip): y is still written (it is
    the next residual) but the second GEMM reads it from LDS, and the pair is
    one launch.  Only the stride-1 pairs inside a ResNet stage qualify.  Both
    outputs land in their own named buffers, so either may be a slice frontier.
    fp32: csrc/kernels/pw_pair_f32.hip, ResNet stage 2 (64 -> 256 -> 64) only."""
    from ..ops.conv import pair_f32_supported, pair_supported   # static shape tables, no device needed

    def conv1x1(st: Step, relu: int, res: bool) -> bool:
        p = st.p
        return (st.kind == "conv" and p.get("kernel") == (1, 1) and p.get("stride") == 1
                and p.get("pads") == ((0, 0), (0, 0)) and p.get("relu") == relu and bool(p.get("residual")) == res
                and not p.get("packed_input") and not p.get("sibling"))

    drop: Set[int] = set()
    repl: Dict[int, Step] = {}
    for ja, a in enumerate(steps):
        if ja in drop or ja in repl or not conv1x1(a, 1, True):
            continue
        users = [j for j, st in enumerate(steps) if a.out in st.ins]
        firsts = [j for j in users if steps[j].ins[0] == a.out and conv1x1(steps[j], 1, False)
                  and len(steps[j].ins) == 1]
        if len(firsts) != 1 or firsts[0] <= ja or firsts[0] in repl:
            continue
        jb = firsts[0]
        b = steps[jb]
        xl = g.layers[a.ins[0].split("#")[0]]
        if len(xl.out_shape) != 3:
            continue
        cin, co, cm = xl.out_shape[2], a.p["filters"], b.p["filters"]
        if not (pair_f32_supported(cin, co, cm) if fp32 else pair_supported(cin, co, cm)):
            continue
        p = {"c3": a.p, "c1": b.p, "out2": b.out, "cin": cin, "co": co, "cm": cm}
        repl[ja] = Step("pair", a.out, list(a.ins), a.covers + b.covers, p)
        drop.add(jb)
    return [repl.get(j, st) for j, st in enumerate(steps) if j not in drop]


def merge_siblings(steps: List[Step]) -> List[Step]:
    """Two 1x1 convs that read the same tensor with the same stride and no
    residual become ONE GEMM with N = N0 + N1 and two outputs: ResNet's
    projection shortcut ``conv{s}_block1_0`` and ``conv{s}_block1_1`` (one
    launch and one read of the block input instead of two; the kernels route
    columns >= N0 to the second output, csrc/kernels/kernels.h `epi_dst`).
    The merged step sits at the first sibling's position (its input is ready
    there); the second output merely becomes available earlier."""
    out: List[Step] = []
    taken: Set[int] = set()
    for i, st in enumerate(steps):
        if i in taken:
            continue
        p = st.p
        if st.kind == "conv" and not p.get("residual") and p.get("kernel") == (1, 1) and not p.get("packed_input"):
            for j in range(i + 1, min(i + 4, len(steps))):
                sj = steps[j]
                q = sj.p
                if (j not in taken and sj.kind == "conv" and sj.ins[0] == st.ins[0] and not q.get("residual")
                        and q.get("kernel") == (1, 1) and q["stride"] == p["stride"] and q["pads"] == p["pads"]
                        and p["filters"] % 256 == 0 and q["filters"] % 8 == 0):
                    # nothing between them may consume the first sibling's output before
                    # ... (it is produced at i either way) -- only the second moves earlier
                    p["sibling"] = dict(q)
                    p["out2"] = sj.out
                    p["relu2"] = q["relu"]
                    st.covers = st.covers + sj.covers
                    taken.add(j)
                    break
        out.append(st)
    return out


STEM_MAX_OW = 112     # csrc/kernels/stem.hip ST_OWMAX


def _fuse_stem_f32(g: Graph, steps: List[Step], outset: Set[str]) -> List[Step]:
    """fp32 path: conv(image, 7x7/s2, 3 -> 64, BN+ReLU) -> maxpool 3x3/s2 pad 1  ==>  one
    ``stem_f32`` step (csrc/kernels/stem_f32.hip).  The image is the conv's
    input as it is (the fp32 plan has no pack step)."""
    def users(t: str) -> List[int]:
        return [j for j, s in enumerate(steps) if t in s.ins]

    for i, cv in enumerate(steps):
        if cv.kind != "conv" or len(cv.ins) != 1 or g.layers[cv.ins[0]].op != "input":
            continue
        p = cv.p
        h, w, c = g.layers[cv.ins[0]].out_shape
        oh, ow = g.layers[p["conv"]].out_shape[:2]
        (pt, _), (pl, _) = p["pads"]
        if (p["kernel"] != (7, 7) or p["stride"] != 2 or p["filters"] != 64 or p["relu"] != 1 or p["residual"]
                or c != 3 or w % 4 or ow > STEM_MAX_OW or pl != 3 or cv.out in outset):
            continue
        mu = users(cv.out)
        if len(mu) != 1 or steps[mu[0]].kind != "maxpool":
            continue
        mp = steps[mu[0]]
        if not (mp.p["pool"] in (3, (3, 3)) and mp.p["stride"] in (2, (2, 2)) and mp.p["pads"] == ((1, 1), (1, 1))):
            continue
        stem = Step("stem_f32", mp.out, [cv.ins[0]], list(cv.covers) + list(mp.covers),
                    {"conv": p["conv"], "bn": p["bn"], "pads": p["pads"], "pool": True, "pool_pad": 1,
                     "filters": 64})
        return [stem if j == i else s for j, s in enumerate(steps) if j != mu[0]]
    return steps


def _fuse_stem(g: Graph, steps: List[Step], outset: Set[str]) -> List[Step]:
    """pack -> conv(7x7/s2, 64 filters, BN+ReLU) [-> maxpool 3x3/s2 pad 1]  ==>  one ``stem`` step."""
    def users(t: str) -> List[int]:
        return [j for j, s in enumerate(steps) if t in s.ins]

    for i, st in enumerate(steps):
        if st.kind != "pack" or st.p["cin"] > 4:
            continue
        u = users(st.out)
        if len(u) != 1 or steps[u[0]].kind != "conv":
            continue
        cv = steps[u[0]]
        p = cv.p
        oh, ow = g.layers[p["conv"]].out_shape[:2]
        if (p["kernel"] != (7, 7) or p["stride"] != 2 or p["filters"] != 64 or p["relu"] != 1 or p["residual"]
                or ow > STEM_MAX_OW):
            continue
        drop = {i, u[0]}
        covers = list(cv.covers)
        out = cv.out
        pool = None
        mu = users(cv.out)
        if cv.out not in outset and len(mu) == 1 and steps[mu[0]].kind == "maxpool":
            mp = steps[mu[0]]
            if mp.p["pool"] in (3, (3, 3)) and mp.p["stride"] in (2, (2, 2)) and mp.p["pads"] == ((1, 1), (1, 1)):
                pool = mp.p["pads"][0][0]
                covers += mp.covers
                out = mp.out
                drop.add(mu[0])
        stem = Step("stem", out, [st.ins[0]], covers,
                    {"conv": p["conv"], "bn": p["bn"], "pads": p["pads"], "pool": pool is not None,
                     "pool_pad": pool or 0, "filters": 64})
        first = min(drop)
        return [stem if j == first else s for j, s in enumerate(steps) if j == first or j not in drop]
    return steps
