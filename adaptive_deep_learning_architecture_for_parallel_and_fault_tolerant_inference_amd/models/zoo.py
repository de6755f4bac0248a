"""Other `tf.keras.applications` families, rebuilt in our IR with Keras layer
names, creation order and `get_weights()` order.

The reference's dispatcher is model-agnostic: `DEFER.run_defer(model, ...)`
takes any Keras functional model and `dag_util.construct_model` cuts it at
named layers (`src/dispatcher.py:39-53`, `src/dag_util.py:50-62`); its demo
happens to use ResNet50 (`test/test.py:13`).  These builders give that
generality a concrete footing beyond ResNet (and `graph/keras_json.py`
takes an arbitrary Keras JSON):

* VGG16 / VGG19  (plain conv stacks, Conv2D(activation='relu'), Flatten, Dense relu)
* MobileNetV2    (ReLU6, DepthwiseConv2D, 'same' padding at stride 2, inverted residuals)
* DenseNet121/169/201 (pre-activation BN-ReLU, Concatenate, AveragePooling2D)
* EfficientNetB0-B7   (Rescaling/Normalization inside the model, swish, squeeze-excite Multiply)
* InceptionV3         (BatchNormalization(scale=False), asymmetric 1x7 / 7x1 kernels, multi-branch concats)

Parameter totals (Keras, include_top, 1000 classes; checked by tests):
VGG16 138,357,544; VGG19 143,667,240; MobileNetV2 3,538,984; DenseNet121 8,062,504;
EfficientNetB0 5,330,571; InceptionV3 23,851,784.
"""
from __future__ import annotations

from typing import Callable, Dict

from ..graph.ir import Graph, Layer


def _conv(g: Graph, x: str, name: str, filters: int, k: int, stride: int = 1, padding: str = "valid",
          use_bias: bool = True, activation=None) -> str:
    a = {"filters": filters, "kernel": (k, k), "stride": stride, "padding": padding, "use_bias": use_bias}
    if activation:
        a["activation"] = activation
    return g.add(Layer(name, "conv", [x], a))


# ------------------------------------------------------------------- VGG
VGG_BLOCKS = {"vgg16": (2, 2, 3, 3, 3), "vgg19": (2, 2, 4, 4, 4)}


def build_vgg(name: str = "vgg16", classes: int = 1000, input_shape=(224, 224, 3)) -> Graph:
    """`keras.applications.vgg16/vgg19` with include_top=True."""
    g = Graph(name)
    x = g.add(Layer("input_1", "input", [], {"shape": tuple(input_shape)}))
    for b, (n, f) in enumerate(zip(VGG_BLOCKS[name], (64, 128, 256, 512, 512)), start=1):
        for i in range(1, n + 1):
            x = _conv(g, x, f"block{b}_conv{i}", f, 3, padding="same", activation="relu")
        x = g.add(Layer(f"block{b}_pool", "maxpool", [x], {"pool": 2, "stride": 2, "padding": "valid"}))
    x = g.add(Layer("flatten", "flatten", [x]))
    x = g.add(Layer("fc1", "dense", [x], {"units": 4096, "activation": "relu", "use_bias": True}))
    x = g.add(Layer("fc2", "dense", [x], {"units": 4096, "activation": "relu", "use_bias": True}))
    g.add(Layer("predictions", "dense", [x], {"units": classes, "activation": "softmax", "use_bias": True}))
    g.output_names = ["predictions"]
    return g


# ------------------------------------------------------------- MobileNetV2
MBV2_EPS = 1e-3
# (filters, stride, expansion) per inverted-residual block, block_id = index
MBV2_BLOCKS = [(16, 1, 1), (24, 2, 6), (24, 1, 6), (32, 2, 6), (32, 1, 6), (32, 1, 6), (64, 2, 6), (64, 1, 6),
               (64, 1, 6), (64, 1, 6), (96, 1, 6), (96, 1, 6), (96, 1, 6), (160, 2, 6), (160, 1, 6), (160, 1, 6),
               (320, 1, 6)]


def _make_divisible(v: float, divisor: int = 8) -> int:
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    return new_v + divisor if new_v < 0.9 * v else new_v


def build_mobilenet_v2(name: str = "mobilenetv2_1.00_224", classes: int = 1000, input_shape=(224, 224, 3),
                       alpha: float = 1.0) -> Graph:
    """`keras.applications.MobileNetV2(alpha=1.0, include_top=True)`."""
    g = Graph(name)
    x = g.add(Layer("input_1", "input", [], {"shape": tuple(input_shape)}))
    x = _conv(g, x, "Conv1", _make_divisible(32 * alpha), 3, stride=2, padding="same", use_bias=False)
    x = g.add(Layer("bn_Conv1", "bn", [x], {"epsilon": MBV2_EPS}))
    x = g.add(Layer("Conv1_relu", "relu", [x], {"max_value": 6.0}))
    for block_id, (filters, stride, expansion) in enumerate(MBV2_BLOCKS):
        inp = x
        cin = g.layers[x].out_shape[-1]
        out_c = _make_divisible(int(filters * alpha), 8)
        if block_id:
            prefix = f"block_{block_id}_"
            x = _conv(g, x, prefix + "expand", expansion * cin, 1, padding="same", use_bias=False)
            x = g.add(Layer(prefix + "expand_BN", "bn", [x], {"epsilon": MBV2_EPS}))
            x = g.add(Layer(prefix + "expand_relu", "relu", [x], {"max_value": 6.0}))
        else:
            prefix = "expanded_conv_"
        if stride == 2:
            h = g.layers[x].out_shape[0]
            adj = 1 - h % 2                    # imagenet_utils.correct_pad(x, 3)
            x = g.add(Layer(prefix + "pad", "zeropad", [x], {"pad": ((1 - adj, 1), (1 - adj, 1))}))
        x = g.add(Layer(prefix + "depthwise", "dwconv", [x],
                        {"kernel": (3, 3), "stride": stride, "padding": "same" if stride == 1 else "valid",
                         "use_bias": False}))
        x = g.add(Layer(prefix + "depthwise_BN", "bn", [x], {"epsilon": MBV2_EPS}))
        x = g.add(Layer(prefix + "depthwise_relu", "relu", [x], {"max_value": 6.0}))
        x = _conv(g, x, prefix + "project", out_c, 1, padding="same", use_bias=False)
        x = g.add(Layer(prefix + "project_BN", "bn", [x], {"epsilon": MBV2_EPS}))
        if cin == out_c and stride == 1:
            x = g.add(Layer(prefix + "add", "add", [inp, x]))
    last = _make_divisible(1280 * alpha, 8) if alpha > 1.0 else 1280
    x = _conv(g, x, "Conv_1", last, 1, use_bias=False)
    x = g.add(Layer("Conv_1_bn", "bn", [x], {"epsilon": MBV2_EPS}))
    x = g.add(Layer("out_relu", "relu", [x], {"max_value": 6.0}))
    x = g.add(Layer("global_average_pooling2d", "gap", [x]))
    g.add(Layer("predictions", "dense", [x], {"units": classes, "activation": "softmax", "use_bias": True}))
    g.output_names = ["predictions"]
    return g


# ---------------------------------------------------------------- DenseNet
DENSENET_BLOCKS = {"densenet121": (6, 12, 24, 16), "densenet169": (6, 12, 32, 32), "densenet201": (6, 12, 48, 32)}
DN_EPS = 1.001e-5


def build_densenet(name: str = "densenet121", classes: int = 1000, input_shape=(224, 224, 3)) -> Graph:
    """`keras.applications.DenseNet121/169/201(include_top=True)`."""
    g = Graph(name)
    x = g.add(Layer("input_1", "input", [], {"shape": tuple(input_shape)}))
    x = g.add(Layer("zero_padding2d", "zeropad", [x], {"pad": ((3, 3), (3, 3))}))
    x = _conv(g, x, "conv1/conv", 64, 7, stride=2, use_bias=False)
    x = g.add(Layer("conv1/bn", "bn", [x], {"epsilon": DN_EPS}))
    x = g.add(Layer("conv1/relu", "relu", [x]))
    x = g.add(Layer("zero_padding2d_1", "zeropad", [x], {"pad": ((1, 1), (1, 1))}))
    x = g.add(Layer("pool1", "maxpool", [x], {"pool": 3, "stride": 2, "padding": "valid"}))
    blocks = DENSENET_BLOCKS[name]
    for s, n in enumerate(blocks, start=2):
        for i in range(1, n + 1):
            p = f"conv{s}_block{i}"
            y = g.add(Layer(p + "_0_bn", "bn", [x], {"epsilon": DN_EPS}))
            y = g.add(Layer(p + "_0_relu", "relu", [y]))
            y = _conv(g, y, p + "_1_conv", 128, 1, use_bias=False)
            y = g.add(Layer(p + "_1_bn", "bn", [y], {"epsilon": DN_EPS}))
            y = g.add(Layer(p + "_1_relu", "relu", [y]))
            y = _conv(g, y, p + "_2_conv", 32, 3, padding="same", use_bias=False)
            x = g.add(Layer(p + "_concat", "concat", [x, y]))
        if s < 2 + len(blocks) - 1:
            p = f"pool{s}"
            c = g.layers[x].out_shape[-1]
            y = g.add(Layer(p + "_bn", "bn", [x], {"epsilon": DN_EPS}))
            y = g.add(Layer(p + "_relu", "relu", [y]))
            y = _conv(g, y, p + "_conv", int(c * 0.5), 1, use_bias=False)
            x = g.add(Layer(p + "_pool", "avgpool", [y], {"pool": 2, "stride": 2, "padding": "valid"}))
    x = g.add(Layer("bn", "bn", [x], {"epsilon": DN_EPS}))
    x = g.add(Layer("relu", "relu", [x]))
    x = g.add(Layer("avg_pool", "gap", [x]))
    g.add(Layer("predictions", "dense", [x], {"units": classes, "activation": "softmax", "use_bias": True}))
    g.output_names = ["predictions"]
    return g


# ---------------------------------------------------------------- EfficientNet
EFFNET_BLOCKS = [  # kernel, repeats, filters_in, filters_out, expand_ratio, strides (se_ratio 0.25, id_skip)
    (3, 1, 32, 16, 1, 1), (3, 2, 16, 24, 6, 2), (5, 2, 24, 40, 6, 2), (3, 3, 40, 80, 6, 2),
    (5, 3, 80, 112, 6, 1), (5, 4, 112, 192, 6, 2), (3, 1, 192, 320, 6, 1)]
EFFNET_SCALE = {  # width, depth, resolution
    "efficientnetb0": (1.0, 1.0, 224), "efficientnetb1": (1.0, 1.1, 240), "efficientnetb2": (1.1, 1.2, 260),
    "efficientnetb3": (1.2, 1.4, 300), "efficientnetb4": (1.4, 1.8, 380), "efficientnetb5": (1.6, 2.2, 456),
    "efficientnetb6": (1.8, 2.6, 528), "efficientnetb7": (2.0, 3.1, 600)}


def build_efficientnet(name: str = "efficientnetb0", classes: int = 1000, input_shape=None) -> Graph:
    """`keras.applications.EfficientNetB0..B7(include_top=True, weights=None)` (tf.keras 2.15): Rescaling +
    Normalization preprocessing inside the model, swish, squeeze-excite (GAP -> Reshape -> 1x1 swish ->
    1x1 sigmoid -> Multiply), drop-connect Dropout before the residual Add (identity at inference)."""
    import math
    width, depth, res = EFFNET_SCALE[name]
    input_shape = tuple(input_shape or (res, res, 3))

    def round_filters(f: float) -> int:
        f *= width
        new = max(8, int(f + 4) // 8 * 8)
        return int(new + 8 if new < 0.9 * f else new)

    g = Graph(name)
    x = g.add(Layer("input_1", "input", [], {"shape": input_shape}))
    x = g.add(Layer("rescaling", "rescale", [x], {"scale": 1.0 / 255.0, "offset": 0.0}))
    x = g.add(Layer("normalization", "normalization", [x]))

    def correct_pad(t: str, k: int):
        h = g.layers[t].out_shape[0]
        adj = 1 - h % 2
        c = k // 2
        return ((c - adj, c), (c - adj, c))

    x = g.add(Layer("stem_conv_pad", "zeropad", [x], {"pad": correct_pad(x, 3)}))
    x = _conv(g, x, "stem_conv", round_filters(32), 3, stride=2, use_bias=False)
    x = g.add(Layer("stem_bn", "bn", [x], {"epsilon": 1e-3}))
    x = g.add(Layer("stem_activation", "act", [x], {"fn": "swish"}))
    total = float(sum(int(math.ceil(depth * r)) for _, r, *_ in EFFNET_BLOCKS))
    b = 0
    for i, (k, reps, f_in, f_out, expand, stride) in enumerate(EFFNET_BLOCKS):
        f_in, f_out = round_filters(f_in), round_filters(f_out)
        for j in range(int(math.ceil(depth * reps))):
            if j > 0:
                stride, f_in = 1, f_out
            p = f"block{i + 1}{chr(j + 97)}_"
            drop_rate = 0.2 * b / total
            inp = x
            filters = f_in * expand
            if expand != 1:
                x = _conv(g, x, p + "expand_conv", filters, 1, padding="same", use_bias=False)
                x = g.add(Layer(p + "expand_bn", "bn", [x], {"epsilon": 1e-3}))
                x = g.add(Layer(p + "expand_activation", "act", [x], {"fn": "swish"}))
            if stride == 2:
                x = g.add(Layer(p + "dwconv_pad", "zeropad", [x], {"pad": correct_pad(x, k)}))
            x = g.add(Layer(p + "dwconv", "dwconv", [x], {"kernel": (k, k), "stride": stride,
                                                        "padding": "valid" if stride == 2 else "same",
                                                        "use_bias": False}))
            x = g.add(Layer(p + "bn", "bn", [x], {"epsilon": 1e-3}))
            x = g.add(Layer(p + "activation", "act", [x], {"fn": "swish"}))
            se_f = max(1, int(f_in * 0.25))
            se = g.add(Layer(p + "se_squeeze", "gap", [x]))
            se = g.add(Layer(p + "se_reshape", "reshape", [se], {"shape": (1, 1, filters)}))
            se = _conv(g, se, p + "se_reduce", se_f, 1, padding="same", activation="swish")
            se = _conv(g, se, p + "se_expand", filters, 1, padding="same", activation="sigmoid")
            x = g.add(Layer(p + "se_excite", "binary", [x, se], {"fn": "mul"}))
            x = _conv(g, x, p + "project_conv", f_out, 1, padding="same", use_bias=False)
            x = g.add(Layer(p + "project_bn", "bn", [x], {"epsilon": 1e-3}))
            if stride == 1 and f_in == f_out:
                if drop_rate > 0:
                    x = g.add(Layer(p + "drop", "identity", [x]))
                x = g.add(Layer(p + "add", "add", [x, inp]))
            b += 1
    x = _conv(g, x, "top_conv", round_filters(1280), 1, padding="same", use_bias=False)
    x = g.add(Layer("top_bn", "bn", [x], {"epsilon": 1e-3}))
    x = g.add(Layer("top_activation", "act", [x], {"fn": "swish"}))
    x = g.add(Layer("avg_pool", "gap", [x]))
    x = g.add(Layer("top_dropout", "identity", [x]))
    g.add(Layer("predictions", "dense", [x], {"units": classes, "activation": "softmax", "use_bias": True}))
    g.output_names = ["predictions"]
    return g


# ------------------------------------------------------------- InceptionV3
def build_inception_v3(name: str = "inception_v3", classes: int = 1000, input_shape=(299, 299, 3)) -> Graph:
    """`keras.applications.InceptionV3(include_top=True)`.  Its conv2d_bn units are unnamed, so the
    layers carry Keras' auto-names of a fresh session (conv2d, conv2d_1, ..., batch_normalization_N,
    activation_N, max_pooling2d_N, average_pooling2d_N, concatenate_N) in creation order;
    BatchNormalization(scale=False) (no gamma), asymmetric 1x7 / 7x1 / 1x3 / 3x1 kernels.
    Weight-list order follows creation order: Keras' own `get_weights()` order for this
    multi-branch graph is unpinned here (no TensorFlow to compare with)."""
    g = Graph(name)
    cnt: Dict[str, int] = {}

    def auto(kind: str) -> str:
        i = cnt.get(kind, 0)
        cnt[kind] = i + 1
        return kind if i == 0 else f"{kind}_{i}"

    def cbn(x: str, f: int, kh: int, kw: int, padding: str = "same", stride: int = 1) -> str:
        x = g.add(Layer(auto("conv2d"), "conv", [x], {"filters": f, "kernel": (kh, kw), "stride": stride,
                                                       "padding": padding, "use_bias": False}))
        x = g.add(Layer(auto("batch_normalization"), "bn", [x], {"epsilon": 1e-3, "scale": False}))
        return g.add(Layer(auto("activation"), "relu", [x]))

    def maxpool(x: str) -> str:
        return g.add(Layer(auto("max_pooling2d"), "maxpool", [x], {"pool": 3, "stride": 2, "padding": "valid"}))

    def avgpool(x: str) -> str:
        return g.add(Layer(auto("average_pooling2d"), "avgpool", [x], {"pool": 3, "stride": 1, "padding": "same"}))

    def cat(xs, nm=None) -> str:
        return g.add(Layer(nm or auto("concatenate"), "concat", list(xs)))

    x = g.add(Layer("input_1", "input", [], {"shape": tuple(input_shape)}))
    x = cbn(x, 32, 3, 3, "valid", 2)
    x = cbn(x, 32, 3, 3, "valid")
    x = cbn(x, 64, 3, 3)
    x = maxpool(x)
    x = cbn(x, 80, 1, 1, "valid")
    x = cbn(x, 192, 3, 3, "valid")
    x = maxpool(x)
    for i, pool_f in enumerate((32, 64, 64)):                     # mixed0-2: 35 x 35
        b1 = cbn(x, 64, 1, 1)
        b5 = cbn(cbn(x, 48, 1, 1), 64, 5, 5)
        b3 = cbn(cbn(cbn(x, 64, 1, 1), 96, 3, 3), 96, 3, 3)
        bp = cbn(avgpool(x), pool_f, 1, 1)
        x = cat([b1, b5, b3, bp], f"mixed{i}")
    b3 = cbn(x, 384, 3, 3, "valid", 2)                            # mixed3: 17 x 17
    bd = cbn(cbn(cbn(x, 64, 1, 1), 96, 3, 3), 96, 3, 3, "valid", 2)
    x = cat([b3, bd, maxpool(x)], "mixed3")
    for i, c7 in enumerate((128, 160, 160, 192)):                 # mixed4-7
        b1 = cbn(x, 192, 1, 1)
        b7 = cbn(cbn(cbn(x, c7, 1, 1), c7, 1, 7), 192, 7, 1)
        bd = cbn(x, c7, 1, 1)
        for f, (kh, kw) in ((c7, (7, 1)), (c7, (1, 7)), (c7, (7, 1)), (192, (1, 7))):
            bd = cbn(bd, f, kh, kw)
        bp = cbn(avgpool(x), 192, 1, 1)
        x = cat([b1, b7, bd, bp], f"mixed{4 + i}")
    b3 = cbn(cbn(x, 192, 1, 1), 320, 3, 3, "valid", 2)            # mixed8: 8 x 8
    b7 = cbn(cbn(cbn(cbn(x, 192, 1, 1), 192, 1, 7), 192, 7, 1), 192, 3, 3, "valid", 2)
    x = cat([b3, b7, maxpool(x)], "mixed8")
    for i in range(2):                                            # mixed9, mixed10
        b1 = cbn(x, 320, 1, 1)
        b3 = cbn(x, 384, 1, 1)
        b3 = cat([cbn(b3, 384, 1, 3), cbn(b3, 384, 3, 1)], f"mixed9_{i}")
        bd = cbn(cbn(x, 448, 1, 1), 384, 3, 3)
        bd = cat([cbn(bd, 384, 1, 3), cbn(bd, 384, 3, 1)])
        bp = cbn(avgpool(x), 192, 1, 1)
        x = cat([b1, b3, bd, bp], f"mixed{9 + i}")
    x = g.add(Layer("avg_pool", "gap", [x]))
    g.add(Layer("predictions", "dense", [x], {"units": classes, "activation": "softmax", "use_bias": True}))
    g.output_names = ["predictions"]
    return g


BUILDERS: Dict[str, Callable[..., Graph]] = {
    "vgg16": lambda **kw: build_vgg("vgg16", **kw),
    "vgg19": lambda **kw: build_vgg("vgg19", **kw),
    "mobilenet_v2": lambda **kw: build_mobilenet_v2(**kw),
    "densenet121": lambda **kw: build_densenet("densenet121", **kw),
    "densenet169": lambda **kw: build_densenet("densenet169", **kw),
    "densenet201": lambda **kw: build_densenet("densenet201", **kw),
    **{n: (lambda n: lambda **kw: build_efficientnet(n, **kw))(n) for n in EFFNET_SCALE},
    "inception_v3": lambda **kw: build_inception_v3(**kw),
}


def build_model(name: str, **kw) -> Graph:
    """Any supported family by name: resnet50/101/152 (+ test sizes) or a key of BUILDERS."""
    from .resnet import STACKS, build_resnet
    if name in STACKS:
        return build_resnet(name, **kw)
    if name not in BUILDERS:
        raise KeyError(f"unknown model {name!r}; known: {sorted(STACKS) + sorted(BUILDERS)}")
    return BUILDERS[name](**kw)
