"""Network IR for the gale model zoo, parameter packing and plan building.

The reference serves an opaque TF SavedModel (``model/saved_model.pb``, InferenceBolt.java:49-58)
whose only pinned contract is ``input:0`` (NHWC float) -> ``output/Softmax:0`` (float[N][10],
:82-86). gale instead describes each supported CNN as a small static layer list. From it we get:

* seeded random initialisation (``init_params``) with BatchNorm statistics calibrated on synthetic
  data, so random-init networks keep unit-scale activations like trained ones do;
* BatchNorm folding into conv weight/bias (``fold_params``);
* one flat packed parameter buffer (``pack_params``) whose layout (``param_layout``) depends only
  on the architecture, so rank 0 can fill it and RCCL-broadcast it to every other GPU;
* the executor plan (``build_plan``): a flat list of gfx950 kernels with buffer ids.
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple, Union

import torch

ALIGN = 256  # byte alignment of every packed parameter


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def stored_channels(c: int) -> int:
    """Channel stride of an activation tensor in memory (16-B vector loads need multiples of 8)."""
    return round_up(c, 8)


def conv_n_tiles(cout_stored: int) -> int:
    """Mirror of ``gale::conv_n_tiles`` (csrc/kernels/conv_mfma.hip): 16-channel tiles per n-block."""
    if cout_stored <= 16:
        return 1
    if cout_stored <= 32:
        return 2
    if cout_stored <= 64:
        return 4
    return 8


@dataclass
class Conv:
    name: str
    inp: str
    out: str
    cin: int
    cout: int
    k: int
    stride: int = 1
    pad: int = 0
    bn: bool = True
    bias: bool = False
    relu: bool = True
    residual: Optional[str] = None
    res_mode: str = "identity"  # "identity" | "pad" (ResNet option A: subsample + zero channels)
    out_f32: bool = False  # fp32 output (classifier logits)


@dataclass
class MaxPool:
    name: str
    inp: str
    out: str
    k: int
    s: int
    p: int = 0


@dataclass
class AvgPool:
    name: str
    inp: str
    out: str


@dataclass
class Head:
    """Global average pool (if spatial) + dense (fp32 weights) + softmax -> network output."""

    name: str
    inp: str
    classes: int


@dataclass
class Softmax:
    name: str
    inp: str
    classes: int


Layer = Union[Conv, MaxPool, AvgPool, Head, Softmax]


@dataclass
class Network:
    name: str
    input_shape: Tuple[int, int, int]  # H, W, C of one image (InstObj.instances[i])
    classes: int
    layers: List[Layer]
    dataset: str = ""
    shapes: Dict[str, Tuple[int, int, int]] = field(default_factory=dict)

    def __post_init__(self):
        self.shapes = infer_shapes(self)

    @property
    def per_image(self) -> int:
        h, w, c = self.input_shape
        return h * w * c

    def macs_per_image(self) -> int:
        total = 0
        for L in self.layers:
            if isinstance(L, Conv):
                ho, wo, _ = self.shapes[L.out]
                total += ho * wo * L.cout * L.cin * L.k * L.k
            elif isinstance(L, Head):
                _, _, c = self.shapes[L.inp]
                total += c * L.classes
        return total


def infer_shapes(net: Network) -> Dict[str, Tuple[int, int, int]]:
    shapes = {"input": tuple(net.input_shape)}
    for L in net.layers:
        h, w, c = shapes[L.inp]
        if isinstance(L, Conv):
            if c != L.cin:
                raise ValueError(f"{L.name}: input has {c} channels, layer expects {L.cin}")
            ho = (h + 2 * L.pad - L.k) // L.stride + 1
            wo = (w + 2 * L.pad - L.k) // L.stride + 1
            shapes[L.out] = (ho, wo, L.cout)
            if L.residual is not None:
                rh, rw, rc = shapes[L.residual]
                if L.res_mode == "identity" and (rh, rw, rc) != (ho, wo, L.cout):
                    raise ValueError(f"{L.name}: identity residual shape mismatch")
                if L.res_mode == "pad" and (rh != ho * 2 or rw != wo * 2 or rc > L.cout):
                    raise ValueError(f"{L.name}: option-A residual shape mismatch")
        elif isinstance(L, MaxPool):
            ho = (h + 2 * L.p - L.k) // L.s + 1
            wo = (w + 2 * L.p - L.k) // L.s + 1
            shapes[L.out] = (ho, wo, c)
        elif isinstance(L, AvgPool):
            shapes[L.out] = (1, 1, c)
        elif isinstance(L, (Head, Softmax)):
            shapes["output"] = (1, 1, L.classes)
    return shapes


# --------------------------------------------------------------------------------------------
# parameters
# --------------------------------------------------------------------------------------------

BN_EPS = 1e-5


def init_params(net: Network, seed: int = 0, calibrate: bool = True,
                calib_batch: int = 8) -> Dict[str, torch.Tensor]:
    """Seeded random init (Kaiming convs, U(0,1)-input BN calibration). fp32 CPU tensors."""
    g = torch.Generator().manual_seed(seed)
    p: Dict[str, torch.Tensor] = {}
    for L in net.layers:
        if isinstance(L, Conv):
            fan_in = L.cin * L.k * L.k
            std = math.sqrt(2.0 / fan_in)
            p[f"{L.name}.weight"] = torch.randn(L.cout, L.cin, L.k, L.k, generator=g) * std
            if L.bias or not L.bn:
                p[f"{L.name}.bias"] = (torch.rand(L.cout, generator=g) - 0.5) * 0.1
            if L.bn:
                p[f"{L.name}.bn.gamma"] = 0.5 + torch.rand(L.cout, generator=g) * 0.5
                p[f"{L.name}.bn.beta"] = (torch.rand(L.cout, generator=g) - 0.5) * 0.2
                p[f"{L.name}.bn.mean"] = torch.zeros(L.cout)
                p[f"{L.name}.bn.var"] = torch.ones(L.cout)
        elif isinstance(L, Head):
            _, _, c = net.shapes[L.inp]
            p[f"{L.name}.weight"] = torch.randn(L.classes, c, generator=g) * math.sqrt(1.0 / c) * 2.0
            p[f"{L.name}.bias"] = (torch.rand(L.classes, generator=g) - 0.5) * 0.1
    if calibrate and any(isinstance(L, Conv) and L.bn for L in net.layers):
        from gale.models.reference import calibrate_bn

        x = torch.rand((calib_batch,) + tuple(net.input_shape), generator=g)
        calibrate_bn(net, p, x)
    return p


def fold_params(net: Network, p: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Fold inference BatchNorm into the preceding conv: w' = w*s, b' = beta + (b - mean)*s."""
    f: Dict[str, torch.Tensor] = {}
    for L in net.layers:
        if isinstance(L, Conv):
            w = p[f"{L.name}.weight"].float()
            b = p.get(f"{L.name}.bias", torch.zeros(L.cout)).float()
            if L.bn:
                s = p[f"{L.name}.bn.gamma"] / torch.sqrt(p[f"{L.name}.bn.var"] + BN_EPS)
                w = w * s.view(-1, 1, 1, 1)
                b = p[f"{L.name}.bn.beta"] + (b - p[f"{L.name}.bn.mean"]) * s
            f[f"{L.name}.weight"] = w.contiguous()
            f[f"{L.name}.bias"] = b.contiguous()
        elif isinstance(L, Head):
            f[f"{L.name}.weight"] = p[f"{L.name}.weight"].float().contiguous()
            f[f"{L.name}.bias"] = p[f"{L.name}.bias"].float().contiguous()
    return f


def unfolded_params(net: Network, p: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Parameters for the unfolded-BN plan (``fold_bn=False``): raw conv weight/bias and each
    BatchNorm as a per-channel affine (scale = gamma/sqrt(var+eps), shift = beta - mean*scale)
    applied by the standalone ``bn_act`` kernel after the conv (TF's Conv2D -> FusedBatchNorm)."""
    f: Dict[str, torch.Tensor] = {}
    for L in net.layers:
        if isinstance(L, Conv):
            f[f"{L.name}.weight"] = p[f"{L.name}.weight"].float().contiguous()
            f[f"{L.name}.bias"] = p.get(f"{L.name}.bias", torch.zeros(L.cout)).float().contiguous()
            if L.bn:
                s = p[f"{L.name}.bn.gamma"] / torch.sqrt(p[f"{L.name}.bn.var"] + BN_EPS)
                f[f"{L.name}.bn_scale"] = s.float().contiguous()
                f[f"{L.name}.bn_shift"] = (p[f"{L.name}.bn.beta"]
                                           - p[f"{L.name}.bn.mean"] * s).float().contiguous()
        elif isinstance(L, Head):
            f[f"{L.name}.weight"] = p[f"{L.name}.weight"].float().contiguous()
            f[f"{L.name}.bias"] = p[f"{L.name}.bias"].float().contiguous()
    return f


# --------------------------------------------------------------------------------------------
# packing: one flat byte buffer, architecture-determined layout
# --------------------------------------------------------------------------------------------


@dataclass
class PackedEntry:
    offset: int
    nbytes: int
    dtype: torch.dtype
    shape: Tuple[int, ...]


def stem_packed(net: Network, L: Conv, wdtype: str = "bf16") -> bool:
    """A 7x7/2 (pad 3) conv on the <= 4-channel network input runs as a packed-stem GEMM
    (ConvDesc::stem, csrc/kernels/conv_gemm.hip): the input is repacked to bf16 [H][2*Wo+6][4]
    so every kernel row of an output pixel is one 64-byte run."""
    return (wdtype == "bf16" and L.inp == "input" and L.k == 7 and L.stride == 2 and L.pad == 3
            and L.cin <= 4 and stored_channels(L.cout) % 64 == 0 and not L.out_f32
            and L.residual is None)


def _conv_geometry(net: Network, L: Conv, wdtype: str = "bf16") -> Dict[str, int]:
    h, w, _ = net.shapes[L.inp]
    ho, wo, _ = net.shapes[L.out]
    if stem_packed(net, L, wdtype):
        cout_s = stored_channels(L.cout)
        return dict(H=h, W=2 * wo + 6, Cin=4, Ho=ho, Wo=wo, Cout=cout_s, KH=8, KW=8, stride=2,
                    pad=3, K=256, Kpad=256, Npad=round_up(cout_s, conv_n_tiles(cout_s) * 16),
                    stem=1)
    cin_s = L.cin if L.inp == "input" else stored_channels(L.cin)
    cout_s = stored_channels(L.cout)
    K = L.k * L.k * cin_s
    Kpad = round_up(K, 32)
    nt = conv_n_tiles(cout_s)
    Npad = round_up(cout_s, nt * 16)
    if wdtype == "fp32":  # conv_f32.hip: K chunks of 16, 64-channel tiles (rows >= Npad read 0)
        Kpad, Npad = round_up(K, 16), cout_s
    return dict(H=h, W=w, Cin=cin_s, Ho=ho, Wo=wo, Cout=cout_s, KH=L.k, KW=L.k, stride=L.stride,
                pad=L.pad, K=K, Kpad=Kpad, Npad=Npad)


def param_layout(net: Network, wdtype: str = "bf16",
                 fold_bn: bool = True) -> Tuple[Dict[str, PackedEntry], int]:
    """Byte layout of the packed parameter buffer (depends only on the architecture).
    ``fold_bn=False`` (bf16 / fp32) adds a BN scale and shift vector per BatchNorm conv."""
    if not fold_bn and wdtype == "fp8":
        raise ValueError("the unfolded-BN plan is bf16 / fp32 only")
    wbytes = {"bf16": 2, "fp8": 1, "fp32": 4}[wdtype]
    layout: Dict[str, PackedEntry] = {}
    off = 0

    def add(name, nbytes, dtype, shape):
        nonlocal off
        layout[name] = PackedEntry(off, nbytes, dtype, tuple(shape))
        off = round_up(off + nbytes, ALIGN)

    for L in net.layers:
        if isinstance(L, Conv):
            gm = _conv_geometry(net, L, wdtype)
            wdt = {"bf16": torch.bfloat16, "fp8": torch.uint8, "fp32": torch.float32}[wdtype]
            add(f"{L.name}.w", gm["Npad"] * gm["Kpad"] * wbytes, wdt, (gm["Npad"], gm["Kpad"]))
            add(f"{L.name}.b", gm["Npad"] * 4, torch.float32, (gm["Npad"],))
            if wdtype == "fp8":
                add(f"{L.name}.s", gm["Npad"] * 4, torch.float32, (gm["Npad"],))
            if not fold_bn and L.bn:
                add(f"{L.name}.bn_s", gm["Npad"] * 4, torch.float32, (gm["Npad"],))
                add(f"{L.name}.bn_t", gm["Npad"] * 4, torch.float32, (gm["Npad"],))
        elif isinstance(L, Head):
            _, _, c = net.shapes[L.inp]
            cs = stored_channels(c)
            add(f"{L.name}.w", L.classes * cs * 4, torch.float32, (L.classes, cs))
            add(f"{L.name}.b", L.classes * 4, torch.float32, (L.classes,))
    if wdtype == "fp8":
        # per-tensor activation scales travel with the weights (one RCCL broadcast)
        from gale.models.quant import activation_tensors

        n = len(activation_tensors(net))
        add("act_scales", n * 4, torch.float32, (n,))
    return layout, round_up(off, ALIGN)


def pack_conv_weight(w: torch.Tensor, cin_s: int, Npad: int, Kpad: int) -> torch.Tensor:
    """[cout, cin, kh, kw] fp32 -> [Npad, Kpad] with k = (kh*KW + kw)*cin_s + ci (zero padded)."""
    cout, cin, kh, kw = w.shape
    wp = torch.zeros(cout, kh, kw, cin_s, dtype=torch.float32)
    wp[..., :cin] = w.permute(0, 2, 3, 1)
    flat = torch.zeros(Npad, Kpad, dtype=torch.float32)
    flat[:cout, : kh * kw * cin_s] = wp.reshape(cout, -1)
    return flat


def pack_params(net: Network, folded: Dict[str, torch.Tensor], wdtype: str = "bf16",
                fold_bn: bool = True) -> torch.Tensor:
    """Fill the flat packed buffer (uint8 CPU tensor) from folded fp32 parameters
    (``fold_params``), or with ``fold_bn=False`` from ``unfolded_params``."""
    layout, total = param_layout(net, wdtype, fold_bn)
    buf = torch.zeros(total, dtype=torch.uint8)

    def put(name: str, t: torch.Tensor):
        e = layout[name]
        raw = t.contiguous().view(torch.uint8).reshape(-1)
        assert raw.numel() == e.nbytes, (name, raw.numel(), e.nbytes)
        buf[e.offset : e.offset + e.nbytes] = raw

    for L in net.layers:
        if isinstance(L, Conv):
            gm = _conv_geometry(net, L, wdtype)
            wt = folded[f"{L.name}.weight"]
            if gm.get("stem"):  # zero-pad the 7x7 kernel to 8x8: k = kh*32 + kw*4 + c
                w8 = torch.zeros(wt.shape[0], wt.shape[1], 8, 8, dtype=wt.dtype)
                w8[:, :, :L.k, :L.k] = wt
                wt = w8
            w = pack_conv_weight(wt, gm["Cin"], gm["Npad"], gm["Kpad"])
            b = torch.zeros(gm["Npad"])
            b[: L.cout] = folded[f"{L.name}.bias"]
            if wdtype == "bf16":
                put(f"{L.name}.w", w.to(torch.bfloat16))
            elif wdtype == "fp32":
                put(f"{L.name}.w", w)
            else:
                from gale.models.quant import quantize_rows_e4m3

                q, s = quantize_rows_e4m3(w)
                put(f"{L.name}.w", q)
                put(f"{L.name}.s", s)
            put(f"{L.name}.b", b)
            if not fold_bn and L.bn:
                for key, src in (("bn_s", "bn_scale"), ("bn_t", "bn_shift")):
                    v = torch.zeros(gm["Npad"])
                    v[: L.cout] = folded[f"{L.name}.{src}"]
                    put(f"{L.name}.{key}", v)
        elif isinstance(L, Head):
            _, _, c = net.shapes[L.inp]
            cs = stored_channels(c)
            w = torch.zeros(L.classes, cs)
            w[:, :c] = folded[f"{L.name}.weight"]
            put(f"{L.name}.w", w)
            put(f"{L.name}.b", folded[f"{L.name}.bias"])
    if wdtype == "fp8":
        from gale.models.quant import activation_tensors, calibrate_act_scales

        sc = calibrate_act_scales(net, folded)
        put("act_scales", torch.tensor([sc[n] for n in activation_tensors(net)],
                                       dtype=torch.float32))
    return buf


def act_scales_from_packed(net: Network, packed: torch.Tensor) -> Dict[str, float]:
    """Read the fp8 activation scales back out of a packed buffer (any device)."""
    from gale.models.quant import activation_tensors

    layout, _ = param_layout(net, "fp8")
    e = layout["act_scales"]
    raw = packed[e.offset: e.offset + e.nbytes].cpu().contiguous()
    vals = raw.view(torch.float32).tolist()
    return dict(zip(activation_tensors(net), vals))


# --------------------------------------------------------------------------------------------
# executor plan
# --------------------------------------------------------------------------------------------

(OP_CONV, OP_MAXPOOL, OP_AVGPOOL, OP_HEAD, OP_SOFTMAX, OP_RESNET20, OP_STEM_PACK, OP_BN_ACT,
 OP_LENET5, OP_BOTTLENECK, OP_STEM_POOL, OP_CONV_PROJ) = range(12)


def is_cifar_resnet20(net: Network) -> bool:
    """True for the exact architecture the fused whole-network kernel implements."""
    from gale.models.zoo import resnet20

    ref = resnet20()
    return (net.input_shape == ref.input_shape and net.classes == ref.classes
            and [repr(L) for L in net.layers] == [repr(L) for L in ref.layers])


def is_mnist_lenet5(net: Network) -> bool:
    """True for the exact architecture the fused LeNet-5 kernel implements."""
    from gale.models.zoo import lenet5

    ref = lenet5()
    return (net.input_shape == ref.input_shape and net.classes == ref.classes
            and [repr(L) for L in net.layers] == [repr(L) for L in ref.layers])


def _fused_lenet5_plan(net: Network, base_ptr: int) -> Tuple[List[dict], List[int]]:
    layout, _ = param_layout(net, "bf16")
    names = ("conv1", "conv2", "fc1", "fc2", "fc3")
    ptrs = []
    for nm in names:
        ptrs += [base_ptr + layout[f"{nm}.w"].offset, base_ptr + layout[f"{nm}.b"].offset]
    op = dict(kind=OP_LENET5, **{"in": 0}, out=1, ptrs=ptrs)
    return [op], [_tensor_bytes(net, "input"), net.classes * 4]


def _fused_resnet20_plan(net: Network, base_ptr: int, wdtype: str = "bf16",
                         act_scales: Optional[Dict[str, float]] = None
                         ) -> Tuple[List[dict], List[int]]:
    layout, _ = param_layout(net, wdtype)
    convs = [L for L in net.layers if isinstance(L, Conv)]
    ptrs = [base_ptr + layout[f"{L.name}.w"].offset for L in convs]
    ptrs += [base_ptr + layout[f"{L.name}.b"].offset for L in convs]
    ptrs += [base_ptr + layout["fc.w"].offset, base_ptr + layout["fc.b"].offset]
    op = dict(kind=OP_RESNET20, **{"in": 0}, out=1, ptrs=ptrs)
    if wdtype == "fp8":
        op["fp8"] = 1
        op["ptrs"] = ptrs + [base_ptr + layout[f"{L.name}.s"].offset for L in convs]
        op["scales"] = ([act_scales[L.inp] for L in convs] + [act_scales[L.out] for L in convs]
                        + [act_scales[L.residual] if L.residual else 1.0 for L in convs])
    return [op], [_tensor_bytes(net, "input"), net.classes * 4]


def _tensor_bytes(net: Network, name: str, wdtype: str = "bf16") -> int:
    h, w, c = net.shapes[name]
    if name == "input":
        return h * w * c * 4
    return h * w * stored_channels(c) * {"fp8": 1, "bf16": 2, "fp32": 4}[wdtype]


def _is_conv(op: dict, kh: int, cin: int, cout: int, relu: int, res: bool, hw: int = 56) -> bool:
    if op["kind"] != OP_CONV:
        return False
    d = op["conv"]
    return (d["KH"] == kh and d["KW"] == kh and d["stride"] == 1 and d["H"] == hw
            and d["W"] == hw and d["Cin"] == cin and d["Cout"] == cout and d["Npad"] == cout
            and d["relu"] == relu and bool(d.get("has_res", 0)) == res
            and not d.get("stem") and not d.get("fp8") and not d.get("f32")
            and not d.get("in_f32") and not d.get("out_f32")
            and (kh == 1 or d["pad"] == 1))


def fuse_stem_pool(ops: List[dict]) -> List[dict]:
    """The ResNet-50 packed stem conv followed by its 3x3/2 max-pool becomes ONE
    ``OP_STEM_POOL`` (csrc/kernels/stem_pool.hip: the 112x112x64 stem output stays in LDS), when
    nothing else reads the stem output."""
    out: List[dict] = []
    i = 0
    while i < len(ops):
        c = ops[i]
        if (i + 1 < len(ops) and c["kind"] == OP_CONV and c["conv"].get("stem")
                and ops[i + 1]["kind"] == OP_MAXPOOL and ops[i + 1]["in"] == c["out"]):
            m, d = ops[i + 1], c["conv"]
            H, W, C, k, s_, p, Ho, Wo = m["p"]
            if (d["H"] == 224 and d["W"] == 230 and d["Ho"] == 112 and d["Wo"] == 112
                    and d["Cout"] == 64 and d["Npad"] == 64 and d["K"] == 256 and d["relu"]
                    and not d.get("has_res") and not d.get("fp8") and not d.get("f32")
                    and (H, W, C, k, s_, p, Ho, Wo) == (112, 112, 64, 3, 2, 1, 56, 56)
                    and m.get("et", 0) == 0):
                live = False
                for o in ops[i + 2:]:  # the stem output's buffer, read before it is rewritten?
                    if o.get("in") == c["out"] or o.get("res", -1) == c["out"]:
                        live = True
                        break
                    if o.get("out") == c["out"]:
                        break
                if not live:
                    out.append(dict(kind=OP_STEM_POOL, conv=d, **{"in": c["in"]}, out=m["out"],
                                    res=-1, w=c["w"], bias=c["bias"], p=list(m["p"]),
                                    bpi=[c["bpi"][0], m["bpi"][1], 0], layer=m.get("layer", 0)))
                    i += 2
                    continue
        out.append(c)
        i += 1
    return out


def fuse_bottlenecks(ops: List[dict]) -> List[dict]:
    """Replace every ResNet-50 56x56 bottleneck of a bf16 plan - conv1 / conv2 / conv3 (+ the
    block-0 projection before them) - by ONE ``OP_BOTTLENECK`` (csrc/kernels/bottleneck_fused.hip:
    the 64-channel intermediates stay in LDS). A chain is fused only when its intermediate
    tensors are read by nothing after it."""
    def live_after(k: int, buf: int) -> bool:
        # buffers are reused by liveness: the tensor in `buf` is live at op k when an op from k
        # on reads `buf` before one overwrites it
        for o in ops[k:]:
            if o.get("in") == buf or o.get("res", -1) == buf:
                return True
            if o.get("out") == buf:
                return False
        return False

    out: List[dict] = []
    i = 0
    while i < len(ops):
        down = None
        j = i
        if (i + 3 < len(ops) and _is_conv(ops[i], 1, 64, 256, 0, False)
                and _is_conv(ops[i + 1], 1, 64, 64, 1, False) and ops[i + 1]["in"] == ops[i]["in"]):
            down, j = ops[i], i + 1
        if (j + 2 < len(ops) and (down is not None or _is_conv(ops[j], 1, 256, 64, 1, False))
                and _is_conv(ops[j + 1], 3, 64, 64, 1, False)
                and _is_conv(ops[j + 2], 1, 64, 256, 1, True)
                and ops[j + 1]["in"] == ops[j]["out"] and ops[j + 2]["in"] == ops[j + 1]["out"]
                and ops[j + 2]["conv"].get("res_stride", 1) == 1
                and ops[j + 2]["res"] == (down["out"] if down is not None else ops[j]["in"])
                and ops[j + 2]["out"] != ops[j]["in"]
                and not live_after(j + 2, ops[j]["out"]) and not live_after(j + 3, ops[j + 1]["out"])
                and (down is None or not live_after(j + 3, down["out"]))):
            c1, c2, c3 = ops[j], ops[j + 1], ops[j + 2]
            ptrs = [c1["w"], c1["bias"], c2["w"], c2["bias"], c3["w"], c3["bias"]]
            if down is not None:
                ptrs += [down["w"], down["bias"]]
            out.append(dict(kind=OP_BOTTLENECK, **{"in": c1["in"]}, out=c3["out"], res=-1,
                            p=[c1["conv"]["Cin"], int(down is not None)], ptrs=ptrs,
                            bpi=[c1["bpi"][0], c3["bpi"][1], 0], layer=c3.get("layer", 0)))
            i = j + 3
            continue
        out.append(ops[i])
        i += 1
    return out


def projection_pairs(net: Network) -> Dict[str, str]:
    """Bottleneck conv3 layers whose residual is a strided 1x1 projection read by nothing else:
    {conv3 name: projection name}. Each pair can run as one GEMM over the concatenated
    reduction (``fuse_projections``); stride-1 projections stay with the 56x56 block kernel."""
    by_out = {L.out: L for L in net.layers if isinstance(L, Conv)}
    readers: Dict[str, int] = {}
    for L in net.layers:
        readers[L.inp] = readers.get(L.inp, 0) + 1
        if isinstance(L, Conv) and L.residual is not None:
            readers[L.residual] = readers.get(L.residual, 0) + 1
    pairs = {}
    for L in net.layers:
        if not (isinstance(L, Conv) and L.residual is not None and L.res_mode == "identity"
                and L.k == 1 and L.stride == 1 and L.pad == 0 and not L.out_f32):
            continue
        D = by_out.get(L.residual)
        if (D is not None and D.k == 1 and D.stride > 1 and D.pad == 0 and not D.relu
                and D.residual is None and not D.out_f32 and D.cout == L.cout
                and readers.get(D.out, 0) == 1 and D.cin % 64 == 0 and L.cin % 64 == 0
                and L.cout % 128 == 0):  # (conv2d_gemm_proj's 128-channel tiles)
            pairs[L.name] = D.name
    return pairs


def fuse_projections(ops: List[dict], pairs: Dict[int, int]) -> List[dict]:
    """Each (projection, conv3) op pair of ``pairs`` ({index of conv3: index of the projection},
    op indices) becomes ONE ``OP_CONV_PROJ`` at conv3's place (csrc/kernels/conv_gemm.hip
    conv2d_gemm_proj: the projection's output tensor never exists). build_plan keeps the block
    input alive up to conv3 for these."""
    drop = set(pairs.values())
    out: List[dict] = []
    for i, op in enumerate(ops):
        if i in drop:
            continue
        if i in pairs:
            dn = ops[pairs[i]]
            dd, cd = dn["conv"], dict(op["conv"])
            for k in ("has_res", "res_H", "res_W", "res_C", "res_stride"):
                cd.pop(k, None)
            out.append(dict(kind=OP_CONV_PROJ, conv=cd, **{"in": op["in"]}, out=op["out"],
                            res=dn["in"], ptrs=[op["w"], op["bias"], dn["w"], dn["bias"]],
                            p=[dd["H"], dd["W"], dd["Cin"], dd["stride"], dd["Kpad"]],
                            bpi=[op["bpi"][0], op["bpi"][1], dn["bpi"][0]],
                            layer=op.get("layer", 0)))
            continue
        out.append(op)
    return out


def build_plan(net: Network, base_ptr: int, wdtype: str = "bf16",
               act_scales: Optional[Dict[str, float]] = None,
               fused: bool = True, fold_bn: bool = True,
               chunk_layers: int = 0,
               fuse_blocks: Optional[bool] = None) -> Tuple[List[dict], List[int]]:
    """Executor plan for a packed parameter buffer living at device address ``base_ptr``.

    Returns (ops, buf_bytes_per_image). Buffer 0 = fp32 input, 1 = fp32 softmax output, >= 2 =
    bf16 (fp8: e4m3) activations assigned by liveness so concurrently-live tensors never share a
    buffer. ``act_scales`` (fp8 only): per-tensor scales, see ``act_scales_from_packed``.
    ``fused``: the CIFAR ResNet-20 (bf16 or fp8) and the MNIST LeNet-5 (bf16 weights, fp32
    math) become ONE whole-network kernel each (activations resident in LDS). ``fold_bn=False`` (bf16, layer-wise; the buffer from ``pack_params(...,
    fold_bn=False)``): every BatchNorm conv is followed by a standalone ``bn_act`` kernel that
    applies the BN affine, the residual and the ReLU in place (the debugging / parity plan).
    ``fuse_blocks`` (bf16, folded BN, no chunking; default on, ``GALE_FUSE_BLOCKS=0`` off): the
    ResNet-50 stem + max-pool (``fuse_stem_pool``) and each 56x56 bottleneck
    (``fuse_bottlenecks``) run as one kernel, and each strided projection shortcut runs inside
    its block's conv3 (``fuse_projections``).
    ``chunk_layers``: the first ``chunk_layers`` layers may run per batch chunk (the executor's
    PlanSpec::chunk_ops; every op carries ``layer``, its layer index): each tensor they produce
    that is still read after them gets a buffer of its own, so a later chunk cannot overwrite an
    earlier chunk's live-out rows.
    """
    fp8 = wdtype == "fp8"
    f32 = wdtype == "fp32"  # reference-precision plan: fp32 everything, fp32 MFMA convs
    et = 2 if f32 else int(fp8)  # pool / head activation element type (kernels.h ElemType)
    if fp8 and act_scales is None:
        raise ValueError("build_plan: the fp8 plan needs the activation scales")
    if fused and fold_bn and is_cifar_resnet20(net) and not f32:
        return _fused_resnet20_plan(net, base_ptr, wdtype, act_scales)
    if fused and is_mnist_lenet5(net) and wdtype == "bf16":
        return _fused_lenet5_plan(net, base_ptr)
    layout, _ = param_layout(net, wdtype, fold_bn)
    if fuse_blocks is None:
        fuse_blocks = os.environ.get("GALE_FUSE_BLOCKS", "1") != "0"
    fuse_blocks = bool(fuse_blocks and fused and wdtype == "bf16" and fold_bn and chunk_layers == 0)
    # (GALE_FUSE_PROJ=0: the projections stay separate convs, for A/B runs)
    proj = projection_pairs(net) if fuse_blocks and os.environ.get("GALE_FUSE_PROJ", "1") != "0" \
        else {}
    layer_index = {L.name: i for i, L in enumerate(net.layers)}
    # liveness: last layer index reading each tensor
    last_use: Dict[str, int] = {}
    for i, L in enumerate(net.layers):
        last_use[L.inp] = i
        if isinstance(L, Conv) and L.residual is not None:
            last_use[L.residual] = i
    for c3, dn in proj.items():
        # a fused projection reads the block input at conv3's place: keep it alive until then
        x = net.layers[layer_index[dn]].inp
        last_use[x] = max(last_use[x], layer_index[c3])
    conv_op: Dict[str, int] = {}  # conv layer name -> index of its OP_CONV in ops
    buf_of: Dict[str, int] = {"input": 0}
    buf_bytes: List[int] = [_tensor_bytes(net, "input"), net.classes * 4]
    # bytes per image of a tensor as stored (every op also carries bpi = [in, out, res] for the
    # executor's batch chunking, PlanSpec::chunk_ops)
    tbytes: Dict[str, int] = {"input": _tensor_bytes(net, "input"), "output": net.classes * 4}
    free: List[int] = []
    ops: List[dict] = []
    # fp32 logits tensors (Conv.out_f32) get their own dedicated buffers
    for i, L in enumerate(net.layers):
        out_name = getattr(L, "out", "output")
        if isinstance(L, (Head, Softmax)):
            buf_of["output"] = 1
        else:
            need = _tensor_bytes(net, out_name, wdtype)
            if isinstance(L, Conv) and L.out_f32:
                h, w, c = net.shapes[out_name]
                need = h * w * stored_channels(c) * 4
            bid = None
            live_out = i < chunk_layers and last_use.get(out_name, len(net.layers)) >= chunk_layers
            for j, b in enumerate(free):
                if live_out:
                    break  # (a fresh buffer: no other prefix tensor ever used it)
                bid = b
                free.pop(j)
                break
            if bid is None:
                bid = len(buf_bytes)
                buf_bytes.append(0)
            buf_bytes[bid] = max(buf_bytes[bid], need)
            buf_of[out_name] = bid
            tbytes[out_name] = need
        if isinstance(L, Conv):
            gm = _conv_geometry(net, L, wdtype)
            d = dict(gm)
            d["relu"] = int(L.relu)
            d["in_f32"] = int(L.inp == "input")
            src = buf_of[L.inp]
            if gm.get("stem"):
                # fp32 input -> packed-stem bf16 image in a buffer of its own
                h, w, c = net.shapes[L.inp]
                src = len(buf_bytes)
                buf_bytes.append(h * gm["W"] * 4 * 2)
                ops.append(dict(kind=OP_STEM_PACK, p=[h, w, c, gm["W"], 3], **{"in": 0},
                                out=src, bpi=[tbytes["input"], buf_bytes[src], 0]))
                d["in_f32"] = 0
            d["out_f32"] = int(L.out_f32)
            d["fp8"] = int(fp8)
            d["f32"] = int(f32)
            if fp8:
                d["in_scale"] = act_scales[L.inp]
                d["out_scale"] = 1.0 if L.out_f32 else act_scales[L.out]
            res = -1
            unfold = not fold_bn and L.bn
            if unfold:
                d["relu"] = 0  # BN, residual and ReLU move to the bn_act op below
            if L.residual is not None and not unfold:
                rh, rw, rc = net.shapes[L.residual]
                d.update(has_res=1, res_H=rh, res_W=rw, res_C=stored_channels(rc),
                         res_stride=2 if L.res_mode == "pad" else 1)
                if fp8:
                    d["res_scale"] = act_scales[L.residual]
                res = buf_of[L.residual]
            in_bpi = buf_bytes[src] if gm.get("stem") else tbytes[L.inp]
            op = dict(kind=OP_CONV, conv=d, **{"in": src}, out=buf_of[out_name], res=res,
                      w=base_ptr + layout[f"{L.name}.w"].offset,
                      bias=base_ptr + layout[f"{L.name}.b"].offset,
                      bpi=[in_bpi, tbytes[out_name], tbytes[L.residual] if res >= 0 else 0])
            if wdtype == "fp8":
                op["wscale"] = base_ptr + layout[f"{L.name}.s"].offset
            conv_op[L.name] = len(ops)
            ops.append(op)
            if unfold:
                ho, wo, c = net.shapes[L.out]
                bn = dict(kind=OP_BN_ACT, **{"in": buf_of[out_name]}, out=buf_of[out_name], res=-1,
                          w=base_ptr + layout[f"{L.name}.bn_s"].offset,
                          bias=base_ptr + layout[f"{L.name}.bn_t"].offset,
                          et=2 if f32 else 0, bpi=[tbytes[out_name], tbytes[out_name], 0])
                p = [ho * wo, wo, stored_channels(c), int(L.relu), 0, 0, 0, 1]
                if L.residual is not None:
                    rh, rw, rc = net.shapes[L.residual]
                    p[4:] = [rh, rw, stored_channels(rc), 2 if L.res_mode == "pad" else 1]
                    bn["res"] = buf_of[L.residual]
                    bn["bpi"][2] = tbytes[L.residual]
                bn["p"] = p
                ops.append(bn)
        elif isinstance(L, MaxPool):
            h, w, c = net.shapes[L.inp]
            ho, wo, _ = net.shapes[L.out]
            ops.append(dict(kind=OP_MAXPOOL, p=[h, w, stored_channels(c), L.k, L.s, L.p, ho, wo],
                            **{"in": buf_of[L.inp]}, out=buf_of[L.out], et=et,
                            bpi=[tbytes[L.inp], tbytes[L.out], 0]))
        elif isinstance(L, AvgPool):
            h, w, c = net.shapes[L.inp]
            ops.append(dict(kind=OP_AVGPOOL, p=[h * w, stored_channels(c)],
                            **{"in": buf_of[L.inp]}, out=buf_of[L.out], et=et,
                            bpi=[tbytes[L.inp], tbytes[L.out], 0]))
        elif isinstance(L, Head):
            h, w, c = net.shapes[L.inp]
            ops.append(dict(kind=OP_HEAD, p=[h * w, stored_channels(c), L.classes],
                            **{"in": buf_of[L.inp]}, out=1,
                            w=base_ptr + layout[f"{L.name}.w"].offset,
                            bias=base_ptr + layout[f"{L.name}.b"].offset,
                            et=et, scale=act_scales[L.inp] if fp8 else 1.0,
                            bpi=[tbytes[L.inp], tbytes["output"], 0]))
        elif isinstance(L, Softmax):
            h, w, c = net.shapes[L.inp]
            ops.append(dict(kind=OP_SOFTMAX, p=[L.classes, stored_channels(c)],
                            **{"in": buf_of[L.inp]}, out=1,
                            bpi=[tbytes[L.inp], tbytes["output"], 0]))
        for op in ops:
            op.setdefault("layer", i)
        # release buffers whose tensors die here
        for t, lu in list(last_use.items()):
            if lu == i and t in buf_of and buf_of[t] >= 2:
                free.append(buf_of[t])
                del last_use[t]
    if fuse_blocks:
        ops = fuse_projections(ops, {conv_op[c3]: conv_op[dn] for c3, dn in proj.items()})
        ops = fuse_bottlenecks(fuse_stem_pool(ops))
    return ops, buf_bytes
