"""The CNN classifiers gale serves (BASELINE.json configs; README.md:16 of the reference names
MNIST and CIFAR-10 classifiers, SURVEY.md §2.5 the op set).

* ``lenet5``   — MNIST 28x28x1, conv5x5(6,pad2)-pool-conv5x5(16)-pool-fc120-fc84-fc10.
* ``resnet20`` — CIFAR-10 32x32x3, He et al. 2016 CIFAR ResNet (3 stages x 3 basic blocks,
  16/32/64 channels, parameter-free option-A shortcuts, 0.27 M params, ~40.6 M MAC/img).
* ``resnet50`` — ImageNet 224x224x3, bottleneck [3,4,6,3], projection shortcuts, 25.6 M params.

Dense layers are expressed as convolutions (a dense layer over a flattened HxWxC tensor is a
HxW "valid" convolution producing a 1x1 map), so every GEMM runs on the same MFMA conv kernel.
"""

from __future__ import annotations

from typing import Callable, Dict, List

from gale.models.graph import AvgPool, Conv, Head, Layer, MaxPool, Network, Softmax


def lenet5() -> Network:
    L: List[Layer] = [
        Conv("conv1", "input", "c1", 1, 6, 5, pad=2, bn=False, bias=True),
        MaxPool("pool1", "c1", "p1", 2, 2),
        Conv("conv2", "p1", "c2", 6, 16, 5, bn=False, bias=True),
        MaxPool("pool2", "c2", "p2", 2, 2),
        Conv("fc1", "p2", "f1", 16, 120, 5, bn=False, bias=True),  # 5x5x16=400 -> 120
        Conv("fc2", "f1", "f2", 120, 84, 1, bn=False, bias=True),
        Head("fc3", "f2", 10),
    ]
    return Network("lenet5", (28, 28, 1), 10, L, dataset="mnist")


def resnet20() -> Network:
    L: List[Layer] = [Conv("stem", "input", "s0", 3, 16, 3, pad=1)]
    cur, cin = "s0", 16
    for stage, cout in enumerate((16, 32, 64)):
        for blk in range(3):
            stride = 2 if (stage > 0 and blk == 0) else 1
            n = f"l{stage + 1}.{blk}"
            L.append(Conv(f"{n}.conv1", cur, f"{n}.a", cin, cout, 3, stride=stride, pad=1))
            mode = "pad" if stride == 2 else "identity"
            L.append(Conv(f"{n}.conv2", f"{n}.a", f"{n}.out", cout, cout, 3, pad=1,
                          residual=cur, res_mode=mode))
            cur, cin = f"{n}.out", cout
    L.append(Head("fc", cur, 10))
    return Network("resnet20", (32, 32, 3), 10, L, dataset="cifar10")


def resnet50() -> Network:
    L: List[Layer] = [
        Conv("stem", "input", "s0", 3, 64, 7, stride=2, pad=3),
        MaxPool("pool", "s0", "p0", 3, 2, 1),
    ]
    cur, cin = "p0", 64
    for stage, (width, blocks) in enumerate(((64, 3), (128, 4), (256, 6), (512, 3))):
        cout = width * 4
        for blk in range(blocks):
            stride = 2 if (stage > 0 and blk == 0) else 1
            n = f"l{stage + 1}.{blk}"
            res = cur
            if blk == 0:
                L.append(Conv(f"{n}.down", cur, f"{n}.sc", cin, cout, 1, stride=stride, relu=False))
                res = f"{n}.sc"
            L.append(Conv(f"{n}.conv1", cur, f"{n}.a", cin, width, 1))
            L.append(Conv(f"{n}.conv2", f"{n}.a", f"{n}.b", width, width, 3, stride=stride, pad=1))
            L.append(Conv(f"{n}.conv3", f"{n}.b", f"{n}.out", width, cout, 1, residual=res))
            cur, cin = f"{n}.out", cout
    L.append(AvgPool("avgpool", cur, "pooled"))
    L.append(Conv("fc", "pooled", "logits", 2048, 1000, 1, bn=False, bias=True, relu=False,
                  out_f32=True))
    L.append(Softmax("softmax", "logits", 1000))
    return Network("resnet50", (224, 224, 3), 1000, L, dataset="imagenet")


MODELS: Dict[str, Callable[[], Network]] = {
    "lenet5": lenet5,
    "resnet20": resnet20,
    "resnet50": resnet50,
}


def get_model(name: str) -> Network:
    try:
        return MODELS[name]()
    except KeyError:
        raise ValueError(f"unknown model {name!r}; choose from {sorted(MODELS)}") from None
