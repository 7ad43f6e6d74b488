"""Model weight files (SURVEY.md §5.4 "Weights: random init with a fixed seed, or .npz /
safetensors-style load").

The reference ships its model as a frozen TF SavedModel inside the jar
(``model/saved_model.pb``, InferenceBolt.java:48-57). TF is not available here and the only
pinned contract is input -> softmax, so gale stores the parameters of its own layer list in
framework-neutral files with PyTorch conventions: conv weights ``[Cout, Cin, KH, KW]``, dense
weights ``[N, C]`` and BatchNorm ``gamma/beta/mean/var`` — the names ``init_params`` produces
(``stem.weight``, ``stem.bn.gamma``, ``fc.bias``, ...). Files are read with loaders that execute
nothing from the file (``numpy.load(allow_pickle=False)``, safetensors).
"""

from __future__ import annotations

import os
from typing import Dict

import numpy as np
import torch

from gale.models.graph import Network, init_params


def save_params(params: Dict[str, torch.Tensor], path: str) -> None:
    arrays = {k: v.detach().cpu().float().numpy() for k, v in params.items()}
    if path.endswith(".safetensors"):
        from safetensors.numpy import save_file

        save_file(arrays, path)
    else:
        np.savez(path, **arrays)


def load_params(path: str, net: Network) -> Dict[str, torch.Tensor]:
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file

        arrays = load_file(path)
    else:
        with np.load(path, allow_pickle=False) as z:
            arrays = {k: z[k] for k in z.files}
    template = init_params(net, calibrate=False)
    missing = sorted(set(template) - set(arrays))
    extra = sorted(set(arrays) - set(template))
    if missing or extra:
        raise ValueError(f"{path}: parameter names do not match {net.name}: "
                         f"missing {missing[:5]}, unexpected {extra[:5]}")
    out = {}
    for k, t in template.items():
        a = np.asarray(arrays[k], dtype=np.float32)
        if tuple(a.shape) != tuple(t.shape):
            raise ValueError(f"{path}: {k} has shape {a.shape}, {net.name} expects {tuple(t.shape)}")
        out[k] = torch.from_numpy(a.copy())
    return out
