"""GPU prediction text (csrc/kernels/format.hip) against the host's Java Float.toString
(codec::format_float_java, itself pinned to Java's output in tests/test_codec.py): every value
must produce the identical string. The reference writes each probability with Jackson, i.e.
Float.toString (InferenceBolt.java:88-90)."""

import json
import re

import numpy as np
import pytest
import torch

from gale._native import native

C = native()
pytestmark = pytest.mark.gpu


def gpu_format(x: np.ndarray) -> list:
    x = np.ascontiguousarray(x, dtype=np.float32)
    xd = torch.from_numpy(x).cuda()
    out = torch.zeros((x.size, 16), dtype=torch.uint8, device="cuda")
    C.format_floats_java(x.size, xd.data_ptr(), out.data_ptr(),
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    return [bytes(r[:r[15]]).decode() for r in o]


def special_values() -> np.ndarray:
    v = [0.0, -0.0, 1.0, -1.0, 0.5, 0.1, 0.2, 0.3, 1e-3, 9.999999e-4, 1e-4, 1e7, 9999999.0,
         1e8, 123456.7, 3.4028235e38, 1.17549435e-38, 1.4e-45, 2.8e-45, 1e-45, 7e-45,
         np.inf, -np.inf, np.nan, 0.001, 0.00999, 0.0999, 0.999, 0.9999999, 1.0000001,
         2.0 ** -126, 2.0 ** -127, 2.0 ** -149, 2.0 ** 23, 2.0 ** 24, 2.0 ** -20, 100.0,
         1e-5, 5e-5, 4.4e-5, 3.3333333e-1, 6.6666667e-1]
    v += [2.0 ** k for k in range(-149, 128, 3)]
    v += [10.0 ** k for k in range(-45, 39)]
    return np.array(v, dtype=np.float32)


def test_format_special_values_match_host():
    x = special_values()
    got = gpu_format(x)
    for v, s in zip(x, got):
        assert s == C.format_float_java(float(v)), (repr(float(v)), s)


@pytest.mark.parametrize("kind", ["probs", "loguniform", "bits"])
def test_format_random_match_host(kind):
    rng = np.random.default_rng({"probs": 1, "loguniform": 2, "bits": 3}[kind])
    n = 40000
    if kind == "probs":  # softmax rows: what the engine formats
        z = rng.normal(size=(n // 10, 10)).astype(np.float32) * 4
        e = np.exp(z - z.max(axis=1, keepdims=True))
        x = (e / e.sum(axis=1, keepdims=True)).astype(np.float32).ravel()
    elif kind == "loguniform":
        x = (10.0 ** rng.uniform(-45, 38, n)).astype(np.float32)
    else:  # every finite binary32 pattern class, both signs
        b = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        x = b.view(np.float32)
        x = x[np.isfinite(x)]
    got = gpu_format(x)
    bad = [(float(v), s, C.format_float_java(float(v))) for v, s in zip(x, got)
           if s != C.format_float_java(float(v))]
    assert not bad, bad[:5]


def test_engine_gpu_encode_text_is_host_text():
    """End to end with gpu_encode on: every number in the output records is the host's
    Float.toString of the value it denotes."""
    from gale.config import GaleConfig
    from gale.engine import Engine

    b = C.kafka.Broker()
    b.start()
    try:
        b.create_topic("in", 1)
        b.create_topic("out", 1)
        rng = np.random.default_rng(4)
        for i in range(12):
            b.append("in", 0, [C.encode_instances(rng.random((1 + i % 3, 32, 32, 3),
                                                             dtype=np.float32))])
        cfg = GaleConfig(topology_name="f", input_topic="in", output_topic="out",
                         model="resnet20", bootstrap=f"127.0.0.1:{b.port}",
                         start_offset="earliest", max_batch=16, max_wait_us=500,
                         gpu_encode=True)
        eng = Engine(cfg, devices=[0], max_records=12)
        eng.start()
        assert eng.wait(120), eng.stats()
        eng.stop()
        out = b.read("out", 0)
    finally:
        b.stop()
    assert len(out) == 12
    n = 0
    for r in out:
        txt = r["value"].decode()
        assert json.loads(txt)["predictions"]
        for tok in re.findall(r"[-0-9.E]+", txt):
            assert tok == C.format_float_java(float(np.float32(tok))), tok
            n += 1
    assert n == 10 * sum(1 + i % 3 for i in range(12))
