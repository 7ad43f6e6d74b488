"""Host JSON codec: the InstObj/PredObj contract (InstObj.java:8, PredObj.java:9) and Jackson
compatibility (FAIL_ON_UNKNOWN_PROPERTIES, Java Float.toString output)."""

import json

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from gale._native import native

C = native()
OK, BAD_ENVELOPE, UNKNOWN_KEY, BAD_SHAPE, EMPTY, BAD_NUMBER, NULL_INSTANCES = range(7)


def rec(arr):
    return json.dumps({"instances": arr}).encode()


def img(h, w, c, base=0.0):
    return [[[base + (i * w + j) * c + k for k in range(c)] for j in range(w)] for i in range(h)]


@pytest.mark.parametrize("n", [1, 2, 5])
def test_scan_counts_images(n):
    data = rec([img(4, 3, 2, base=i) for i in range(n)])
    st_, off, ln, images = C.scan_instances(data, 4, 3, 2)
    assert st_ == OK and images == n
    assert data[off:off + 1] == b"[" and data[off + ln - 1:off + ln] == b"]"


@pytest.mark.parametrize("data,expected", [
    (b'{"instances": [[[[1,2]]]], "extra": 1}', UNKNOWN_KEY),      # Jackson FAIL_ON_UNKNOWN
    (b'{"other": [[[[1,2]]]]}', UNKNOWN_KEY),
    (b'{"instances": null}', NULL_INSTANCES),
    (b'{}', NULL_INSTANCES),
    (b'{"instances": []}', EMPTY),
    (b'not json', BAD_ENVELOPE),
    (b'[1,2,3]', BAD_ENVELOPE),
    (b'{"instances": [[[[1,2]]]]', BAD_ENVELOPE),                  # unterminated object
    (b'{"instances": [[["a","b"]]]}', BAD_NUMBER),
    (b'  {  "instances" :  [[[[1,2]]]]  }  ', OK),                  # whitespace everywhere
])
def test_scan_statuses(data, expected):
    st_ = C.scan_instances(data, 1, 1, 2)[0]
    assert st_ == expected, C.status_name(st_)


def test_parse_host_matches_json():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((3, 4, 5, 2)).astype(np.float32)
    data = rec(x.tolist())
    st_, out = C.parse_instances_host(data, 4, 5, 2)
    assert st_ == OK
    np.testing.assert_array_equal(out, x)  # float64 repr -> float32 rounds back exactly


@pytest.mark.parametrize("bad", [
    [[[[1, 2]], [[3]]]],          # ragged innermost
    [[[[1, 2], [3, 4]]]],         # W=2 where the model expects W=1
    [[[1, 2]]],                   # rank 3
    [[[[1, 2, 3]]]],              # C=3
])
def test_parse_host_rejects_bad_shapes(bad):
    st_, _ = C.parse_instances_host(rec(bad), 1, 1, 2)
    assert st_ in (BAD_SHAPE, EMPTY), C.status_name(st_)


@pytest.mark.parametrize("num", ["01", "1.", ".5", "+1", "1e", "--1", "0x10", "1.2.3", "NaN"])
def test_parse_host_rejects_bad_numbers(num):
    data = b'{"instances": [[[[' + num.encode() + b', 1]]]]}'
    st_, _ = C.parse_instances_host(data, 1, 1, 2)
    assert st_ in (BAD_NUMBER, BAD_SHAPE), C.status_name(st_)


# Java Float.toString (JDK >= 19 shortest-digit spec; identical to JDK 8 for these values)
@pytest.mark.parametrize("v,s", [
    (0.0, "0.0"), (-0.0, "-0.0"), (1.0, "1.0"), (0.1, "0.1"), (0.5, "0.5"), (3.0, "3.0"),
    (100.0, "100.0"), (0.001, "0.001"), (0.0001, "1.0E-4"), (1e-5, "1.0E-5"),
    (1.25e-5, "1.25E-5"), (9999999.0, "9999999.0"), (1e7, "1.0E7"), (1.5e7, "1.5E7"),
    (123456.7, "123456.7"), (-2.5, "-2.5"), (float("inf"), "Infinity"),
    (float("-inf"), "-Infinity"), (float("nan"), "NaN"), (0.3, "0.3"),
    (0.09874, "0.09874"), (3.4028235e38, "3.4028235E38"), (1.4e-45, "1.4E-45"),
])
def test_format_float_java(v, s):
    assert C.format_float_java(v) == s


@settings(max_examples=300, deadline=None)
@given(st.floats(width=32, allow_nan=False, allow_infinity=False))
def test_format_float_java_roundtrips(v):
    s = C.format_float_java(v)
    assert np.float32(float(s)) == np.float32(v)


# Java 8 Float.toString (the reference runtime, --float-format java8; csrc/codec/java8_float.cpp).
# Pinned cases: values whose Java 8 text is widely documented - (float) 2^31 prints
# "2.14748365E9" and Float.MIN_NORMAL "1.17549435E-38" on Java 8 (JDK 19+: "2.1474836E9",
# "1.1754944E-38"); everything else is a property (no JVM here to pin more).
@pytest.mark.parametrize("v,s", [
    (0.0, "0.0"), (-0.0, "-0.0"), (1.0, "1.0"), (0.1, "0.1"), (0.5, "0.5"), (100.0, "100.0"),
    (0.001, "0.001"), (0.0001, "1.0E-4"), (1e-5, "1.0E-5"), (1e7, "1.0E7"),
    (123456.7, "123456.7"), (float("inf"), "Infinity"), (float("nan"), "NaN"),
    (3.4028235e38, "3.4028235E38"), (1.4e-45, "1.4E-45"), (1 / 3, "0.33333334"),
    (2.0 ** 31, "2.14748365E9"), (2.0 ** 30, "1.07374182E9"),
    (1.1754943508222875e-38, "1.17549435E-38"),
])
def test_format_float_java8(v, s):
    assert C.format_float_java8(v) == s


def _sig(s):
    return len(s.lstrip("-").split("E")[0].replace(".", "").strip("0"))


@settings(max_examples=500, deadline=None)
@given(st.floats(width=32, allow_nan=False, allow_infinity=False))
def test_format_float_java8_roundtrips_and_is_never_shorter(v):
    s8, s19 = C.format_float_java8(v), C.format_float_java(v)
    assert np.float32(float(s8)) == np.float32(v)
    assert _sig(s8) >= _sig(s19)


def test_java8_and_jdk19_agree_on_probabilities():
    """Softmax outputs (0, 1]: the two rules print the same text (200 k samples, incl. tiny)."""
    rng = np.random.default_rng(3)
    p = np.concatenate([rng.random(100_000), rng.random(100_000) ** 12]).astype(np.float32)
    diff = [float(x) for x in p if C.format_float_java8(float(x)) != C.format_float_java(float(x))]
    assert not diff, diff[:5]
    big = np.float32(2.0 ** 31)
    assert C.encode_predictions(np.array([[big]], np.float32), False, True) == \
        b'{"predictions":[[2.14748365E9]]}'


def test_encode_predictions_json_and_json_string():
    p = np.array([[0.5, 0.25, 1e-5], [0.1, 0.2, 0.7]], dtype=np.float32)
    out = C.encode_predictions(p, False)
    assert out == b'{"predictions":[[0.5,0.25,1.0E-5],[0.1,0.2,0.7]]}'
    d = json.loads(out)
    np.testing.assert_allclose(np.array(d["predictions"], dtype=np.float32), p)
    s = C.encode_predictions(p[:1], True)  # spring JsonSerializer double encoding (E8)
    assert json.loads(json.loads(s)) == {"predictions": [[0.5, 0.25, 1e-5]]}


def test_encode_error_record():
    e = json.loads(C.encode_error(UNKNOWN_KEY, 'bad "key"', False))
    assert e == {"error": "unknown_key", "detail": 'bad "key"'}
    e2 = json.loads(json.loads(C.encode_error(BAD_SHAPE, "", True)))
    assert e2 == {"error": "bad_shape"}


@settings(max_examples=40, deadline=None)
@given(st.integers(1, 3), st.integers(1, 4), st.integers(1, 4), st.integers(1, 3),
       st.integers(0, 2**31 - 1))
def test_instances_roundtrip(n, h, w, c, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, h, w, c)) * 10.0 ** rng.integers(-6, 6)).astype(np.float32)
    data = C.encode_instances(x)
    assert json.loads(data)["instances"] is not None
    st_, off, ln, images = C.scan_instances(data, h, w, c)
    assert st_ == OK and images == n
    st2, y = C.parse_instances_host(data, h, w, c)
    assert st2 == OK
    np.testing.assert_array_equal(y, x)


@pytest.mark.parametrize("json_string", [False, True])
def test_encode_predictions_text_slots_match_float_encoder(json_string):
    """The engine's path for device-formatted predictions (16-byte slots, length in byte 15,
    csrc/kernels/format.hip) produces exactly the bytes of the float encoder."""
    rng = np.random.default_rng(7)
    p = rng.random((3, 10)).astype(np.float32)
    p[0, 0], p[1, 1], p[2, 2] = 0.0, 1.0, 1.4e-45
    slots = bytearray()
    for v in p.ravel():
        s = C.format_float_java(float(v)).encode()
        slots += s + bytes(15 - len(s)) + bytes([len(s)])
    got = C.encode_predictions_text(bytes(slots), 3, 10, json_string)
    assert got == C.encode_predictions(p, json_string)
