"""Bit-exact decimal -> float32 conversion of the GPU JSON parser against a correctly rounded
reference (the reference's decoder is Jackson -> Java Float.parseFloat, which rounds the exact
decimal value to the nearest binary32, ties to even; InferenceBolt.java:76).

The reference value is computed with exact rational arithmetic (fractions.Fraction): NOT
``np.float32(float(text))``, which rounds twice (decimal -> double -> float) and is wrong on
halfway cases. The GPU parser is exact for any number of digits: the first 19 decide unless a
binary32 midpoint lies within 1e-19 (relative) of the token, and then every digit is compared
with the midpoint's exact decimal expansion (midpoints written out in full, +- one unit in a
far digit, subnormal midpoints of ~110 digits, integers past 2^64 are checked here).
"""

import random
import struct
from fractions import Fraction

import numpy as np
import pytest

from gale._native import native

C = native()


def f32_correct(text: str) -> int:
    """Bits of the binary32 nearest to the decimal `text` (ties to even), Java semantics."""
    x = Fraction(text)
    sign = 0x80000000 if text.strip().startswith("-") else 0
    x = abs(x)
    if x == 0:
        return sign
    e = x.numerator.bit_length() - x.denominator.bit_length()
    if Fraction(2) ** e > x:
        e -= 1
    if e < -126:  # subnormal range: quantum 2^-149
        m = round(x / Fraction(2) ** -149)
        return sign | m  # m == 2^23 becomes the smallest normal, bit-exactly
    m = round(x / Fraction(2) ** (e - 23))  # in [2^23, 2^24]
    if m == 1 << 24:
        m >>= 1
        e += 1
    if e > 127:
        return sign | 0x7F800000
    return sign | ((e + 127) << 23) | (m & 0x7FFFFF)


def sig_digits(text: str) -> int:
    m = text.lower().lstrip("+-").split("e")[0].replace(".", "").lstrip("0")
    return len(m.rstrip("0")) if m else 0


def bits(v: float) -> int:
    return struct.unpack("<I", struct.pack("<f", v))[0]


TRICKY = [
    "1.000000059604644775390625",        # exactly halfway 1 .. 1+2^-23: ties to even -> 1
    "1.000000178813934326171875",        # halfway, odd below -> rounds up
    "1.000000059604644775000000000001",  # 31 digits: a dropped nonzero tail (sticky bit)
    "1.000000059604644775",              # 19 digits, just below the midpoint
    "1.000000059604644776",              # 19 digits, just above
    "0.1", "0.2", "0.3", "3.4028235e38", "3.4028234e38", "3.4028236e38",
    "340282356779733661637539395458142568448",      # FLT_MAX + half ulp: ties -> inf
    "340282356779733661637539395458142568447",      # just below -> FLT_MAX
    "1e-45", "7e-46", "7.006492321624086e-46", "7.1e-46", "1.401298464324817e-45",
    "1.1754942e-38", "1.17549435e-38", "1.1754943508222875e-38", "5.877471754111438e-39",
    "8388608.5", "8388609.5", "16777217", "16777219", "33554433",
    "9007199254740993", "123456789012345678", "1.7976931348623157e308", "4.9e-324",
    "-0.0", "-1.000000059604644775390625", "1E10", "2.5e+5", "6.02214076e23",
    "0.000000000000000000000000000000000000000000001",
]


def dyadic_text(x: Fraction) -> str:
    """Exact decimal expansion of a dyadic rational (denominator 2^k): k fraction digits."""
    k = x.denominator.bit_length() - 1
    assert x.denominator == 1 << k
    digits = str(x.numerator * 5 ** k).rjust(k + 1, "0")
    return digits[:-k] + "." + digits[-k:] if k else digits


def long_cases(rng, n=300):
    """Decimals of > 19 significant digits at and around binary32 midpoints."""
    out = []
    for i in range(n):
        kind = i % 3
        if kind == 0:  # normal range
            f = np.float32(rng.uniform(1, 2) * 2.0 ** rng.randint(-126, 126))
        elif kind == 1:  # subnormal: midpoints of up to ~110 significant digits
            f = np.float32(rng.randint(1, (1 << 23) - 2) * 2.0 ** -149)
        else:  # integers: midpoints above 2^64
            f = np.float32(rng.uniform(1, 2) * 2.0 ** rng.randint(64, 126))
        up = np.nextafter(f, np.float32(np.inf))
        mid = (Fraction(float(f)) + Fraction(float(up))) / 2
        t = dyadic_text(mid)
        out += [t,                                   # exact tie: to even
                t + ("0000000000" if "." in t else ".0000000000"),  # zeros after the tie
                dyadic_text(mid + Fraction(1, 1 << 400)) if kind != 2 else t + ".00001",
                dyadic_text(mid - Fraction(1, 1 << 400)) if kind != 2 else str(int(mid) - 1)]
        # the same value in exponent form, mantissa digits shifted
        m = t.replace(".", "").lstrip("0")
        e = len(t.split(".")[0]) - (len(t.replace(".", "")) - len(m)) - 1
        out.append(f"{m[0]}.{m[1:]}E{e}")
        out.append(t[:30])  # truncated
    return out


def gpu_parse_numbers(texts):
    import torch

    arr = ("[[[" + ",".join(f"[{t}]" for t in texts) + "]]]").encode()
    n = len(texts)
    rec = np.zeros(1, dtype=[("off", "<i8"), ("len", "<i4"), ("slot", "<i4"), ("images", "<i4"),
                             ("status", "<i4"), ("tile0", "<i4"), ("has_cnt", "<i4"),
                             ("cnt_off", "<i8"), ("pad", "<i8")])
    tiles = C.json_tile_count(0, len(arr))
    rec[0] = (0, len(arr), 0, 1, 0, 0, 0, 0, 0)
    raw = np.frombuffer(arr + b" " * (16 + (-len(arr)) % 16), dtype=np.uint8)
    d_raw = torch.from_numpy(raw.copy()).cuda()
    d_rec = torch.from_numpy(rec.view(np.uint8).copy()).cuda()
    d_map = torch.zeros(tiles, dtype=torch.int32, device="cuda")
    d_cnt = torch.zeros(tiles, dtype=torch.int32, device="cuda")
    out = torch.zeros(n, device="cuda")
    C.json_parse_instances(1, tiles, d_rec.data_ptr(), d_map.data_ptr(), d_raw.data_ptr(), 1, n,
                           1, d_cnt.data_ptr(), out.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    st = int(d_rec.cpu().numpy().view(rec.dtype)["status"][0])
    return out.cpu().numpy().view(np.uint32), st


def test_reference_rounding_is_exact():
    """The host oracle itself: ties to even and no double rounding."""
    assert f32_correct("1.000000059604644775390625") == bits(1.0)
    assert f32_correct("1.000000059604644775390626") == bits(1.0) + 1
    assert f32_correct("1e-45") == 1
    assert f32_correct("340282356779733661637539395458142568448") == 0x7F800000
    # np.float32(float(s)) double-rounds this one (the reason for the exact oracle)
    s = "1.00000005960464477539062500000000001"
    assert f32_correct(s) == bits(1.0) + 1


@pytest.mark.gpu
def test_gpu_json_float_is_correctly_rounded():
    rng = random.Random(7)
    texts = list(TRICKY)
    for _ in range(3000):  # 9-digit decimals over the whole binary32 range
        texts.append(f"{rng.randint(1, 999999999)}e{rng.randint(-54, 30)}")
    for _ in range(3000):  # Java Float.toString output must round-trip bit-exactly
        v = np.float32(rng.uniform(-1, 1) * 10.0 ** rng.randint(-40, 38))
        texts.append(C.format_float_java(float(v)))
    for _ in range(2000):  # double repr (17 digits: the slow, exact path)
        texts.append(repr(rng.uniform(0, 1) * 10.0 ** rng.randint(-30, 30)))
    for _ in range(500):  # decimals right at binary32 midpoints, +- one unit in the 20th digit
        f = np.float32(rng.uniform(0.5, 2.0))
        mid = (Fraction(float(f)) + Fraction(float(np.nextafter(f, np.float32(3))))) / 2
        d = f"{float(mid):.18e}"  # 19 significant digits, within 1e-19 of the midpoint
        texts.append(d)
    texts += long_cases(rng)
    texts += ["0." + "0" * 40 + "1" + "0" * 60 + "1", "9" * 60, "1" + "0" * 38 + ".5",
              "0.99999997019767761230468750000000000001", "0.9999999701976776123046874999999999"]
    got, st = gpu_parse_numbers(texts)
    assert st == 0
    want = np.array([f32_correct(t) for t in texts], dtype=np.uint32)
    assert sum(sig_digits(t) > 19 for t in texts) > 1000
    bad = [(texts[i], hex(got[i]), hex(want[i])) for i in np.nonzero(got != want)[0][:10]]
    assert not bad, bad
