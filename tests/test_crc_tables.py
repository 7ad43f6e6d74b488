"""The GPU CRC32C kernel's algorithm (csrc/kernels/ingest.hip) emulated on the host with the
exact tables it loads (kafka.crc32c_device_tables): slicing-by-4 folding of 64-byte lane pieces,
per-lane shifts by a GF(2) multiply with x^(8*64*(63-lane)) mod P, XOR reduction, and the host-side
join of 4 KiB windows into a record batch's standard CRC. Checked against the host CRC32C."""

import os

import numpy as np
import pytest

from gale._native import native

K = native().kafka
T = np.array(K.crc32c_device_tables(), dtype=np.uint64)


def _byte(c, b):
    return int((c >> 8) ^ T[(c ^ b) & 0xFF])


def _word(c, w):
    x = c ^ w
    return int(T[768 + (x & 0xFF)] ^ T[512 + ((x >> 8) & 0xFF)] ^ T[256 + ((x >> 16) & 0xFF)]
               ^ T[x >> 24])


def _mulmod(a, b):  # the device's gf2_mulmod: a * b mod P, reflected
    r = 0
    for i in range(32):
        if (a >> (31 - i)) & 1:
            r ^= b
        b = (b >> 1) ^ (0x82F63B78 if b & 1 else 0)
    return r


def window_crc(buf, end, length):
    """What one wave computes for the window [end - length, end)."""
    cs = end - length
    acc = 0
    for lane in range(64):
        wa = end - 64 * (64 - lane)
        hi = wa + 64
        q = max(wa, cs)
        c = 0
        while q < hi and q & 3:
            c = _byte(c, buf[q]); q += 1
        while q + 4 <= hi:
            c = _word(c, int.from_bytes(buf[q:q + 4], "little")); q += 4
        while q < hi:
            c = _byte(c, buf[q]); q += 1
        acc ^= _mulmod(c, int(T[1024 + lane]))
    return acc


@pytest.mark.parametrize("start,length", [(0, 100), (3, 4096), (21, 5000), (7, 12289)])
def test_window_join_matches_host_crc32c(start, length):
    buf = os.urandom(start + length + 8)
    end = start + length
    n = -(-length // 4096)
    raw = 0
    for k in range(n):
        e = end - 4096 * (n - 1 - k)
        ln = length - 4096 * (n - 1) if k == 0 else 4096
        c = window_crc(buf, e, ln)
        raw = c if k == 0 else K.crc32c_shift(raw, 4096) ^ c
    std = raw ^ K.crc32c_shift(0xFFFFFFFF, length) ^ 0xFFFFFFFF
    assert std == K.crc32c(buf[start:end])
