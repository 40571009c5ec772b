"""Host reference of the message integrity checksum (erasurehead_amd/parallel/integrity.py)."""
import struct

import numpy as np

from erasurehead_amd.parallel.integrity import parse_tags, row_checksum


def test_checksum_definition():
    x = np.array([1.5, -2.0, 0.0], dtype=np.float64)
    bits = [struct.unpack("<Q", struct.pack("<d", v))[0] for v in x]
    want = sum(b * (2 * j + 1) for j, b in enumerate(bits)) % 2**64
    assert row_checksum(x) == want
    y = np.array([1.5, -2.0, 0.25, 3.0], dtype=np.float32)
    bits = [struct.unpack("<I", struct.pack("<f", v))[0] for v in y]
    assert row_checksum(y) == sum(b * (2 * j + 1) for j, b in enumerate(bits)) % 2**64


def test_checksum_sees_single_flips_swaps_and_stale_rows():
    rng = np.random.RandomState(0)
    x = rng.randn(1000)
    base = row_checksum(x)
    for j in (0, 1, 499, 999):
        for bit in (0, 7, 31, 52, 63):
            y = x.copy()
            y.view(np.uint64)[j] ^= np.uint64(1) << np.uint64(bit)
            assert row_checksum(y) != base
    y = x.copy()
    y[[3, 700]] = y[[700, 3]]
    assert row_checksum(y) != base
    assert row_checksum(rng.randn(1000)) != base  # a different (stale) row


def test_parse_tags():
    raw = struct.pack("<IIQ", 5, 2, 2**64 - 3) + struct.pack("<IIQ", 6, 0, 17)
    assert parse_tags(raw) == [(5, 2, 2**64 - 3), (6, 0, 17)]
