"""Seeded synthetic packet batches: splitmix64 byte streams.

Content does not change SHA-2 cost; determinism does matter for parity, so
every test input is a pure function of (seed, shape).
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, count: int) -> np.ndarray:
    """count successive splitmix64 outputs from state `seed`."""
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) + _GOLDEN * np.arange(1, count + 1, dtype=np.uint64))
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def random_bytes(seed: int, nbytes: int) -> np.ndarray:
    words = splitmix64(seed, (nbytes + 7) // 8)
    return words.view(np.uint8)[:nbytes].copy()


def fixed_batch(seed: int, n: int, length: int, stride: int = None) -> np.ndarray:
    """n packets of `length` bytes at `stride` (default = length), flat uint8."""
    stride = length if stride is None else stride
    return random_bytes(seed, n * stride)


def mixed_lengths(seed: int, n: int, choices=(64, 512, 1500)) -> np.ndarray:
    r = splitmix64(seed, n)
    return np.asarray(choices, dtype=np.uint32)[r % np.uint64(len(choices))]


def packed(seed: int, lens: np.ndarray, align: int = 1, gap: int = 0):
    """Pack packets of `lens` back to back (each start rounded up to `align`,
    plus `gap` spare bytes) -> (data, offsets)."""
    lens = np.asarray(lens, dtype=np.uint64)
    step = ((lens + np.uint64(gap) + np.uint64(align - 1)) // np.uint64(align)) * np.uint64(align)
    offsets = np.zeros(len(lens), dtype=np.uint64)
    if len(lens) > 1:
        offsets[1:] = np.cumsum(step)[:-1]
    total = int(offsets[-1] + lens[-1]) if len(lens) else 0
    return random_bytes(seed, max(total, 1)), offsets
