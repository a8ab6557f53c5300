"""Deterministic inputs the golden fixtures refer to (regenerated, never stored).

* ``blob()``: the byte blob every flat/chain fixture case indexes into: the repo's
  splitmix64 stream (aipstack_amd/synth.py, seed 42) with three constant regions.
* ``mt19937_64_bytes(seed, n)``: low 8 bits of successive std::mt19937_64(seed) outputs
  (MT19937-64 as standardised in C++11 [rand.predef]); SURVEY.md 8(c)'s sample known
  answers were taken by the survey on these bytes with the reference itself.
"""
from __future__ import annotations

import numpy as np

from aipstack_amd import synth

BLOB_SIZE = 140000
BLOB_SPEC = {
    "seed": 42,
    "size": BLOB_SIZE,
    "zeros": [100000, 110000],   # all 0x00
    "ones": [110000, 120000],    # all 0xFF
    "mod0": [120000, 140000],    # 0x00 at 120000, then 0xFF: sums = 0 (mod 0xFFFF)
}


def blob() -> np.ndarray:
    b = synth.random_bytes(BLOB_SPEC["seed"], BLOB_SIZE)
    z0, z1 = BLOB_SPEC["zeros"]
    f0, f1 = BLOB_SPEC["ones"]
    m0, m1 = BLOB_SPEC["mod0"]
    b[z0:z1] = 0x00
    b[f0:f1] = 0xFF
    b[m0:m1] = 0xFF
    b[m0] = 0x00
    return b


def mt19937_64_bytes(seed: int, n: int) -> np.ndarray:
    """Low bytes of the first n outputs of std::mt19937_64(seed)."""
    nn, mm = 312, 156
    mask = (1 << 64) - 1
    mt = [0] * nn
    mt[0] = seed & mask
    for i in range(1, nn):
        mt[i] = (6364136223846793005 * (mt[i - 1] ^ (mt[i - 1] >> 62)) + i) & mask
    idx = nn
    out = np.zeros(n, dtype=np.uint8)
    upper, lower = 0xFFFFFFFF80000000, 0x7FFFFFFF
    for k in range(n):
        if idx >= nn:
            for i in range(nn):
                x = (mt[i] & upper) | (mt[(i + 1) % nn] & lower)
                xa = x >> 1
                if x & 1:
                    xa ^= 0xB5026F5AA96619E9
                mt[i] = mt[(i + mm) % nn] ^ xa
            idx = 0
        y = mt[idx]
        idx += 1
        y ^= (y >> 29) & 0x5555555555555555
        y ^= (y << 17) & 0x71D67FFFEDA60000
        y ^= (y << 37) & 0xFFF7EEE000000000
        y ^= y >> 43
        out[k] = y & 0xFF
    return out
