"""Per-env RNG state: numpy Generator(PCG64) packed as 5 uint64 words.

The reference drives all board randomness from ONE ``np.random.default_rng(seed)``
per env (tile_match_env.py:49-51, set_seed :79-82).  The device keeps that
stream bit-exactly; its state per env is

    words[0:2] = 128-bit LCG state (lo, hi)
    words[2:4] = 128-bit increment (lo, hi)
    words[4]   = has_uint32 << 32 | uinteger   (numpy's persistent 32-bit half-word buffer)

Seeding uses numpy's own SeedSequence -> PCG64 (numpy, not reference code).
"""
from __future__ import annotations

import numpy as np

_M64 = (1 << 64) - 1


def rng_words_from_generator(gen) -> np.ndarray:
    bg = gen.bit_generator if isinstance(gen, np.random.Generator) else gen
    st = bg.state
    if st.get("bit_generator") != "PCG64":
        raise ValueError(f"only PCG64 generators are supported, got {st.get('bit_generator')}")
    s, inc = st["state"]["state"], st["state"]["inc"]
    return np.array([s & _M64, s >> 64, inc & _M64, inc >> 64,
                     (int(st["has_uint32"]) << 32) | int(st["uinteger"])], dtype=np.uint64)


def rng_words_from_seed(seed) -> np.ndarray:
    """== np.random.default_rng(seed) state (tile_match_env.py:49)."""
    return rng_words_from_generator(np.random.PCG64(seed))


def generator_from_words(words) -> np.random.Generator:
    w = [int(x) for x in np.asarray(words, dtype=np.uint64)]
    bg = np.random.PCG64()
    bg.state = {"bit_generator": "PCG64",
                "state": {"state": w[0] | (w[1] << 64), "inc": w[2] | (w[3] << 64)},
                "has_uint32": (w[4] >> 32) & 1, "uinteger": w[4] & 0xFFFFFFFF}
    return np.random.Generator(bg)


def batch_rng_words(seeds) -> np.ndarray:
    """(N,5) uint64 state words for a sequence of integer seeds."""
    seeds = list(seeds)
    out = np.empty((len(seeds), 5), dtype=np.uint64)
    for i, s in enumerate(seeds):
        out[i] = rng_words_from_seed(int(s))
    return out
