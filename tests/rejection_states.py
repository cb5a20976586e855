"""PCG64 states whose next 32-bit draws are Lemire rejections (test helper).

numpy's Generator.integers(1, k+1) draws 32-bit words with Lemire's method and
rejects a word x when (x * k) mod 2^32 < (2^32 - k) mod k — probability
<= k / 2^32, so random seeds essentially never hit it.  These helpers build
the 5-word state (tile_match_gym_amd.seeding layout: state lo / hi, inc lo /
hi, has_uint32 << 32 | uinteger) whose *next* PCG64 output is a chosen value:
the output of state s' is XSL-RR(s'), so s' = (hi = 0, lo = value) gives
exactly `value` (rotation 0), and the state before it is (s' - inc) * A^-1.
A low word 0 is rejected for every k that is not a power of two.
"""
import numpy as np

PCG_A = 0x2360ED051FC65DA44385DF649FCCF645
M128 = (1 << 128) - 1


def state_before_output(value: int, inc: int) -> int:
    """The 128-bit state whose next output is `value` (< 2^58, so the rotation is 0)."""
    nxt = value & ((1 << 64) - 1)                # hi = 0
    return ((nxt - inc) * pow(PCG_A, -1, 1 << 128)) & M128


def rejecting_words(base_words: np.ndarray, value: int = 0x0000123400000000) -> np.ndarray:
    """Copies of 5-word states (same increments) moved so that the next output
    is `value`: its low half — the next draw — is 0, a Lemire rejection."""
    out = np.array(base_words, dtype=np.uint64).copy()
    for i in range(out.shape[0]):
        inc = int(out[i, 2]) | (int(out[i, 3]) << 64)
        s = state_before_output(value, inc)
        out[i, 0] = np.uint64(s & ((1 << 64) - 1))
        out[i, 1] = np.uint64(s >> 64)
        out[i, 4] = np.uint64(0)                 # no buffered half-word
    return out
