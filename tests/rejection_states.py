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


def _jump(j: int):
    """(A^j, G_j = sum_{i<j} A^i) mod 2^128: s_j = A^j s + G_j inc."""
    a, g = 1, 0
    # binary powering of the affine map s -> A s + inc, as (mult, add-coefficient of inc)
    am, gm = PCG_A, 1
    while j:
        if j & 1:
            a, g = (a * am) & M128, (g * am + gm) & M128
        am, gm = (am * am) & M128, (gm * am + gm) & M128
        j >>= 1
    return a, g


def words_rejecting_at(base_words: np.ndarray, positions, buffered=None) -> np.ndarray:
    """Copies of 5-word states (same increments) moved so that the 32-bit draw
    at `positions[i]` (0 = the next draw of env i) is a rejected word (0),
    every earlier draw accepted.  buffered[i]: the state holds a buffered
    half-word (numpy's has_uint32), which is draw 0; draws 1, 2 are then the
    low / high halves of the next output, and so on.  The output holding the
    rejected half is (0x1234 << 32 | 0) or (0 << 32 | 0x1234), with rotation 0
    (state hi = 0), and the state j + 1 steps before it is recovered through
    s = A^-(j+1) (s_out - G_(j+1) inc)."""
    out = np.array(base_words, dtype=np.uint64).copy()
    n = out.shape[0]
    positions = np.broadcast_to(np.asarray(positions), (n,))
    buffered = np.zeros(n, bool) if buffered is None else np.broadcast_to(np.asarray(buffered, bool), (n,))
    ainv = pow(PCG_A, -1, 1 << 128)
    for i in range(n):
        inc = int(out[i, 2]) | (int(out[i, 3]) << 64)
        d = int(positions[i])
        if buffered[i]:
            if d == 0:                               # the buffered word itself is rejected
                out[i, 4] = np.uint64(1 << 32)
                continue
            d -= 1
            out[i, 4] = np.uint64((1 << 32) | 0x5678)
        else:
            out[i, 4] = np.uint64(0)
        j, half = d // 2, d & 1
        value = 0x1234 if half else (0x1234 << 32)   # the rejected half is 0, the other accepted
        a, g = _jump(j + 1)
        s = ((value - g * inc) * pow(ainv, j + 1, 1 << 128)) & M128
        out[i, 0] = np.uint64(s & ((1 << 64) - 1))
        out[i, 1] = np.uint64(s >> 64)
    return out
