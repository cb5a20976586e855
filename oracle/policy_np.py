"""numpy restatement of tmg_sample_effective — TEST INFRASTRUCTURE (the checker
for tests/ and bench.py's cpu_baseline leg, never the product path): the
examples' uniform choice over info["effective_actions"]
(src/examples/q_learning.py:19-25), drawn from the counter-based stream of
shard.synthetic_actions."""
import numpy as np

from tile_match_gym_amd.shard import _splitmix64


def sample_effective_np(eff: np.ndarray, num_actions: int, key: int, first_env: int, t: int) -> np.ndarray:
    """eff: (n, W) uint64 effective-action bitmasks -> (n,) int32 actions."""
    eff = np.ascontiguousarray(eff, dtype=np.uint64)
    n = eff.shape[0]
    g = np.arange(first_env, first_env + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = _splitmix64(np.uint64(key) * np.uint64(0xD1B54A32D192ED03) + g)
        h = _splitmix64(base ^ (np.uint64(t) * np.uint64(0x9E3779B97F4A7C15))) >> np.uint64(32)
    bits = np.unpackbits(eff.view(np.uint8).reshape(n, -1), axis=1, bitorder="little").astype(np.int64)
    count = bits.sum(axis=1).astype(np.uint64)
    r = ((h * count) >> np.uint64(32)).astype(np.int64)
    pick = np.argmax(np.cumsum(bits, axis=1) > r[:, None], axis=1)
    uni = ((h * np.uint64(num_actions)) >> np.uint64(32)).astype(np.int64)
    return np.where(count > 0, pick, uni).astype(np.int32)
