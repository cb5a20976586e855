"""CPU check of the lane-per-board step logic (tile-match-gym_amd/csrc/tmg_lane.h):
tools/lane_host compiles the header for the host and runs its per-env step env
by env; every field of every env at every step must equal the oracle's
(tile_match_env.py:93-124 over board.py:330-395).  The lane kernel leaves a
finished board's regeneration to reset_kernel (FL_RESET); here the oracle's
own reset of those envs stands in for that launch, as the product's reset
kernel is checked against the oracle elsewhere (test_gpu_paths.py, the golden
trajectories).  The GPU parity suite then checks the compiled kernel itself."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as orc
from vector_ref import reset_subset

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LANE_DIR = os.path.join(ROOT, "tools", "lane_host")
P, I, I64, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64

# (R, C, k): the c2 shape, 3-plane colours, the 128-cell maximum, small boards that shuffle
SHAPES = [(10, 10, 4), (10, 10, 5), (6, 8, 3), (12, 10, 4), (8, 16, 4), (7, 8, 6), (4, 4, 3)]


def _load(name):
    subprocess.run(["make", "-C", LANE_DIR, name], check=True, stdout=subprocess.DEVNULL)
    L = ctypes.CDLL(os.path.join(LANE_DIR, name))
    L.lane_host_step.argtypes = [I, I, I, I64] + [P] * 9 + [I, I, I, U64, I64, I]
    L.lane_host_step.restype = I
    return L


@pytest.fixture(scope="module")
def lane():
    return _load("liblane_host.so")


def _p(a):
    return a.ctypes.data_as(P)


class LaneBatch:
    def __init__(self, L, o):
        self.L, self.R, self.C, self.k, self.M = L, o.R, o.C, o.k, o.num_moves
        self.smask, self.num_moves = 0, o.num_moves
        self.board, self.rng, self.timer, self.eff = o.board.copy(), o.rng.copy(), o.timer.copy(), o.eff.copy()
        n = o.board.shape[0]
        self.reward, self.n_new, self.n_act = (np.zeros(n, np.int32) for _ in range(3))
        self.flags = np.zeros(n, np.uint8)

    def step(self, a, code, sample=0, key=0, first=0, t=0):
        a = np.ascontiguousarray(a, dtype=np.int32)
        st = self.L.lane_host_step(self.R, self.C, self.k, a.size, _p(self.board), _p(self.rng), _p(self.timer),
                                   _p(a), _p(self.reward), _p(self.n_new), _p(self.n_act), _p(self.flags),
                                   _p(self.eff), self.M, code, sample, key, first, t)
        assert st >= 0, "shape not instantiated in tools/lane_host"
        return st, a


FIELDS = ("board", "rng", "timer", "eff", "reward", "n_new", "n_act", "flags")


def _compare(lb, o, tag):
    n = lb.board.shape[0]
    for f in FIELDS:
        got, want = getattr(lb, f), getattr(o, f)
        bad = np.nonzero((got.reshape(n, -1) != want.reshape(n, -1)).any(axis=1))[0]
        assert bad.size == 0, f"{tag}: {f} differs in {bad.size} envs, first {bad[:5]}"


def _actions(rs, o, A, n):
    """half uniform, half uniform over the effective actions (examples/random_agent.py)"""
    a = rs.integers(0, A, n).astype(np.int32)
    effm = np.unpackbits(o.eff.view(np.uint8).reshape(n, -1), axis=1, bitorder="little")[:, :A]
    for i in np.nonzero(rs.random(n) < 0.5)[0]:
        nz = np.nonzero(effm[i])[0]
        if nz.size:
            a[i] = nz[rs.integers(nz.size)]
    return a


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode", ["same_step", "none"])
def test_lane_step_vs_oracle(lane, shape, mode):
    from tile_match_gym_amd.seeding import batch_rng_words
    R, C, k = shape
    n, M, steps = 1200, 7, 22
    o = orc.OracleBatch(R, C, k, 0, M, batch_rng_words(range(3000, 3000 + n)), threads=8)
    o.reset()
    lb = LaneBatch(lane, o)
    rs = np.random.default_rng(R * 100 + C * 10 + k)
    A = 2 * R * C - R - C
    shuffled = resets = 0
    for t in range(steps):
        a = _actions(rs, o, A, n)
        st, _ = lb.step(a, 2 if mode == "same_step" else 0)
        if mode == "same_step":                    # reset_kernel, masked by FL_RESET
            reset_subset(lb, np.nonzero(lb.flags & 8)[0])
        o.step(a, autoreset=mode == "same_step")
        _compare(lb, o, f"{shape} {mode} step {t}")
        shuffled += int(((o.flags & 4) != 0).sum())
        resets += int(((o.flags & 8) != 0).sum())
        assert st == (4 if ((o.flags & 0x80) != 0).any() else 0)
    if mode == "same_step":
        assert resets > 0
    if shape == (4, 4, 3):
        assert shuffled > 0, "the small board was meant to shuffle"


@pytest.mark.parametrize("shape", [(10, 10, 4), (7, 8, 6)])
def test_lane_policy_and_next_step(lane, shape):
    """The in-kernel policy's draw (oracle/policy_np.py) and the next-step
    autoreset (an env that ended last call is reset instead of stepped)."""
    from oracle.policy_np import sample_effective_np
    from tile_match_gym_amd.seeding import batch_rng_words
    R, C, k = shape
    n, M, steps, key, first = 900, 5, 17, 777, 4096
    o = orc.OracleBatch(R, C, k, 0, M, batch_rng_words(range(9000, 9000 + n)), threads=8)
    o.reset()
    lb = LaneBatch(lane, o)
    A = 2 * R * C - R - C
    pending = np.zeros(n, bool)
    for t in range(steps):
        want_a = sample_effective_np(o.eff, A, key, first, t)
        _, a = lb.step(np.zeros(n, np.int32), 4, sample=1, key=key, first=first, t=t)
        assert np.array_equal(a, want_a), f"step {t}: policy actions"
        reset_subset(lb, np.nonzero(lb.flags & 8)[0])
        # the oracle: pending envs regenerate (reward 0, flags FL_RESET), the rest step
        live = ~pending
        idx = np.nonzero(pending)[0]
        o.step(np.where(live, want_a, 0), autoreset=False)
        reset_subset(o, idx)
        o.reward[idx] = 0
        o.flags[idx] = 8
        pending = (o.flags & 1) != 0
        _compare(lb, o, f"{shape} next-step {t}")


def _asan_body():
    from tile_match_gym_amd.seeding import batch_rng_words
    L = _load("liblane_host_asan.so")
    for R, C, k in [(10, 10, 4), (4, 4, 3), (8, 16, 4)]:
        o = orc.OracleBatch(R, C, k, 0, 4, batch_rng_words(range(64)))
        o.reset()
        lb = LaneBatch(L, o)
        rs = np.random.default_rng(5)
        for t in range(6):
            a = _actions(rs, o, 2 * R * C - R - C, 64)
            lb.step(a, 2)
            reset_subset(lb, np.nonzero(lb.flags & 8)[0])
            o.step(a, autoreset=True)
            _compare(lb, o, f"asan {R}x{C} step {t}")
    print("asan-ok")


def test_lane_host_asan():
    """The same logic under AddressSanitizer + UBSan (shifts, the tail stores),
    in a child process with the ASan runtime preloaded."""
    subprocess.run(["make", "-C", LANE_DIR, "liblane_host_asan.so"], check=True, stdout=subprocess.DEVNULL)
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=libasan, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1")
    code = ("import sys; sys.path[:0] = [%r, %r, %r]; import test_lane_host as t; t._asan_body()"
            % (os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "tile-match-gym_amd")))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "asan-ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
