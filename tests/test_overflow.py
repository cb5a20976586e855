"""Capacity limits of the general kernels: adversarial boards (tests/adversarial.py)
whose cascades outgrow the LDS lists are queued by the step kernel and re-run by
spill_kernel on worst-case global-memory lists (tmg_board.hip ListStore /
WsSerialBig).  Every step must still equal the oracle (tmg_oracle.c, the C
restatement of board.py:330-395 pinned by the reference's goldens) bit for bit.

The first step of each board takes an action the oracle finds effective; later
steps take effective actions from the oracle's own masks, so the cascades keep
running on the refilled boards."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from adversarial import MODES, adversarial_boards, effective_actions
from oracle import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU_DIR = os.path.join(ROOT, "tools", "wave_emu")

SHAPES = [(20, 20, 6, 15), (10, 10, 4, 14), (8, 8, 3, 15), (12, 30, 6, 15)]


def _next_actions(o, rs):
    A = o.A
    m = np.unpackbits(o.eff.view(np.uint8).reshape(o.n, -1), axis=1, bitorder="little")[:, :A]
    a = rs.integers(0, A, o.n).astype(np.int32)
    for i in range(o.n):
        nz = np.nonzero(m[i])[0]
        if nz.size:
            a[i] = nz[rs.integers(nz.size)]
    return a


@pytest.fixture(scope="module")
def emu_lib():
    subprocess.run(["make", "-C", EMU_DIR, "libwave_emu.so"], check=True, stdout=subprocess.DEVNULL)
    sys.path.insert(0, EMU_DIR)
    import emu
    return emu, emu.load()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("R,C,k,sm", SHAPES)
def test_spill_path_emulated(emu_lib, mode, R, C, k, sm):
    """The kernel source on the host wave emulator (CPU): step + spill_kernel vs the oracle."""
    from tile_match_gym_amd.seeding import batch_rng_words
    emu, L = emu_lib
    n = 4
    b = adversarial_boards(n, R, C, k, sm, 11, mode)
    words = batch_rng_words(range(300, 300 + n))
    e = emu.EmuBatch(L, R, C, k, sm, 30, words)
    o = orc.OracleBatch(R, C, k, sm, 30, words)
    e.board[:] = b
    o.board[:] = b
    e.trust = False
    s0 = L.emu_spills()
    rs = np.random.default_rng(5)
    a = effective_actions(b)
    for t in range(3):
        e.step(a)
        o.step(a)
        e.trust = True
        for f in ("board", "rng", "reward", "n_new", "n_act", "flags", "eff", "timer"):
            assert np.array_equal(getattr(e, f), getattr(o, f)), (t, f)
        a = _next_actions(o, rs)
    assert L.emu_status() == 0
    if (R, C) in ((20, 20), (10, 10)) and mode != "stripes":
        # 20x20: the 512-cell kernel's lists (spill_kernel<512>); 10x10: the
        # 128-cell general kernel's 64-cell lists (spill_kernel<128>)
        assert L.emu_spills() > s0, "the adversarial boards were meant to outgrow the LDS lists"


class _Vec:
    def __init__(self, env):
        self.env = env

    def __getattr__(self, f):
        if f == "rng":
            return self.env.rng_words()
        if f == "eff":
            return self.env.eff.cpu().numpy().view(np.uint64)
        return getattr(self.env, f).cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("R,C,k,sm", SHAPES)
def test_spill_path_gpu(R, C, k, sm):
    """Adversarial boards on the MI355X: every field equals the oracle at every
    step, the 20x20 ones go through spill_kernel, nothing is flagged."""
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    cl = ["cookie"] if sm & 1 else []
    co = [nm for bit, nm in ((8, "bomb"), (2, "vertical_laser"), (4, "horizontal_laser")) if sm & bit]
    per = 128
    b = np.concatenate([adversarial_boards(per, R, C, k, sm, 17 + i, m) for i, m in enumerate(MODES)])
    n = b.shape[0]
    env = TileMatchVecEnv(n, R, C, k, 30, cl, co, seed=900, device="cuda:0", groups=2)
    o = orc.OracleBatch(R, C, k, sm, 30, env.rng_words().copy(), threads=16)
    env.board.copy_(torch.from_numpy(b))
    o.board[:] = b
    env.invalidate_effective_cache()
    s0 = env.ctx.spills()
    rs = np.random.default_rng(9)
    a = effective_actions(b)
    for t in range(4):
        env.step(torch.from_numpy(a).to("cuda:0"))
        o.step(a, autoreset=True)
        v = _Vec(env)
        for f in ("board", "rng", "reward", "n_new", "n_act", "flags", "eff", "timer"):
            assert np.array_equal(getattr(v, f), getattr(o, f)), (t, f)
        a = _next_actions(o, rs)
    assert env.status() == 0
    if (R, C) in ((20, 20), (10, 10)):            # spill_kernel<512> / spill_kernel<128> re-ran steps
        assert env.ctx.spills() > s0


@pytest.mark.gpu
def test_spill_queue_holds_every_env_of_a_launch():
    """More envs outgrowing the LDS lists in one launch than round 2's fixed
    queue held (4096): the per-stream spill queue is sized by the host for the
    launch (tmg_capi.hip spill_for), so every one of them is re-run on the
    worst-case lists, bit-exact vs the oracle, and nothing is flagged (the
    reference's Python lists are unbounded, board.py:149-215, 269-327)."""
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    R, C, k, sm = 20, 20, 6, 15
    n = 6144
    b = adversarial_boards(n, R, C, k, sm, 3, "combo_grid")
    a = effective_actions(b)
    env = TileMatchVecEnv(n, R, C, k, 30, ["cookie"], ["vertical_laser", "horizontal_laser", "bomb"], seed=5,
                          device="cuda:0")
    o = orc.OracleBatch(R, C, k, sm, 30, env.rng_words().copy(), threads=16)
    env.board.copy_(torch.from_numpy(b))
    o.board[:] = b
    env.invalidate_effective_cache()
    s0 = env.ctx.spills()
    _, _, _, _, info = env.step(torch.from_numpy(a).to("cuda:0"))
    o.step(a, autoreset=True)
    spilled = env.ctx.spills() - s0
    assert spilled > 4096, f"only {spilled} envs of the launch outgrew the LDS lists"
    v = _Vec(env)
    for f in ("board", "rng", "reward", "n_new", "n_act", "flags", "eff", "timer"):
        assert np.array_equal(getattr(v, f), getattr(o, f)), f
    assert not info["overflow"].any() and not info["error"].any()
    assert env.status() == 0
