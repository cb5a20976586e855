"""Depth for the wave-parallel cascade steps (tmg_sb.hip sb_simple_step,
tmg_board.hip simple_step_lds / bomb_plan / the activation closure): large
rollouts of the c3 / c5 shapes and of 12x12 / 16x16 boards on the product
library against the CPU oracle, every field of every env at every step, and a
TMG_COVER diagnostic run of the very same trajectories that shows each step
form was taken at least 100 times (tests/deep_rollouts.py).

Reference: board.py:269-327 (process_colour_lines), :429-458
(get_special_creation_pos), :473-556 (activate_special), :600-719
(combination_match)."""
import json
import os

import numpy as np
import pytest

from deep_rollouts import CONFIGS, COVER_LIB, cover_counts, run

pytestmark = pytest.mark.gpu


FIELDS = ("board", "rng", "timer", "eff", "reward", "n_new", "n_act", "flags")


def _host(env, f):
    if f == "rng":
        return env.rng_words()
    v = getattr(env, f).cpu().numpy()
    return v.view(np.uint64) if f == "eff" else v


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_deep_rollout_vs_oracle(name):
    """Every env, every step, every field equal to the oracle."""
    def check(t, env, ref):
        for f in FIELDS:
            got, want = _host(env, f), getattr(ref, f)
            if not np.array_equal(got, want):
                n = got.shape[0]
                bad = np.nonzero((got.reshape(n, -1) != want.reshape(n, -1)).any(axis=1))[0]
                raise AssertionError(f"{name} step {t}: {f} differs in {bad.size} envs, first {bad[:5]}")
    env = run(name, check=check)
    assert env.status() == 0
    env.close()


# Branches each group of configurations must take >= MIN_HITS times (CV_* names,
# _native.COVER_NAMES).  Bitboard path (<= 128 cells with specials) and the
# 512-cell LDS path.
MIN_HITS = 100
REQUIRED = {
    ("c3_uniform", "c3_effective", "c3_cookie_effective"): (
        "sb_normal", "sb_laser", "sb_perp_bomb", "sb_row_bomb", "sb_closure", "sb_fallback", "serial_step",
        "serial_act", "combo"),
    ("c5_uniform", "c5_effective", "s12_effective", "s16_effective"): (
        "lds_normal", "lds_laser", "lds_bomb", "lds_fallback", "serial_step", "serial_act", "serial_cookie",
        "combo"),
}
# Natural rollouts never outgrow the LDS lists, so the spill tier is driven by
# the adversarial boards of tests/test_overflow.py instead (> 4096 spills in
# one launch, asserted there).


def test_cascade_branch_coverage():
    """The TMG_COVER build (loaded beside the product library, its own
    contexts and kernels) on the same trajectories: per-branch hit counts."""
    assert os.path.exists(COVER_LIB), "build() makes libtmg_cover.so"
    res = cover_counts()
    keep = os.environ.get("TMG_COVER_OUT")
    if keep:
        with open(keep, "w") as f:
            json.dump(res, f, indent=1)
    assert res["build"]["variant"] == "cover"
    for names, branches in REQUIRED.items():
        tot = {b: sum(res["configs"][n]["counts"][b] for n in names) for b in branches}
        low = {b: v for b, v in tot.items() if v < MIN_HITS}
        assert not low, f"{names}: branches below {MIN_HITS} hits: {low}"
    for n, c in res["configs"].items():
        assert c["status"] == 0, (n, c["status"])
