"""The oracle driven with the Gymnasium vector-env autoreset semantics of
tmg_plan_config (test infrastructure): per step the expected state and the
per-env outputs the step kernels write — terminated / combo / shuffled /
error bytes, action-mask bytes, moves left and (same step) final boards."""
import numpy as np

from oracle import oracle as orc


def reset_subset(o, idx):
    """OracleBatch has no masked reset: regenerate the envs `idx` through a sub-batch
    (their own streams, continued: reset() without a seed)."""
    if len(idx) == 0:
        return
    sub = orc.OracleBatch(o.R, o.C, o.k, o.smask, o.num_moves, o.rng[idx].copy())
    sub.reset()
    o.board[idx], o.rng[idx], o.timer[idx], o.eff[idx] = sub.board, sub.rng, sub.timer, sub.eff


def mask_bytes(eff, A):
    n = eff.shape[0]
    return np.unpackbits(eff.view(np.uint8).reshape(n, -1), axis=1, bitorder="little")[:, :A].astype(np.uint8)


class VectorOracle:
    """mode "next_step" (an env that ended last step is reset instead of stepped)
    or "same_step" (an ending env is reset in the same step; final boards kept)."""

    def __init__(self, o, mode):
        self.o, self.mode = o, mode
        self.A = 2 * o.R * o.C - o.R - o.C
        self.pending = np.zeros(o.board.shape[0], bool)

    def step(self, a):
        o = self.o
        o.step(a, autoreset=False)            # pending envs: step-after-done error, state untouched
        live = ~self.pending if self.mode == "next_step" else np.ones_like(self.pending)
        f = o.flags
        out = {"terminated": np.stack([(f & 1) != 0, (f & 2) != 0, (f & 4) != 0, (f & 0xC0) != 0], 1)
               & live[:, None],
               "reward": np.where(live, o.reward, 0), "n_new": np.where(live, o.n_new, 0),
               "n_act": np.where(live, o.n_act, 0)}
        term = out["terminated"][:, 0]
        if self.mode == "next_step":
            reset_subset(o, np.nonzero(self.pending)[0])
            self.pending = term.copy()
        else:
            out["final_board"] = o.board.copy()
            reset_subset(o, np.nonzero(term)[0])
        out["action_mask"] = mask_bytes(o.eff, self.A)
        out["moves_left"] = (o.num_moves - o.timer).astype(np.int64)
        out["terminated"] = out["terminated"].astype(np.uint8)
        return out
