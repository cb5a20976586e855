"""Loaders for the golden fixtures in tests/golden/ (recorded from the reference
by tests/golden/make_goldens.py)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SHAPE_KEYS = ("R", "C", "k", "smask")


def load_records(name, prefix="fn"):
    """<prefix>_<name>.npz -> list of dict records (see make_goldens.pack_records).
    prefix "fn": random boards (make_goldens.py); "ref": the reference's own
    hand-built test boards (make_ref_cases.py)."""
    z = np.load(os.path.join(GOLDEN, f"{prefix}_{name}.npz"), allow_pickle=False)
    n = int(z["n"])
    keys = [k for k in z.files if k not in ("n",) and not k.endswith("_off")]
    recs = []
    for i in range(n):
        r = {}
        for k in keys:
            if k == "shape":
                r.update(dict(zip(SHAPE_KEYS, (int(x) for x in z["shape"][i]))))
            elif k + "_off" in z.files:
                o = z[k + "_off"]
                r[k] = z[k][o[i]:o[i + 1]]
            else:
                r[k] = z[k][i]
        R, C = r["R"], r["C"]
        for bk in ("board", "out"):
            if bk in r and r[bk].size == 2 * R * C:
                r[bk] = r[bk].reshape(2, R, C)
        recs.append(r)
    return recs


def load_traj(name):
    z = np.load(os.path.join(GOLDEN, f"traj_{name}.npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    R, C, k, smask, moves = (int(x) for x in d["shape"])
    d.update(R=R, C=C, k=k, smask=smask, num_moves=moves)
    A = 2 * R * C - R - C
    d["eff"] = np.unpackbits(d["eff"], axis=1)[:, :A].astype(bool)
    d["A"] = A
    return d


def traj_names():
    return sorted(f[5:-4] for f in os.listdir(GOLDEN) if f.startswith("traj_") and f.endswith(".npz"))


def eff_words_to_bool(words, A):
    w = np.asarray(words, dtype=np.uint64)
    bits = np.unpackbits(w.view(np.uint8).reshape(*w.shape[:-1], -1), axis=-1, bitorder="little")
    return bits[..., :A].astype(bool)


def traj_events(d):
    """Split a trajectory into per-env aligned event lists.  Returns
    (n_envs, n_events, idx[n_envs, n_events]) — every env has the same event
    structure (reset, num_moves steps, reset, ...)."""
    env = d["env"]
    n_env = int(env.max()) + 1
    idx = np.stack([np.nonzero(env == e)[0] for e in range(n_env)])
    kinds = d["kind"][idx]
    assert (kinds == kinds[0]).all(), "trajectory events are not aligned across envs"
    return n_env, idx


def replay_trajectory(d, backend, autoreset: bool):
    """Drive `backend` (reset()/step(actions, autoreset) with numpy-visible
    board/rng/timer/eff/reward/flags/n_new/n_act fields) through the recorded
    trajectory and compare every event with the reference's outputs.
    Returns the number of compared events."""
    n_env, idx = traj_events(d)
    kinds = d["kind"][idx[0]]
    A = d["A"]
    checked = 0

    def cmp_state(ev, what):
        b = backend.get_board()
        exp = d["board"][ev]
        bad = np.nonzero((b.reshape(n_env, -1) != exp.reshape(n_env, -1)).any(axis=1))[0]
        assert bad.size == 0, f"{what}: board mismatch in envs {bad[:8]} (event {ev[bad[0]]})"
        r = backend.get_rng()
        exp_r = d["rng"][ev]
        bad = np.nonzero((r != exp_r).any(axis=1))[0]
        assert bad.size == 0, f"{what}: rng state mismatch in envs {bad[:8]}"

    j = 0
    backend.reset()
    assert kinds[0] == 0
    ev = idx[:, 0]
    cmp_state(ev, "reset 0")
    assert np.array_equal(eff_words_to_bool(backend.get_eff(), A), d["eff"][ev]), "reset eff mask mismatch"
    checked += n_env
    j = 1
    while j < len(kinds):
        assert kinds[j] == 1
        ev = idx[:, j]
        acts = d["action"][ev].astype(np.int32)
        backend.step(acts, autoreset)
        fl = backend.get_flags()
        assert not (fl & 0x80).any(), "error flag raised"
        assert np.array_equal(backend.get_reward(), d["reward"][ev]), f"reward mismatch at event {j}"
        assert np.array_equal(backend.get_n_new(), d["n_new"][ev]), f"n_new mismatch at event {j}"
        assert np.array_equal(backend.get_n_act(), d["n_act"][ev]), f"n_act mismatch at event {j}"
        assert np.array_equal(fl & 7, d["flags"][ev]), f"flags mismatch at event {j}"
        done = bool(d["flags"][ev][0] & 1)
        has_reset = done and j + 1 < len(kinds) and kinds[j + 1] == 0
        if done and autoreset and has_reset:
            ev2 = idx[:, j + 1]
            cmp_state(ev2, f"autoreset after event {j}")
            assert np.array_equal(eff_words_to_bool(backend.get_eff(), A), d["eff"][ev2])
            j += 2
            checked += 2 * n_env
            continue
        if not (done and autoreset):
            cmp_state(ev, f"step event {j}")
            assert np.array_equal(eff_words_to_bool(backend.get_eff(), A), d["eff"][ev]), f"eff mismatch at event {j}"
        checked += n_env
        j += 1
        if has_reset and not autoreset:
            backend.reset()
            ev2 = idx[:, j]
            cmp_state(ev2, f"reset event {j}")
            assert np.array_equal(eff_words_to_bool(backend.get_eff(), A), d["eff"][ev2])
            checked += n_env
            j += 1
    return checked
