"""ctypes wrapper around oracle/liboracle_tmg.so — the CPU restatement of the
reference Board (see tmg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product (tile_match_gym_amd) never imports
this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_tmg.so")
_lib = None

P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or \
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "tmg_oracle.c")):
        subprocess.run(["make", "-C", _HERE, "-B" if force else "all"], check=True,
                       stdout=subprocess.DEVNULL)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        sig = {
            "orc_get_colour_lines": [I, I, I, I, P, P, P, I, I],
            "orc_process_lines": [I, I, I, I, P, P, P, P, P, I, I],
            "orc_effective_mask": [I, I, P, P],
            "orc_gravity": [I, I, P],
            "orc_activate": [I, I, I, I, P, I, I, P],
            "orc_combination": [I, I, I, I, P, I, P],
            "orc_detect_resolve": [I, I, I, I, P, P, P],
            "orc_move": [I, I, I, I, P, P, I, P],
            "orc_generate": [I, I, I, I, P, P],
            "orc_rng_colours": [P, I, I, P],
            "orc_rng_shuffle": [P, I, P],
            "orc_env_reset_batch": [I, I, I, I, I64, P, P, P, P, I],
            "orc_env_step_batch": [I, I, I, I, I, I64, P, P, P, P, P, P, P, P, P, I, I],
            "orc_count_states": [I, I, I, I, P, P],
        }
        for name, args in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = I
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def num_actions(R, C):
    return 2 * R * C - R - C


def get_colour_lines(board, k=4, smask=15):
    b = np.ascontiguousarray(board, dtype=np.int8)
    R, C = b.shape[1:]
    lens = np.zeros(8 * R * C, np.int16)
    cells = np.zeros(64 * R * C, np.int16)
    n = lib().orc_get_colour_lines(R, C, k, smask, _p(b), _p(lens), _p(cells), lens.size, cells.size)
    assert n >= 0
    out, o = [], 0
    for i in range(n):
        out.append([(int(x) // C, int(x) % C) for x in cells[o:o + lens[i]]])
        o += lens[i]
    return out


def process_lines(board, k=4, smask=15):
    b = np.ascontiguousarray(board, dtype=np.int8)
    R, C = b.shape[1:]
    lens = np.zeros(8 * R * C, np.int16)
    cells = np.zeros(64 * R * C, np.int16)
    names = np.zeros(8 * R * C, np.int8)
    cols = np.zeros(8 * R * C, np.int8)
    n = lib().orc_process_lines(R, C, k, smask, _p(b), _p(lens), _p(cells), _p(names), _p(cols), lens.size, cells.size)
    assert n >= 0
    out, o = [], 0
    for i in range(n):
        out.append([int(x) for x in cells[o:o + lens[i]]])
        o += lens[i]
    return out, names[:n].copy(), cols[:n].copy()


def effective_mask(board):
    b = np.ascontiguousarray(board, dtype=np.int8)
    R, C = b.shape[1:]
    m = np.zeros(num_actions(R, C), np.uint8)
    any_ = lib().orc_effective_mask(R, C, _p(b), _p(m))
    return m.astype(bool), bool(any_)


def gravity(board):
    b = np.ascontiguousarray(board, dtype=np.int8).copy()
    lib().orc_gravity(b.shape[1], b.shape[2], _p(b))
    return b


def activate(board, cell, combo, k=4, smask=15):
    b = np.ascontiguousarray(board, dtype=np.int8).copy()
    na = np.zeros(1, np.int32)
    err = lib().orc_activate(b.shape[1], b.shape[2], k, smask, _p(b), int(cell), int(combo), _p(na))
    return b, int(na[0]), err


def combination(board, action, k=4, smask=15):
    b = np.ascontiguousarray(board, dtype=np.int8).copy()
    na = np.zeros(1, np.int32)
    err = lib().orc_combination(b.shape[1], b.shape[2], k, smask, _p(b), int(action), _p(na))
    return b, int(na[0]), err


def detect_resolve(board, k=4, smask=15):
    b = np.ascontiguousarray(board, dtype=np.int8).copy()
    na = np.zeros(1, np.int32)
    nn = np.zeros(1, np.int32)
    err = lib().orc_detect_resolve(b.shape[1], b.shape[2], k, smask, _p(b), _p(na), _p(nn))
    return b, int(na[0]), int(nn[0]), err


def move(board, rng_words, action, k, smask):
    b = np.ascontiguousarray(board, dtype=np.int8).copy()
    rng = np.array(rng_words, dtype=np.uint64).copy()
    res = np.zeros(5, np.int32)
    err = lib().orc_move(b.shape[1], b.shape[2], k, smask, _p(b), _p(rng), int(action), _p(res))
    return b, rng, res, err


def generate(R, C, k, smask, rng_words):
    b = np.zeros((2, R, C), np.int8)
    rng = np.array(rng_words, dtype=np.uint64).copy()
    lib().orc_generate(R, C, k, smask, _p(b), _p(rng))
    return b, rng


def rng_colours(rng_words, k, n):
    rng = np.array(rng_words, dtype=np.uint64).copy()
    out = np.zeros(n, np.int32)
    lib().orc_rng_colours(_p(rng), k, n, _p(out))
    return out, rng


def rng_shuffle(rng_words, n):
    rng = np.array(rng_words, dtype=np.uint64).copy()
    out = np.zeros(n, np.int32)
    lib().orc_rng_shuffle(_p(rng), n, _p(out))
    return out, rng


def count_states(R, C, k, threads=8):
    """utils.compute_num_states restated (tmg_oracle.c): (playable, line_free)."""
    out = np.zeros(2, np.uint64)
    lib().orc_count_states(R, C, k, threads, out[0:].ctypes.data, out[1:].ctypes.data)
    return int(out[0]), int(out[1])


class OracleBatch:
    """Batched env state in numpy arrays, same layout as the device C-ABI (include/tmg.h)."""

    def __init__(self, R, C, k, smask, num_moves, rng_words: np.ndarray, threads: int = 1):
        self.R, self.C, self.k, self.smask, self.num_moves = R, C, k, smask, num_moves
        self.n = rng_words.shape[0]
        self.A = num_actions(R, C)
        self.W = (self.A + 63) // 64
        self.board = np.zeros((self.n, 2, R, C), np.int8)
        self.rng = np.ascontiguousarray(rng_words, dtype=np.uint64).copy()
        self.timer = np.zeros(self.n, np.int32)
        self.eff = np.zeros((self.n, self.W), np.uint64)
        self.reward = np.zeros(self.n, np.int32)
        self.n_new = np.zeros(self.n, np.int32)
        self.n_act = np.zeros(self.n, np.int32)
        self.flags = np.zeros(self.n, np.uint8)
        self.threads = threads

    def reset(self):
        lib().orc_env_reset_batch(self.R, self.C, self.k, self.smask, self.n, _p(self.board), _p(self.rng),
                                  _p(self.timer), _p(self.eff), self.threads)

    def step(self, actions, autoreset=True):
        a = np.ascontiguousarray(actions, dtype=np.int32)
        assert a.shape == (self.n,)
        lib().orc_env_step_batch(self.R, self.C, self.k, self.smask, self.num_moves, self.n, _p(self.board),
                                 _p(self.rng), _p(self.timer), _p(a), _p(self.reward), _p(self.n_new),
                                 _p(self.n_act), _p(self.flags), _p(self.eff), int(autoreset), self.threads)
