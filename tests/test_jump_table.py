"""The PCG64 jump-ahead table (csrc/pcg64.h build_jump_table), host side.

Rows 0..63 let lane j compute s_j = A^j s + G_j inc in one step, rows 64..71 take
the row-plane generate's lane-local batches back by 64m outputs (bp_ring_state,
m <= 6 since the redraw loop keeps fewer than N + 128 colours filled ahead).
Checked against the LCG itself, s' = s A + inc mod 2^128 (numpy's PCG64 state
step), for random states and increments.  The device multiply (jump128's
three-chain form) is checked by the GPU suite, which compares every env's RNG
words with the oracle after every step.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "tile-match-gym_amd", "csrc")

CHECK = r"""
#define __host__
#define __device__
#define __forceinline__ inline
#include "pcg64.h"
#include <cstdio>
#include <random>
using tmg::U128;
typedef unsigned __int128 u128;
static u128 w(U128 x) { return ((u128)x.hi << 64) | x.lo; }
int main() {
    uint64_t tab[tmg::kJumpRows * 4];
    tmg::build_jump_table(tab);
    const u128 A = ((u128)tmg::PCG_A_HI << 64) | tmg::PCG_A_LO;
    std::mt19937_64 rng(12345);
    for (int trial = 0; trial < 200; trial++) {
        const u128 s0 = ((u128)rng() << 64) | rng();
        const u128 inc = (((u128)rng() << 64) | rng()) | 1;      // numpy's increments are odd
        u128 s = s0;
        for (int j = 1; j <= 64 * 8; j++) {
            s = s * A + inc;
            if (j <= 64) {
                const u128 Aj = ((u128)tab[(j - 1) * 4 + 1] << 64) | tab[(j - 1) * 4];
                const u128 Gj = ((u128)tab[(j - 1) * 4 + 3] << 64) | tab[(j - 1) * 4 + 2];
                if (Aj * s0 + Gj * inc != s) { printf("forward row %d\n", j - 1); return 1; }
                if (w(tmg::jump128(U128{(uint64_t)Aj, (uint64_t)(Aj >> 64)}, U128{(uint64_t)s0, (uint64_t)(s0 >> 64)},
                                   U128{(uint64_t)(Gj * inc), (uint64_t)((Gj * inc) >> 64)})) != s) {
                    printf("jump128 row %d\n", j - 1); return 1;
                }
            }
            if (j % 64 == 0) {
                const int m = j / 64, r = 63 + m;
                const u128 B = ((u128)tab[r * 4 + 1] << 64) | tab[r * 4];
                const u128 D = ((u128)tab[r * 4 + 3] << 64) | tab[r * 4 + 2];
                if (B * s + D * inc != s0) { printf("backward m=%d\n", m); return 1; }
            }
        }
    }
    printf("ok\n");
    return 0;
}
"""


def test_jump_table_forward_and_backward_rows(tmp_path):
    src = tmp_path / "jt.cpp"
    src.write_text(CHECK)
    exe = tmp_path / "jt"
    try:
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", CSRC, "-o", str(exe), str(src)], check=True,
                       capture_output=True, text=True, timeout=120)
    except FileNotFoundError:
        pytest.skip("no g++")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr
