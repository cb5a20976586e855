"""CPU checks of bench.py's launcher and workload definition (no GPU)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_n_spawns_one_rank_per_gpu():
    """`bench.py --gpus N` without a launcher starts N rank processes with the
    torch.distributed.run environment; each owns its contiguous shard
    (shard.shard_range: weak scaling, fixed boards per GPU)."""
    from tile_match_gym_amd.shard import shard_range
    for n in (2, 4):
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run",
                              "--boards", "1000"], capture_output=True, text=True, timeout=300,
                             env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")})
        assert out.returncode == 0, out.stderr
        lines = sorted((json.loads(l) for l in out.stdout.split("\n") if l.strip()), key=lambda d: d["rank"])
        assert [d["rank"] for d in lines] == list(range(n))
        for d in lines:
            assert d["world"] == n and d["local_rank"] == d["rank"]
            r = shard_range(d["rank"], 1000)
            assert d["envs"] == [r.start, r.stop]


def test_staggered_phase_is_ineffective_moves():
    """bench's phase stagger (timer0 = env mod num_moves) is exactly the state
    after that many ineffective moves (board.py:352-353: no board or RNG
    change; tile_match_env.py:100: the timer counts the move), checked on the
    oracle for a few envs."""
    from oracle import oracle as orc
    from tile_match_gym_amd.seeding import batch_rng_words
    R, C, k, smask, moves = 10, 10, 4, 0, 30
    for e in (0, 1, 7, 29, 31):
        m = e % moves
        a = orc.OracleBatch(R, C, k, smask, moves, batch_rng_words([e]))
        a.reset()
        b = orc.OracleBatch(R, C, k, smask, moves, batch_rng_words([e]))
        b.reset()
        a.timer[:] = m
        for _ in range(m):
            bits = np.unpackbits(b.eff[0].view(np.uint8), bitorder="little")[:b.A]
            act = int(np.nonzero(bits == 0)[0][0])
            b.step(np.array([act], np.int32), autoreset=True)
            assert b.reward[0] == 0
        for x, y in ((a.board, b.board), (a.rng, b.rng), (a.timer, b.timer), (a.eff, b.eff)):
            assert np.array_equal(x, y)
        acts = np.array([5], np.int32)
        for _ in range(40):                                  # and the two stay equal afterwards
            a.step(acts, autoreset=True)
            b.step(acts, autoreset=True)
            assert np.array_equal(a.board, b.board) and np.array_equal(a.rng, b.rng)
            acts = (acts * 37 + 11) % a.A
