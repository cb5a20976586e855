"""The N > 1 path on the kernels: independent env shards,
one process per rank, no collective on the data path.  On a one-GPU box every
rank uses cuda:0; the trajectories cannot depend on that (seeds and actions
are functions of the global env index, tile_match_env.py:49-50).

Set TMG_EVIDENCE_DIR to keep the child processes' output (profiles/)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _keep(name, text):
    d = os.environ.get("TMG_EVIDENCE_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name), "w") as f:
            f.write(text)


def test_bench_two_ranks():
    """`bench.py --gpus 2` launches its own two rank processes, each stepping
    its shard on the device, and rank 0 prints the n_gpus = 2 line."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--boards", "4096", "--steps", "30",
           "--warmup", "5", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, timeout=300, capture_output=True, text=True)
    _keep("bench_gpus2.log", " ".join(cmd) + "\n" + r.stdout + r.stderr)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["steps"] == 30
    assert out["config"]["boards_per_gpu"] == 4096


@pytest.mark.parametrize("cfg", [(10, 10, 4, 0, 1536, 40, "uniform"), (10, 10, 4, 14, 1024, 40, "effective"),
                                 (20, 20, 6, 15, 256, 35, "uniform")])
def test_gloo_ranks_step_shards_on_device(cfg):
    """World size 2 over gloo, each rank a fresh process stepping
    TileMatchVecEnv on the device; the all-gathered shards equal the
    single-process oracle over the whole env range, bit for bit."""
    R, C, k, sm, per, steps, policy = cfg
    world, port = 2, _port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                   LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_shard_run.py"),
                                       str(R), str(C), str(k), str(sm), str(per), str(steps), policy],
                                      cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    _keep(f"gloo_shards_{R}x{C}_{sm}_{policy}.log", "\n".join(o + e for _, o, e in outs))
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
    res = [json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]) for _, o, _ in outs]
    r0 = [x for x in res if x["rank"] == 0][0]
    assert r0["envs_total"] == world * per
    assert r0["equal"], r0["mismatches"]
    assert all(x["status"] == 0 for x in res)
    assert sorted(tuple(x["envs"]) for x in res) == [(0, per), (per, 2 * per)]
