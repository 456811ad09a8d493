"""bench.py's multi-rank launcher (`--gpus N` must run N ranks, or refuse).

`python bench.py --gpus 2 --dry-run` with no WORLD_SIZE in the environment: the parent starts
two rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set), they join a gloo
group, run the barrier + max-over-ranks timing, the sweep exchange (all_gather of the best
(F, id) and the winner's broadcast) and the C4 strong-scaling leg's sharded exchange, and rank 0
prints one line.  The dry run replaces the evaluation by a placeholder score (cos-sum of x) so
that the exchange has a known winner; no GPU is touched.
"""
import json
import math
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["MASTER_ADDR"] = "127.0.0.1"
    env.update(extra)
    return env


def _scores(first, count, nt=512):
    out = []
    for r in range(first, first + count):
        rng = np.random.default_rng(1000 + r)
        x = np.concatenate([2 * math.pi * 0.001 * rng.uniform(size=nt), [2 * math.pi * rng.uniform()]])
        out.append(np.sum(np.cos(x)))
    return np.array(out)


def _lines(stdout):
    return [json.loads(line) for line in stdout.splitlines() if line.startswith("{")]


def test_gpus_2_spawns_two_ranks_and_runs_the_exchange():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--batch", "8", "--c4-total", "12"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == 2 and out["dry_run"] is True
    # weak leg: 8 restarts per rank, 16 in all; the winner is the global argmax (smallest id on ties)
    s = _scores(0, 16)
    assert out["sweep"]["restart"] == int(np.argmax(s))
    assert out["sweep"]["owner_rank"] == int(np.argmax(s)) // 8
    assert abs(out["sweep"]["best_F"] - s.max()) < 1e-12
    # strong leg: 12 restarts sharded 6 + 6 over the two ranks, exchange inside the timing
    c4 = out["c4_strong"]
    assert c4["n_gpus"] == 2 and c4["restarts_total"] == 12 and c4["restarts_per_rank"] == 6
    s = _scores(0, 12)
    assert c4["sweep"]["restart"] == int(np.argmax(s))
    assert c4["sweep"]["owner_rank"] == int(np.argmax(s)) // 6


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2
    assert "refusing" in r.stderr
    assert not _lines(r.stdout)


def test_single_rank_dry_run_has_no_process_group():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--batch", "4",
                        "--c4-total", "5"], env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _lines(r.stdout)[0]
    assert out["n_gpus"] == 1
    assert out["sweep"]["restart"] == int(np.argmax(_scores(0, 4)))
    assert out["c4_strong"]["restarts_per_rank"] == 5
