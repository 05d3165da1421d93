"""bench.py's own N-rank launch (`--gpus N` without an external launcher), checked on the CPU with --rank-check:
the parent starts the ranks before any GPU call, they rendezvous (gloo here; nccl in the benchmark proper) and
rank 0's line reaches stdout.  A WORLD_SIZE that disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def test_gpus_n_spawns_n_ranks():
    for n in (2, 3):
        r = _run(["--gpus", str(n), "--rank-check"])
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout
        d = json.loads(lines[0])
        assert d["n_gpus"] == n and d["ranks_seen"] == n
        assert d["rank_sum"] == n * (n + 1) // 2 and d["local_rank"] == 0


def test_gpus_one_runs_in_process():
    r = _run(["--gpus", "1", "--rank-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d == {"n_gpus": 1, "ranks_seen": 1, "rank_sum": 1, "local_rank": 0}


def test_world_size_disagreeing_with_gpus_is_refused():
    r = _run(["--gpus", "4", "--rank-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "refusing" in r.stderr
