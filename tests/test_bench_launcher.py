"""bench.py's multi-rank launcher on the CPU: `--gpus N` outside torchrun starts the
N rank processes itself (replacing PMPC/main_parallel_enhanced.py:200-207's Process spawn), and a --gpus that
disagrees with torchrun's WORLD_SIZE is an error.  --plumbing-only runs the ranks' process group, timing and
C4 shard / gather without a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_the_ranks(n):
    p = _run(["--gpus", str(n), "--dist-backend", "gloo", "--plumbing-only"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout           # one JSON line, from rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == n
    c4 = line["pmpc_c4"]
    assert c4["n_gpus"] == n and c4["per_rank"] == -(-1152 // n)
    assert c4["rank_blocks_consistent"] and c4["gathered_equals_global_rows"]


def test_single_rank_default():
    p = _run(["--plumbing-only"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip())["n_gpus"] == 1


def test_gpus_disagreeing_with_world_size_fails():
    p = _run(["--gpus", "4", "--plumbing-only"], env_extra={"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr
