"""bench.py's launcher contract (no GPU): `--gpus N` either runs under a launcher whose WORLD_SIZE is
N, or (no launcher) spawns N rank processes itself; any other world is refused before a GPU is
touched (`--gpus 8` without torchrun used to measure one GPU)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=300)


def test_world_mismatch_is_refused():
    r = run(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr
    r = run(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0


def test_no_launcher_spawns_n_ranks():
    r = run(["--gpus", "3", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["launch_check"] == {"world": 3, "ranks": [0, 1, 2]}
