"""bench.py's self-launch: `python bench.py --gpus N` outside torchrun starts
N ranks itself before any GPU call, and each rank sees WORLD_SIZE == N.  Runs on the CPU through
`--spawn-check` (gloo, world 2: every rank all-reduces its rank number, rank 0 prints the line's
launch fields)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(env_extra or {})
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout + out.stderr
    return json.loads(lines[0])


def test_bench_spawns_two_ranks():
    r = _run(["--gpus", "2", "--spawn-check"])
    assert r.returncode == 0, r.stderr
    line = _line(r)
    assert line["n_gpus"] == 2 and line["ranks_sum"] == 3  # ranks 0 + 1, each counted as rank + 1
    assert line["scaling"] == "weak" and line["per_gpu_batch"] == 256 and line["global_batch"] == 512
    assert line["parallelism"].startswith("dp2 exact")


def test_bench_global_batch_is_strong_scaling():
    r = _run(["--gpus", "2", "--spawn-check", "--global-batch", "512"])
    assert r.returncode == 0, r.stderr
    line = _line(r)
    assert line["n_gpus"] == 2 and line["per_gpu_batch"] == 256 and line["scaling"] == "strong"


def test_bench_single_rank_label():
    r = _run(["--spawn-check"])
    assert r.returncode == 0, r.stderr
    line = _line(r)
    assert line["n_gpus"] == 1 and line["parallelism"] == "single GPU"


@pytest.mark.parametrize("args,env", [(["--gpus", "2", "--spawn-check"], {"WORLD_SIZE": "1"}),
                                      (["--gpus", "2", "--spawn-check", "--global-batch", "511"], {})])
def test_bench_rejects_inconsistent_world(args, env):
    r = _run(args, env)
    assert r.returncode != 0
