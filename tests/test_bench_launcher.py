"""bench.py's multi-GPU launch path on CPU (gloo, --dry-run: no GPU, no
verification): `python bench.py --gpus N` must start N ranks itself, give
them disjoint contiguous shards, take the max over ranks and print exactly
one JSON line whose n_gpus counts the ranks that ran."""
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
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("gpus", [1, 2])
def test_launcher_weak_scaling(gpus):
    n = 4096
    r = _run(["--gpus", str(gpus), "--dry-run", "--n", str(n), "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["n_gpus"] == gpus and j["scaling"] == "weak" and j["dry_run"]
    shards = j["shards"]
    assert [s[0] for s in shards] == list(range(gpus))
    assert shards[0][1] == 0 and shards[-1][2] == n * gpus
    assert all(a[2] == b[1] for a, b in zip(shards, shards[1:]))     # contiguous, disjoint
    assert j["gathered_items"] == n * gpus and j["value"] > 0


def test_launcher_strong_scaling_global_n():
    r = _run(["--gpus", "2", "--dry-run", "--global-n", "10000", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    (j,) = _json_lines(r.stdout)
    assert j["scaling"] == "strong" and j["config"]["global_batch"] == 10000
    assert [s[2] - s[1] for s in j["shards"]] == [5000, 5000]


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
