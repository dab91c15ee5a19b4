"""bench.py driver contract on the CPU: ``--gpus N`` outside a launcher re-runs itself as N ranks under
torch.distributed.run and rank 0 prints ONE JSON line whose n_gpus is N (dry-run mode: tiny SD2.1 config
over gloo -- the launcher / rendezvous / barrier / max-over-ranks plumbing, not a measurement)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [1, 2])
def test_bench_self_launch_reports_n_gpus(n):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "1",
                        "--warmup", "0", "--batch", "1", "--inference-steps", "2", "--latency-runs", "1",
                        "--cpu-dry-run"], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 1 and d["warmup"] == 0
    assert d["config"]["parallelism"] == f"dp{n}" and d["config"]["global_batch"] == n
    assert d["value"] > 0 and "DRY RUN" in d["data"]


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-dry-run"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)
