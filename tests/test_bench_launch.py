"""bench.py --gpus N without a launcher spawns N rank processes with the
torch.distributed.run environment (CPU only: the children here are a tiny
gloo job, not the GPU bench)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
import torch, torch.distributed as dist
dist.init_process_group("gloo", init_method="env://")
t = torch.tensor([int(os.environ["RANK"])], dtype=torch.int64)
dist.all_reduce(t)
env = {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
env["sum_of_ranks"] = int(t.item())
open(sys.argv[1] + "/rank%s.json" % env["RANK"], "w").write(json.dumps(env))
dist.destroy_process_group()
sys.exit(int(os.environ["RANK"]) == int(os.environ.get("FAIL_RANK", "-1")))
"""


def _spawn(n, tmp, fail_rank=None):
    sys.path.insert(0, ROOT)
    import bench
    env_before = dict(os.environ)
    if fail_rank is not None:
        os.environ["FAIL_RANK"] = str(fail_rank)
    try:
        return bench.spawn_ranks(n, [sys.executable, "-c", CHILD, str(tmp)], timeout=120)
    finally:
        os.environ.clear()
        os.environ.update(env_before)


def test_spawn_ranks_env_and_rendezvous(tmp_path):
    n = 3
    assert _spawn(n, tmp_path) == 0
    envs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(n)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert all(e["sum_of_ranks"] == 3 for e in envs)  # every rank joined the same job


def test_spawn_ranks_reports_a_failed_rank(tmp_path):
    assert _spawn(2, tmp_path, fail_rank=1) == 1


def test_bench_refuses_more_gpus_than_visible():
    # no GPU in this container: --gpus 2 must fail fast instead of running one rank
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert r.returncode == 2, r.stderr
    assert "GPU(s) visible" in r.stderr
