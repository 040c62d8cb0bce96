"""The N > 1 bench path on the GPU: the code the driver's first multi-GPU run
executes -- bench.py's self-launch through torch.distributed.run, the process-group init, the
column-sharded pairs job (sharding.distributed_topk_pairs: per-rank tables and gathers, one
all_gather_into_tensor of the [users, 50] blocks, the merge) and the per_rank record -- run as a
fresh child process with 2 ranks on this box's one GPU over gloo (RCCL needs one GPU per rank) on
a small workload. The test process only starts the child and reads its JSON line (no exec)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_one_json_line():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--num-users", "2000", "--num-pois", "20000", "--steps", "3", "--warmup", "1",
           "--no-fp32-leg", "--no-gather-leg", "--no-train-leg", "--no-cpu-baseline"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    print({k: d[k] for k in ("value", "ms_per_step", "n_gpus", "world_size", "backend")})
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["backend"] == "gloo"
    assert d["steps"] == 3 and d["value"] > 0
    pr = d["per_rank"]
    print(pr["ms_per_step_by_rank"])
    assert pr["world_size_reported"] == 2 and pr["backend"] == "gloo"
    assert list(pr["phases"]) == ["table", "gather", "allgather", "merge", "topk", "wall"]
    rows = pr["ms_per_step_by_rank"]
    assert len(rows) == 2
    for row in rows:             # every phase timed on both ranks
        assert len(row) == 6
        table, gather, allgather, merge, topk, wall = row
        assert table > 0 and gather > 0 and allgather > 0 and merge > 0 and wall > 0
        assert topk >= 0
    sc = d["self_check"]
    assert sc is not None and sc["topk_ok"], sc
