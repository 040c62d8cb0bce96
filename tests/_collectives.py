"""Runner + numpy expectations for tests/collectives_worker.py (shared by the gloo CPU test and the
RCCL GPU test). The expectations restate what each collective must return: the rank blocks in
rank order (all-gathers), the max / min over ranks (all-reduces), rank 0's values (broadcast), the
table rows (sharded load), and the merge's (score desc, id asc) order over the world * k
candidates of each user (merge_topk / merge_topk_f64)."""
import os
import socket
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "collectives_worker.py")
sys.path.insert(0, os.path.join(ROOT, "tests"))
import collectives_worker as cw  # noqa: E402


def run(world, backend, out, timeout=240):
    """Start the worker as a fresh child: torch.distributed.run, `world` ranks, 127.0.0.1."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), WORKER, "--backend", backend,
           "--out", out]
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.setdefault("OMP_NUM_THREADS", "1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return dict(np.load(out))


def expected(world):
    blocks = [cw.rank_block(r, world) for r in range(world)]
    ids, sc, ids64, keys, short = (np.stack([b[i] for b in blocks]) for i in range(5))
    e = {"packed_ids": short, "packed_scores": sc, "wide_ids": short, "wide_scores": sc,
         "f64_ids": ids64, "f64_keys": keys, "merge_in_ids": ids, "merge_in_scores": sc}
    e["f64_rows"] = np.array([[r + 0.1, 1.0 / 3.0, 1e300, -0.0, float(world), 2.0 ** -1074]
                              for r in range(world)])
    gs = []
    for r in range(world):
        g = np.random.default_rng(7 + r).random(cw.N_USERS) * (r + 1)
        g[0] = 0.0
        gs.append(g)
    e["gmax_bits"] = np.max(np.stack(gs), axis=0).view(np.int64)
    e["agree_min"] = np.array(5)
    torch.manual_seed(0)
    m = torch.nn.Module()
    m.embed_history = torch.nn.Embedding(cw.P_ROWS, cw.D_ROWS)
    m.embed_target = torch.nn.Embedding(cw.P_ROWS, cw.D_ROWS)
    m.attn_layer1 = torch.nn.Linear(cw.D_ROWS, 4)
    e["broadcast_w1"] = m.attn_layer1.weight.detach().numpy()
    full = np.arange(cw.P_ROWS * cw.D_ROWS, dtype=np.float32).reshape(cw.P_ROWS, cw.D_ROWS)
    e["tables_h"], e["tables_t"], e["rows"] = full, 2 * full, full + 1
    e["gather_ids"] = np.stack([np.arange(cw.K) + 10 * u for u in range(cw.N_USERS)]).astype(np.int64)
    e["gather_scores"] = np.stack([np.full(cw.K, u / 10.0) for u in range(cw.N_USERS)]).astype(np.float32)
    mi, ms, fi, fs = [], [], [], []
    for u in range(cw.N_USERS):
        ci, cs = ids[:, u].reshape(-1), sc[:, u].reshape(-1)
        o = np.lexsort((ci, -cs))[:cw.K]
        mi.append(ci[o])
        ms.append(cs[o])
        ci, ck = ids64[:, u].reshape(-1), keys[:, u].reshape(-1)
        o = np.lexsort((ci, -ck))[:cw.K]
        fi.append(ci[o])
        fs.append(ck[o].astype(np.float32))
    e["merge_ids"], e["merge_scores"] = np.array(mi), np.array(ms)
    e["merge64_ids"], e["merge64_scores"] = np.array(fi), np.array(fs)
    return e


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint8) if a.dtype.kind in "fiu" else a


def assert_matches_expected(res, world, device_merges):
    exp = expected(world)
    names = [k for k in exp if device_merges or not k.startswith(("merge_ids", "merge_scores", "merge64"))]
    for k in names:
        got, want = np.asarray(res[k]), np.asarray(exp[k])
        assert got.shape == want.shape and got.dtype == want.dtype, (k, got.shape, want.shape, got.dtype, want.dtype)
        assert np.array_equal(bits(got), bits(want)), (k, got, want)
    return names
