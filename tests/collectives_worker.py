"""One rank of every collective the N > 1 path issues (sharding.py), on
deterministic rank-dependent data, with the results written by rank 0 to --out (npz).

Started under torch.distributed.run (never imported by pytest): with `--backend nccl` the tensors
live on the rank's GPU and the calls run on RCCL; with `--backend gloo` they stay on the CPU.
tests/test_gpu_rccl.py runs it at world size 1 both ways on the GPU box and requires the two
result files to be bit-identical (and the device merges to equal their numpy restatement);
tests/test_sharding_gloo.py runs the gloo form at world sizes 2 and 3 and checks every result
against numpy.

Calls, in order (each one is what the product issues, not a stand-in):
  exchange_blocks  -- the column-sharded merge's packed (int32 id, f32 score bits) all-gather,
                      its int64 + f32 form (catalogs of >= 2^31 POIs) and the prior route's f64 keys
  all_gather_cat   -- a float64 row (bench.py's per_rank record)
  allreduce_gmax   -- int64 MAX over the bit patterns of non-negative doubles
  agree_min        -- int64 MIN
  broadcast_module -- parameters from rank 0
  load_sharded_tables / allgather_rows -- P = 1001 rows, not divisible by 2 or 3
  gather_topk      -- the user-sharded route's padded [n_r, k] blocks
  merge_topk / merge_topk_f64 (device only: nais_topk_rows / nais_topk_merge_f64 on the blocks)
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

N_USERS, K, P_COLS, P_ROWS, D_ROWS = 9, 6, 600, 1001, 8


def rank_block(rank, world):
    """This rank's [N_USERS, K] top-k blocks over its column range: (ids, f32 scores) in (score
    desc, id asc) order with ties within and across ranks (scores on a coarse grid), (ids64, f64
    keys) in (key desc, id asc) order, and the f32 ids with one short list (-1 ids) for the
    exchange round trip."""
    from poi_recommendation_models_amd.sharding import column_blocks
    c0, c1 = column_blocks(P_COLS, world)[rank]
    rng = np.random.default_rng(1000 + rank)
    ids = np.empty((N_USERS, K), np.int64)
    sc = np.empty((N_USERS, K), np.float32)
    keys = np.empty((N_USERS, K), np.float64)
    ids64 = np.empty((N_USERS, K), np.int64)
    for u in range(N_USERS):
        cand = rng.choice(np.arange(c0, c1), K, replace=False)
        s = (rng.integers(0, 8, K) / 8.0).astype(np.float32)        # ties within and across ranks
        kk = rng.integers(0, 8, K) / 8.0 + 1e-12 * rng.random(K)
        o = np.lexsort((cand, -s))
        ids[u], sc[u] = cand[o], s[o]
        o64 = np.lexsort((cand, -kk))
        ids64[u], keys[u] = cand[o64], kk[o64]
    short = ids.copy()
    short[-1, K // 2:] = -1
    return ids, sc, ids64, keys, short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", choices=["nccl", "gloo"], required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if a.backend == "nccl":
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
    else:
        dev = torch.device("cpu")
        dist.init_process_group("gloo")
    from poi_recommendation_models_amd import sharding as sh

    res = {"world": np.array(world), "backend": np.array(a.backend)}
    ids, sc, ids64, keys, short = rank_block(rank, world)
    T = lambda x: torch.as_tensor(x, device=dev)
    gi, gk = sh.exchange_blocks(T(short), T(sc), wide_ids=False)
    res["packed_ids"], res["packed_scores"] = gi.cpu().numpy(), gk.cpu().numpy()
    gi_w, gk_w = sh.exchange_blocks(T(short), T(sc), wide_ids=True)
    res["wide_ids"], res["wide_scores"] = gi_w.cpu().numpy(), gk_w.cpu().numpy()
    gi64, gk64 = sh.exchange_blocks(T(ids64), T(keys))
    res["f64_ids"], res["f64_keys"] = gi64.cpu().numpy(), gk64.cpu().numpy()

    row = torch.tensor([rank + 0.1, 1.0 / 3.0, 1e300, -0.0, float(world), 2.0 ** -1074],
                       dtype=torch.float64, device=dev)
    res["f64_rows"] = sh.all_gather_cat(row[None, :]).cpu().numpy()

    g = np.random.default_rng(7 + rank).random(N_USERS) * (rank + 1)
    g[0] = 0.0
    bits = T(g.view(np.int64).copy())
    res["gmax_bits"] = sh.allreduce_gmax(bits).cpu().numpy()
    res["agree_min"] = np.array(sh.agree_min(5 + 3 * (world - 1 - rank), dev))

    torch.manual_seed(rank)                  # ranks start from different weights
    m = torch.nn.Module()
    m.embed_history = torch.nn.Embedding(P_ROWS, D_ROWS)
    m.embed_target = torch.nn.Embedding(P_ROWS, D_ROWS)
    m.attn_layer1 = torch.nn.Linear(D_ROWS, 4)
    m.attn_layer2 = torch.nn.Linear(4, 1, bias=False)
    m = m.to(dev)
    sh.broadcast_module(m)
    res["broadcast_w1"] = m.attn_layer1.weight.detach().cpu().numpy()
    full = torch.arange(P_ROWS * D_ROWS, dtype=torch.float32).reshape(P_ROWS, D_ROWS)
    sh.load_sharded_tables(m, lambda name, s, e: full[s:e] * (2 if name == "embed_target" else 1))
    res["tables_h"] = m.embed_history.weight.detach().cpu().numpy()
    res["tables_t"] = m.embed_target.weight.detach().cpu().numpy()
    s0, e0 = sh.row_block(P_ROWS, rank, world)
    res["rows"] = sh.allgather_rows(T(full[s0:e0].numpy()) + 1, P_ROWS).cpu().numpy()

    hl = np.arange(N_USERS) % 4 + 1
    mine = sh.shard_users(hl, P_COLS, world)[rank]
    li = T(np.stack([np.arange(K) + 10 * u for u in mine]).reshape(-1, K).astype(np.int64))
    ls = T(np.stack([np.full(K, u / 10.0) for u in mine]).reshape(-1, K).astype(np.float32))
    ui, us = sh.gather_topk(mine, li, ls, N_USERS)
    res["gather_ids"], res["gather_scores"] = ui.cpu().numpy(), us.cpu().numpy()

    gi_m, gk_m = sh.exchange_blocks(T(ids), T(sc))     # the merge input, as distributed_topk_pairs
    res["merge_in_ids"], res["merge_in_scores"] = gi_m.cpu().numpy(), gk_m.cpu().numpy()
    if dev.type == "cuda":
        mi, ms = sh.merge_topk(gi_m, gk_m, K)
        res["merge_ids"], res["merge_scores"] = mi.cpu().numpy(), ms.cpu().numpy()
        fi, fs = sh.merge_topk_f64(gi64, gk64, K)
        res["merge64_ids"], res["merge64_scores"] = fi.cpu().numpy(), fs.cpu().numpy()
        torch.cuda.synchronize(dev)
    dist.barrier()
    if rank == 0:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        np.savez(a.out, **res)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
