"""User-sharded multi-GPU evaluation.

One process per GPU. Users are independent units (validation.py:11-27 has no cross-user state),
so the path shards with no collective inside the scoring loop:

1. `broadcast_module`   -- the POI tables + MLP are replicated once from rank 0 (RCCL broadcast
                           over xGMI; `nccl` is RCCL on ROCm).
2. `shard_users`        -- LPT on the per-user cost (P - h_u) * h_u, so ranks finish together.
3. each rank runs `catalog.score_topk` on its users.
4. `gather_topk`        -- one all_gather of the [users_r, k] id/score blocks, reassembled in user
                           order (the reference's recommended_list, validation.py:27).
Works with any torch.distributed backend (gloo on CPU for the tests, nccl/RCCL on the GPUs).
"""
from __future__ import annotations

import heapq

import numpy as np
import torch


def shard_users(hist_len, num_pois, world, users=None):
    """LPT assignment: heaviest remaining user to the least-loaded rank. Returns one sorted
    int64 array of user ids per rank."""
    hist_len = np.asarray(hist_len, dtype=np.int64)
    users = np.arange(len(hist_len)) if users is None else np.asarray(users, dtype=np.int64)
    cost = (num_pois - hist_len[users]) * hist_len[users]
    order = users[np.argsort(-cost, kind="stable")]
    costs = dict(zip(users.tolist(), cost.tolist()))
    heap = [(0, r) for r in range(world)]
    out = [[] for _ in range(world)]
    for u in order.tolist():
        load, r = heapq.heappop(heap)
        out[r].append(u)
        heapq.heappush(heap, (load + costs[u], r))
    return [np.array(sorted(x), dtype=np.int64) for x in out]


def broadcast_module(model, src=0, group=None):
    """Replicate every parameter and buffer of `model` from rank `src` (one broadcast each)."""
    import torch.distributed as dist
    for t in list(model.parameters()) + list(model.buffers()):
        dist.broadcast(t.data, src=src, group=group)


def gather_topk(local_users, local_ids, local_scores, num_users, group=None):
    """All-gather per-rank [n_r, k] top-k blocks and return (ids, scores) as [num_users, k]
    tensors in user order, on every rank. Blocks are padded to the largest n_r."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = local_ids.device
    k = local_ids.shape[1]
    n = torch.tensor([len(local_users)], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    m = max(ns) if ns else 0
    pad_u = torch.full((m,), -1, dtype=torch.int64, device=dev)
    pad_u[:len(local_users)] = torch.as_tensor(np.asarray(local_users, dtype=np.int64), device=dev)
    pad_i = torch.full((m, k), -1, dtype=torch.int64, device=dev)
    pad_i[:len(local_users)] = local_ids.to(torch.int64)
    pad_s = torch.full((m, k), float("nan"), dtype=torch.float32, device=dev)
    pad_s[:len(local_users)] = local_scores
    gu = [torch.empty_like(pad_u) for _ in range(world)]
    gi = [torch.empty_like(pad_i) for _ in range(world)]
    gs = [torch.empty_like(pad_s) for _ in range(world)]
    dist.all_gather(gu, pad_u, group=group)
    dist.all_gather(gi, pad_i, group=group)
    dist.all_gather(gs, pad_s, group=group)
    ids = torch.full((num_users, k), -1, dtype=torch.int64, device=dev)
    sc = torch.full((num_users, k), float("nan"), dtype=torch.float32, device=dev)
    for r in range(world):
        u = gu[r][:ns[r]]
        ids[u] = gi[r][:ns[r]]
        sc[u] = gs[r][:ns[r]]
    return ids, sc


def distributed_recommend(model, args, num_users, train_matrix, group=None, **kw):
    """recommended_list of validation.py:9-27 computed by all ranks of `group` together."""
    import torch.distributed as dist
    from .catalog import device_csr, score_topk
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    model.eval()
    csr = device_csr(train_matrix, model.embed_history.weight.device)
    P = model.embed_history.weight.shape[0]
    mine = shard_users(csr.hist_len[:num_users], P, world)[rank]
    ids, sc = score_topk(model, csr, mine, args.topk, **kw)
    ids, sc = gather_topk(mine, ids, sc, num_users, group=group)
    return ids.cpu().tolist()


def NAIS_validation_distributed(model, args, num_users, test_positive, val_positive, train_matrix,
                                k_list, group=None):
    """validation.NAIS_validation (validation.py:7-31) across all ranks; same 6-tuple on every rank."""
    from . import eval_metrics
    rec = distributed_recommend(model, args, num_users, train_matrix, group=group)
    precision_v, recall_v, hit_v = eval_metrics.evaluate_mp(val_positive, rec, k_list)
    precision_t, recall_t, hit_t = eval_metrics.evaluate_mp(test_positive, rec, k_list)
    return precision_v, recall_v, hit_v, precision_t, recall_t, hit_t


def allgather_rows(local_rows, num_rows, group=None):
    """Assemble a [num_rows, d] table from per-rank row blocks: rank r holds
    rows [r*S, (r+1)*S) with S = ceil(num_rows / world) (the last block zero-padded), one
    all_gather_into_tensor (a ring over xGMI with RCCL; ~7/8 of the table crosses each link)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    S = (num_rows + world - 1) // world
    d = local_rows.shape[1]
    block = torch.zeros(S, d, dtype=local_rows.dtype, device=local_rows.device)
    block[:local_rows.shape[0]] = local_rows
    full = torch.empty(S * world, d, dtype=local_rows.dtype, device=local_rows.device)
    if hasattr(dist, "all_gather_into_tensor") and dist.get_backend(group) != "gloo":
        dist.all_gather_into_tensor(full, block, group=group)
    else:
        dist.all_gather(list(full.chunk(world)), block, group=group)
    return full[:num_rows]


def row_block(num_rows, rank, world):
    """[start, end) of this rank's row block for allgather_rows."""
    S = (num_rows + world - 1) // world
    return min(rank * S, num_rows), min((rank + 1) * S, num_rows)


def load_sharded_tables(model, init_rows, group=None):
    """Each rank materialises only its 1/world slice of every POI-indexed table (init_rows(name,
    start, end) -> [end-start, d] tensor), then the full tables are all-gathered; the small MLP
    parameters are broadcast from rank 0. For tables too large to build on one host."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    for name in ("embed_history", "embed_target"):
        w = getattr(model, name).weight
        s, e = row_block(w.shape[0], rank, world)
        local = init_rows(name, s, e).to(device=w.device, dtype=w.dtype)
        with torch.no_grad():
            w.copy_(allgather_rows(local, w.shape[0], group))
    for n, p in model.named_parameters():
        if not n.startswith(("embed_history", "embed_target")):
            dist.broadcast(p.data, src=0, group=group)
