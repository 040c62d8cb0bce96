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
    tensors in user order, on every rank. Blocks are padded to the largest n_r. Every exchange is
    one all_gather_into_tensor into a [world * m, ...] buffer: the call RCCL runs, and the one the
    gloo tests run."""
    world = _world(group)
    dev = local_ids.device
    k = local_ids.shape[1]
    n = torch.tensor([len(local_users)], dtype=torch.int64, device=dev)
    ns = all_gather_cat(n, group).tolist()
    m = max(ns) if ns else 0
    pad_u = torch.full((m,), -1, dtype=torch.int64, device=dev)
    pad_u[:len(local_users)] = torch.as_tensor(np.asarray(local_users, dtype=np.int64), device=dev)
    pad_i = torch.full((m, k), -1, dtype=torch.int64, device=dev)
    pad_i[:len(local_users)] = local_ids.to(torch.int64)
    pad_s = torch.full((m, k), float("nan"), dtype=torch.float32, device=dev)
    pad_s[:len(local_users)] = local_scores
    gu = all_gather_cat(pad_u, group).view(world, m)
    gi = all_gather_cat(pad_i, group).view(world, m, k)
    gs = all_gather_cat(pad_s, group).view(world, m, k)
    ids = torch.full((num_users, k), -1, dtype=torch.int64, device=dev)
    sc = torch.full((num_users, k), float("nan"), dtype=torch.float32, device=dev)
    for r in range(world):
        u = gu[r][:ns[r]]
        ids[u] = gi[r][:ns[r]]
        sc[u] = gs[r][:ns[r]]
    return ids, sc


def _world(group=None):
    import torch.distributed as dist
    return dist.get_world_size(group)


def all_gather_cat(block, group=None):
    """[world * block.shape[0], ...] <- every rank's `block` in rank order, by ONE
    all_gather_into_tensor (RCCL: a ring over xGMI; gloo accepts the same concatenated form, so
    the CPU tests execute the call the GPUs run)."""
    import torch.distributed as dist
    block = block.contiguous()
    out = torch.empty((_world(group) * block.shape[0], *block.shape[1:]), dtype=block.dtype,
                      device=block.device)
    dist.all_gather_into_tensor(out, block, group=group)
    return out


_SIGN = -(1 << 63)   # int64 with only the top bit set: u64 keys XOR it order as signed int64


def global_kth_keys(lo_keys, lo_count, k, group=None):
    """The bounded route's threshold over every column shard: per user the k-th largest of all
    ranks' lower-bound keys (lo_keys [m, k] uint64 bit patterns as int64, lo_count[m] valid, the
    k best of this rank's columns; nais_pair_bound_topk) -> [m] int64 (u64 bits; 0 where the shards
    hold fewer than k keys together). One all_gather of the [m, k] lists (8 B per entry, the size of
    the top-k exchange) and a torch.topk over world * k per user. Every key is a lower bound of a
    distinct candidate's exact key, so the result bounds the GLOBAL k-th exact key from below
    (include/nais.h nais_pair_refine_topk `tau`)."""
    m = lo_keys.shape[0]
    world = _world(group)
    valid = torch.arange(k, device=lo_keys.device)[None, :] < lo_count[:, None]
    mine = torch.where(valid, lo_keys, torch.zeros_like(lo_keys)) ^ _SIGN     # signed order
    allk = all_gather_cat(mine, group).view(world, m, k).permute(1, 0, 2).reshape(m, world * k)
    return torch.topk(allk, k, dim=1).values[:, k - 1] ^ _SIGN


def column_blocks(num_pois, world):
    """[(c0, c1)] per rank: rank r owns POIs [r*S, (r+1)*S) clipped to P, S = ceil(P / world).
    With P % world != 0 the last block is narrower, and a rank may own no column at all."""
    S = (num_pois + world - 1) // world
    return [(min(r * S, num_pois), min((r + 1) * S, num_pois)) for r in range(world)]


_mbc_cache = {}


def min_block_candidates(csr, users, num_pois, world):
    """min over (listed user, rank) of the candidates the user has inside the rank's column block:
    the block's width minus the user's history POIs that fall in it. The column-sharded merge
    needs >= k of them everywhere (a short block list would be padded with id -1). Cached per
    (CSR, users, world): distributed_topk_pairs checks it on every call, and at config 4 the
    count over 5M history entries costs tens of ms of host time -- a third of an 8-GPU step."""
    users = np.asarray(users, dtype=np.int64).reshape(-1)
    if len(users) == 0:
        return num_pois
    key = (id(csr), num_pois, world, len(users), hash(users.tobytes()))
    hit = _mbc_cache.get(key)
    if hit is not None and hit[0] is csr:
        return hit[1]
    blocks = column_blocks(num_pois, world)
    width = np.array([c1 - c0 for c0, c1 in blocks], dtype=np.int64)
    S = (num_pois + world - 1) // world
    h = csr.hist_len[users]
    rows = np.repeat(np.arange(len(users)), h)
    starts = csr.host_indptr[users]
    pos = np.repeat(starts - np.concatenate([[0], np.cumsum(h)[:-1]]), h) + np.arange(int(h.sum()))
    blk = csr.host_indices[pos] // S
    inside = np.bincount(rows * world + blk, minlength=len(users) * world).reshape(len(users), world)
    out = int((width[None, :] - inside).min())
    if len(_mbc_cache) > 8:
        _mbc_cache.clear()
    _mbc_cache[key] = (csr, out)
    return out


def distributed_plan(csr, num_users, num_pois, k, world, model=None):
    """"pairs" (column-sharded, distributed_topk_pairs) when the users' histories share POIs
    (entries >= catalog.PAIR_MIN_SHARING x distinct POIs) and every rank's column block keeps k
    candidates for every user; else "users" (LPT user sharding with replicated tables). With user
    sharding and shared histories every rank would build the full pair tables; column sharding
    splits them."""
    from . import catalog
    if world < 2 or (model is not None and model._pairs_only):
        return "pairs" if model is not None and model._pairs_only else "users"
    hist = csr.hist_len[:num_users]
    entries = int(hist.sum())
    used = csr.host_indices[:int(csr.host_indptr[num_users])]
    distinct = int(np.count_nonzero(np.bincount(used, minlength=num_pois))) if entries else 0
    if (distinct and entries >= catalog.PAIR_MIN_SHARING * distinct
            and min_block_candidates(csr, range(num_users), num_pois, world) >= k):
        return "pairs"
    return "users"


MERGE_F64_CAP = 2048    # candidates per row of nais_topk_merge_f64 (include/nais.h)


def distributed_topk(model, train_matrix, num_users, k, group=None, **kw):
    """[num_users, k] (ids, scores) of users 0..num_users-1 computed by all ranks of `group`, the
    same on every rank: column-sharded pairs route or user-sharded per-user kernels
    (distributed_plan)."""
    import torch.distributed as dist
    from .catalog import device_csr, score_topk
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    model.eval()
    csr = device_csr(train_matrix, model._check_device())
    P = model._item_tables()[0].shape[0]
    prior = kw.get("prior") is not None
    # the prior's f64 merge (nais_topk_merge_f64) holds at most MERGE_F64_CAP candidates per user
    if distributed_plan(csr, num_users, P, k, world, model) == "pairs" and not (
            prior and (model._pairs_only or world * k > MERGE_F64_CAP)):
        return distributed_topk_pairs(model, csr, range(num_users), k, group=group, **kw)
    mine = shard_users(csr.hist_len[:num_users], P, world)[rank]
    ids, sc = score_topk(model, csr, mine, k, **kw)
    return gather_topk(mine, ids, sc, num_users, group=group)


def distributed_recommend(model, args, num_users, train_matrix, group=None, **kw):
    """recommended_list of validation.py:9-27 computed by all ranks of `group` together."""
    ids, _ = distributed_topk(model, train_matrix, num_users, args.topk, group=group, **kw)
    return ids.cpu().numpy()


def NAIS_validation_distributed(model, args, num_users, test_positive, val_positive, train_matrix,
                                k_list, group=None):
    """validation.NAIS_validation (validation.py:7-31) across all ranks; same 6-tuple on every rank."""
    from . import eval_metrics
    rec = distributed_recommend(model, args, num_users, train_matrix, group=group)
    precision_v, recall_v, hit_v = eval_metrics.evaluate_mp(val_positive, rec, k_list)
    precision_t, recall_t, hit_t = eval_metrics.evaluate_mp(test_positive, rec, k_list)
    return precision_v, recall_v, hit_v, precision_t, recall_t, hit_t


def distributed_topk_pairs(model, train_matrix, users, k, group=None, events=None, **kw):
    """Column-sharded "pairs" strategy: rank r scores every listed user against POIs
    [r*S, (r+1)*S) (S = ceil(P / world)) -- the pair tables for its columns, the per-user gathers,
    a local top-k -- then one all_gather of the [n, k] blocks and a merge by nais_topk_rows over
    the world*k candidates. Ranks own ascending id ranges, so the merge's (score desc, position
    asc) order is the global (score desc, POI id asc). Every user needs k candidates in every
    column block (checked; otherwise raises ValueError -- use the user-sharded path).

    With `prior` = (a, b, alpha, poi_coords) (run.py:537-539): each rank blends its columns with
    the whole catalog's max G (a MAX all-reduce per user inside _score_topk_pairs), the lists carry
    their f64 blended scores, and the merge ranks on those (nais_topk_merge_f64) -- the ranking of
    the single-process blend, bit for bit."""
    import torch.distributed as dist
    from . import _capi
    from .catalog import _score_topk_pairs, device_csr
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = model._check_device()
    csr = device_csr(train_matrix, dev)
    P = csr.shape[1]
    users = np.asarray(users if isinstance(users, np.ndarray) else list(users), dtype=np.int64)
    n = len(users)
    if world > 1 and min_block_candidates(csr, users, P, world) < k:
        raise ValueError("a column block has fewer than k candidates for some user "
                         "(use the user-sharded path, distributed_topk falls back to it)")
    c0, c1 = column_blocks(P, world)[rank]
    prior = kw.get("prior")
    if n == 0:
        z = torch.empty(0, k, dtype=torch.int64, device=dev)
        return z, torch.empty(0, k, dtype=torch.float32, device=dev)
    grp = (group if group is not None else dist.group.WORLD) if world > 1 else None
    out = _score_topk_pairs(model, csr, users, k, kw.get("region_of"), kw.get("coords"),
                            kw.get("latlon_mat"), None, force=True, cols=(c0, c1), events=events,
                            prior=prior, group=grp if prior is not None else None,
                            return_keys=prior is not None, tau_group=grp if prior is None else None)
    if world == 1:
        return out[0], out[1]
    ids, sc = out[0], out[1]
    if prior is None:   # a shard's list may be short on the bounded route (global threshold):
        sc = torch.where(ids >= 0, sc, torch.full_like(sc, float("-inf")))   # padding ranks last
    # the exchange: one all-gather of this rank's [n, k] block per array ([world * n, k], rank
    # order = ascending POI ranges), then the merge over the world * k candidates per user
    mark = _marker(events, dev)
    gi, gk = exchange_blocks(ids, out[2] if prior is not None else sc, group,
                             wide_ids=prior is not None or P > 2**31 - 1)
    mark("allgather")
    res = merge_topk_f64(gi, gk, k) if prior is not None else merge_topk(gi, gk, k)
    mark("merge")
    return res


def exchange_blocks(ids, keys, group=None, wide_ids=False):
    """All-gather every rank's [n, k] top-k block: ids (int64 POI ids, -1 = short list) and keys
    (f32 scores, or the prior route's f64 keys) -> ([world, n, k] int64, [world, n, k] keys), rank
    order = ascending POI ranges. f32 keys with int32-representable ids travel as ONE all-gather of
    (int32 id, f32 score bits) pairs: 8 B per entry instead of 12 in two calls -- at config 4 and
    N = 8 each rank receives 7 x 50k x 50 x 8 B = 140 MB over the ring. `wide_ids` (f64 keys, or a
    catalog of 2^31 POIs or more, whose ids an int32 would wrap) takes two gathers instead."""
    world = _world(group)
    n, k = ids.shape
    if wide_ids or keys.dtype != torch.float32:
        gi = all_gather_cat(ids.contiguous(), group).view(world, n, k)
        gk = all_gather_cat(keys.contiguous(), group).view(world, n, k)
        return gi, gk
    pk = torch.stack([ids.to(torch.int32), keys.contiguous().view(torch.int32)], dim=-1)
    g = all_gather_cat(pk, group).view(world, n, k, 2)
    return g[..., 0].to(torch.int64), g[..., 1].contiguous().view(torch.float32)


def _marker(events, dev):
    """mark(kind): records a (kind, start, end) event pair on the current stream covering the work
    issued since the previous mark (bench.py's per-phase times); a no-op without `events`."""
    if events is None:
        return lambda kind: None
    stream = torch.cuda.current_stream(dev)
    last = [torch.cuda.Event(enable_timing=True)]
    last[0].record(stream)

    def mark(kind):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        events.append((kind, last[0], e, 1))
        last[0] = e
    return mark


def agree_min(value, device, group=None):
    """The smallest `value` over the ranks (an int; e.g. users per pass, so that every rank makes
    the same passes and hence the same per-pass collectives)."""
    import torch.distributed as dist
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item())


def allreduce_gmax(gmax_bits, group=None):
    """In place: each user's max G over every rank's columns. gmax_bits holds the u64 bit patterns
    of non-negative doubles (nais_pair_prior_gather), which order like the doubles, so an int64 MAX
    all-reduce is the float64 max (run.py:55-59's max over the whole catalog)."""
    import torch.distributed as dist
    dist.all_reduce(gmax_bits, op=dist.ReduceOp.MAX, group=group)
    return gmax_bits


def merge_topk_f64(ids, keys, k):
    """[world, n, k] per-column-block lists with f64 ranking keys (global POI ids, -1 = padding)
    -> the [n, k] global top-k by (key desc, id asc), NaN first (nais_topk_merge_f64)."""
    from . import _capi
    world, n, _ = ids.shape
    dev = ids.device
    cand_k = keys.permute(1, 0, 2).reshape(n, world * k).contiguous()
    cand_i = ids.permute(1, 0, 2).reshape(n, world * k).contiguous()
    out_i = torch.empty(n, k, dtype=torch.int64, device=dev)
    out_s = torch.empty(n, k, dtype=torch.float32, device=dev)
    _capi.check(_capi.load().nais_topk_merge_f64(cand_k.data_ptr(), cand_i.data_ptr(), n, world * k, k,
                                                 out_i.data_ptr(), out_s.data_ptr(), None,
                                                 _capi.stream_handle(dev)), "nais_topk_merge_f64")
    return out_i, out_s


def merge_topk(ids, scores, k):
    """[world, n, k] per-column-block top-k lists (blocks in ascending POI-id order) -> the [n, k]
    global top-k, (score desc, POI id asc), with nais_topk_rows over the world*k candidates."""
    from . import _capi
    world, n, _ = ids.shape
    dev = ids.device
    cand_s = scores.permute(1, 0, 2).reshape(n, world * k).contiguous()
    cand_i = ids.permute(1, 0, 2).reshape(n, world * k)
    pos = torch.empty(n, k, dtype=torch.int32, device=dev)
    top = torch.empty(n, k, dtype=torch.float32, device=dev)
    short = torch.zeros(1, dtype=torch.int32, device=dev)
    _capi.check(_capi.load().nais_topk_rows(cand_s.data_ptr(), world * k, world * k, n, k,
                                            pos.data_ptr(), top.data_ptr(), short.data_ptr(),
                                            _capi.stream_handle(dev)), "nais_topk_rows (merge)")
    return torch.gather(cand_i, 1, pos.to(torch.int64)), top


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
    return all_gather_cat(block, group)[:num_rows]


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
