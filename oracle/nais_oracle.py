"""CPU oracle for the NAIS scoring path -- TEST INFRASTRUCTURE ONLY.

This module is the parity checker. Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import it; the product package
(`poi_recommendation_models_amd`) never does, and it never runs as the measured path.

It restates, in numpy float32, the reference's NAIS forward and full-catalog evaluation
op for op, in the reference's order:

* `attention_basic`            <- model.py:57-89 (NAIS_basic.attention_network), mask model.py:92-95
* `forward_basic`              <- model.py:40-55 (NaN count + sigmoid)
* `attention_region`           <- model.py:144-180 (NAIS_regionEmbedding.attention_network)
* `attention_region_distance`  <- model.py:246-297 (NAIS_region_distance_Embedding.attention_network)
* `attention_distance`         <- model.py:355-395 (NAIS_distance_Embedding.attention_network)
* `new4_tables`, `forward_new4` <- model.py:1212-1295 (New4: near-POI self_attention, then the
                                  basic attention over the concatenated rows)
* `near_pool`, `family_tables`, `forward_family` <- the other table-based New4-family members
                                  (New4_padding model.py:1308, all_in_out :1447, nearPOI_embedding
                                  :1578, no_POI_emb :1707, transform_ingoing_outgoing :1822,
                                  only_area_not_inout :2100, transform_attn :1959 with its
                                  dot-product core `attention_dot`, model.py:2015-2055)
* `attention_disentangled`     <- model.py:457-527 (NAIS_region_distance_disentangled_Embedding)
* `complement_candidates`      <- batches.py:52-65 (set(range(P)) - set(history), ascending)
* `catalog_scores_*`           <- validation.py:11-22 / 38-49 / 69-121 (chunked forward over all candidates)
* `topk_ids`                   <- validation.py:26-27 (torch.topk + id lookup), with the build's
                                  deterministic tie rule (score desc, id asc); the reference's own
                                  tie order is implementation defined (SURVEY.md 8(a) tie rule).

Eval mode only: Dropout (model.py:71, 162) is the identity. The oracle is pinned against golden
vectors produced by importing the reference itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def _sigmoid(x):
    x = np.asarray(x, dtype=F32)
    with np.errstate(over="ignore"):
        return (F32(1) / (F32(1) + np.exp(-x))).astype(F32)


def _attention_tail(history, target, user_history, target_item, w1, b1, w2, beta, extra=None):
    """Shared tail of the three attention_network variants.

    history [b,n,D], target [b,D] (already concatenated for the region variants).
    `extra` [b,n,2] is the distance feature appended after h*t (model.py:266-267).
    """
    b = target.shape[0]
    t3 = target.reshape(b, 1, -1)                                # model.py:69
    inp = (history * t3).astype(F32)                             # model.py:70
    if extra is not None:
        inp = np.concatenate([inp, extra.astype(F32)], axis=-1)  # model.py:267
    r1 = inp @ w1.T.astype(F32) + b1.astype(F32)                 # model.py:71 attn_layer1
    r1 = np.maximum(r1, F32(0))                                  # ReLU(Dropout(.)) in eval
    r2 = (r1 @ w2.reshape(-1, 1).astype(F32))[..., 0]            # model.py:73 attn_layer2 (no bias)
    with np.errstate(over="ignore", invalid="ignore"):
        exp_a = np.exp(r2).astype(F32)                           # model.py:75 (no max-subtraction)
        mask = (user_history != target_item.reshape(-1, 1))      # model.py:92-95
        exp_a = (exp_a * mask).astype(F32)                       # model.py:78 (inf*0 -> NaN as in torch)
        exp_sum = exp_a.sum(axis=-1, dtype=F32)                  # model.py:79
        exp_sum = np.power(exp_sum, F32(beta)).astype(F32)       # model.py:80
        attn = (exp_a.T / exp_sum).T.astype(F32)                 # model.py:82
        result = (history * attn[..., None]).astype(F32)         # model.py:84
        pred = np.einsum("bnd,bd->bn", result, target, dtype=F32)  # model.py:87 bmm
        pred = pred.sum(axis=-1, dtype=F32)                      # model.py:88
    return pred.astype(F32)


def attention_basic(p, user_history, target_item, beta=0.5):
    """model.py:57-89. user_history int64 [b,n], target_item int64 [b] -> logits f32 [b]."""
    eh = p["embed_history.weight"]
    et = p["embed_target.weight"]
    history = eh[user_history]                                   # model.py:64
    target = et[target_item]                                     # model.py:66
    return _attention_tail(history, target, user_history, target_item,
                           p["attn_layer1.weight"], p["attn_layer1.bias"],
                           p["attn_layer2.weight"], beta)


def forward_basic(p, user_history, target_item, beta=0.5):
    """model.py:40-55: returns (sigmoid scores f32 [b], NaN count of the logits)."""
    logit = attention_basic(p, user_history, target_item, beta)
    nan_count = int(np.isnan(logit).sum())                       # model.py:50-52
    return _sigmoid(logit), nan_count


def attention_region(p, user_history, target_item, history_region, target_region, beta=0.5):
    """model.py:144-180: [E_hist | E_reg] rows against [E_tgt | E_reg]."""
    er = p["embed_region.weight"]
    history = np.concatenate([p["embed_history.weight"][user_history],
                              er[history_region]], axis=-1)      # model.py:151-153
    target = np.concatenate([p["embed_target.weight"][target_item],
                             er[target_region]], axis=-1)        # model.py:155-157
    return _attention_tail(history, target, user_history, target_item,
                           p["attn_layer1.weight"], p["attn_layer1.bias"],
                           p["attn_layer2.weight"], beta)


def dist_feature(p, target_lat_long, scale=100):
    """model.py:265 (scale 100) / model.py:369 (scale 1000, NAIS_distance_Embedding):
    sigmoid(dist_layer(target_lat_long * scale)) -> [b,n,2] f32."""
    ll = (np.asarray(target_lat_long, dtype=F32) * F32(scale)).astype(F32)
    wd = p["dist_layer.weight"].astype(F32)
    bd = p["dist_layer.bias"].astype(F32)
    return _sigmoid(ll @ wd.T + bd)


def attention_region_distance(p, user_history, target_item, history_region, target_region,
                              target_lat_long, beta=0.5):
    """model.py:246-297 (no dropout in this variant, model.py:268)."""
    er = p["embed_region.weight"]
    history = np.concatenate([p["embed_history.weight"][user_history],
                              er[history_region]], axis=-1)      # model.py:253-255
    target = np.concatenate([p["embed_target.weight"][target_item],
                             er[target_region]], axis=-1)        # model.py:257-259
    dist = dist_feature(p, target_lat_long)                      # model.py:265
    return _attention_tail(history, target, user_history, target_item,
                           p["attn_layer1.weight"], p["attn_layer1.bias"],
                           p["attn_layer2.weight"], beta, extra=dist)


def attention_distance(p, user_history, target_item, target_lat_long, beta=0.5):
    """model.py:355-395 (NAIS_distance_Embedding): basic embeddings + the x1000 distance feature."""
    history = p["embed_history.weight"][user_history]            # model.py:361
    target = p["embed_target.weight"][target_item]               # model.py:362
    dist = dist_feature(p, target_lat_long, scale=1000)          # model.py:369
    return _attention_tail(history, target, user_history, target_item,
                           p["attn_layer1.weight"], p["attn_layer1.bias"],
                           p["attn_layer2.weight"], beta, extra=dist)


def latlon_pairs(coords, target_pois, history_pois):
    """run.py:47-54 latlon_mat entries, computed on demand: (|dlat|, |dlng|) in float64.

    The reference materialises a P x P x 2 float64 matrix and fancy-indexes it
    (validation.py:108-113), then casts to float32 (validation.py:118)."""
    c = np.asarray(coords, dtype=np.float64)
    t = c[np.asarray(target_pois)]
    h = c[np.asarray(history_pois)]
    return np.abs(t[..., :] - h[..., :])


def complement_candidates(history, num_pois):
    """batches.py:56: list(set(range(P)) - set(history)); ascending for int sets."""
    keep = np.ones(num_pois, dtype=bool)
    keep[np.asarray(history, dtype=np.int64)] = False
    return np.nonzero(keep)[0].astype(np.int64)


def catalog_scores_basic(p, history, num_pois, beta=0.5, chunk=1024):
    """validation.py:12-22: sigmoid scores of every non-history POI, ascending id order."""
    cand = complement_candidates(history, num_pois)
    hist = np.asarray(history, dtype=np.int64)
    out = np.empty(len(cand), dtype=F32)
    for s in range(0, len(cand), chunk):
        tg = cand[s:s + chunk]
        uh = np.broadcast_to(hist, (len(tg), len(hist)))         # batches.py:57 (repeat)
        out[s:s + chunk], _ = forward_basic(p, uh, tg, beta)
    return cand, out


def catalog_scores_region(p, history, num_pois, region_of, beta=0.5, chunk=1024):
    """validation.py:38-49 with batches.py:110-139 region lookups."""
    cand = complement_candidates(history, num_pois)
    hist = np.asarray(history, dtype=np.int64)
    region_of = np.asarray(region_of, dtype=np.int64)
    out = np.empty(len(cand), dtype=F32)
    for s in range(0, len(cand), chunk):
        tg = cand[s:s + chunk]
        uh = np.broadcast_to(hist, (len(tg), len(hist)))
        hr = np.broadcast_to(region_of[hist], uh.shape)
        out[s:s + chunk] = _sigmoid(attention_region(p, uh, tg, hr, region_of[tg], beta))
    return cand, out


def catalog_scores_region_distance(p, history, num_pois, region_of, coords, beta=0.5,
                                   chunk=2048):
    """validation.py:69-121 (chunk 2048, latlon from run.py:47-54 cast to f32)."""
    cand = complement_candidates(history, num_pois)
    hist = np.asarray(history, dtype=np.int64)
    region_of = np.asarray(region_of, dtype=np.int64)
    out = np.empty(len(cand), dtype=F32)
    for s in range(0, len(cand), chunk):
        tg = cand[s:s + chunk]
        uh = np.broadcast_to(hist, (len(tg), len(hist)))
        hr = np.broadcast_to(region_of[hist], uh.shape)
        tp = np.broadcast_to(tg.reshape(-1, 1), uh.shape)
        ll = latlon_pairs(coords, tp, uh).astype(F32)           # validation.py:113,118
        out[s:s + chunk] = _sigmoid(attention_region_distance(p, uh, tg, hr, region_of[tg], ll, beta))
    return cand, out


def topk_ids(cand, scores, k):
    """validation.py:26-27 with a deterministic tie rule: score desc, then POI id asc.

    NaN ranks above every number, as in torch.topk."""
    s = np.asarray(scores, dtype=np.float64)
    key = np.where(np.isnan(s), np.inf, s)
    nanrank = np.isnan(s)
    order = np.lexsort((np.asarray(cand), -key, ~nanrank))
    order = order[:k]
    return np.asarray(cand)[order], np.asarray(scores)[order]


def catalog_scores_distance(p, history, num_pois, coords, beta=0.5, chunk=2048):
    """validation.py:69-121 run with NAIS_distance_Embedding (run.py:431): regions ignored."""
    cand = complement_candidates(history, num_pois)
    hist = np.asarray(history, dtype=np.int64)
    out = np.empty(len(cand), dtype=F32)
    for s in range(0, len(cand), chunk):
        tg = cand[s:s + chunk]
        uh = np.broadcast_to(hist, (len(tg), len(hist)))
        tp = np.broadcast_to(tg.reshape(-1, 1), uh.shape)
        ll = latlon_pairs(coords, tp, uh).astype(F32)
        out[s:s + chunk] = _sigmoid(attention_distance(p, uh, tg, ll, beta))
    return cand, out


def _mlp_logit(x, w1, b1, w2):
    r1 = np.maximum((x @ np.asarray(w1, F32).T + np.asarray(b1, F32)).astype(F32), F32(0))
    return (r1 @ np.asarray(w2, F32).reshape(-1, 1))[..., 0].astype(F32)


def attention_disentangled(p, user_history, target_item, history_region, target_region,
                           target_distance, beta=0.5):
    """NAIS_region_distance_disentangled_Embedding.attention_network (model.py:457-527): an
    item MLP and a region MLP, both shifted by d_j = sum_e embed_distance[0][e] * dist_j, each
    normalised with its own beta-smoothed masked exp sum; logits [b]."""
    history = p["embed_history.weight"][user_history]                # :465
    hreg = p["embed_region.weight"][history_region]                 # :466
    target = p["embed_target.weight"][target_item][:, None, :]       # :467, :472
    treg = p["embed_region.weight"][target_region][:, None, :]       # :468, :473
    l1 = _mlp_logit((history * target).astype(F32), p["attn_layer1.weight"], p["attn_layer1.bias"],
                    p["attn_layer2.weight"])                         # :477-478
    l2 = _mlp_logit((hreg * treg).astype(F32), p["region_attn_layer1.weight"],
                    p["region_attn_layer1.bias"], p["region_attn_layer2.weight"])   # :480-481
    wd = p["embed_distance.weight"][0].astype(F32)
    dist = (wd[None, None, :] * np.asarray(target_distance, F32)[..., None]).sum(-1, dtype=F32)  # :488-491
    with np.errstate(over="ignore", invalid="ignore"):
        mask = (user_history != target_item.reshape(-1, 1))
        e1 = (np.exp((l1 + dist).astype(F32)).astype(F32) * mask).astype(F32)       # :496-502
        e2 = (np.exp((l2 + dist).astype(F32)).astype(F32) * mask).astype(F32)
        a1 = (e1.T / np.power(e1.sum(-1, dtype=F32), F32(beta)).astype(F32)).T.astype(F32)   # :504-512
        a2 = (e2.T / np.power(e2.sum(-1, dtype=F32), F32(beta)).astype(F32)).T.astype(F32)
        res = np.concatenate([history * a1[..., None], hreg * a2[..., None]], -1).astype(F32)   # :517-520
        tgt = np.concatenate([target, treg], -1)[:, 0, :]
        pred = np.einsum("bnd,bd->bn", res, tgt, dtype=F32).sum(-1, dtype=F32)   # :523-524
    return pred.astype(F32)


def _softmax(x):
    x = np.asarray(x, dtype=F32)
    e = np.exp(x - x.max(axis=-1, keepdims=True)).astype(F32)
    return (e / e.sum(axis=-1, keepdims=True, dtype=F32)).astype(F32)


def _linear(x, w, b):
    """nn.Linear: x @ W^T + b (float32)."""
    if w is None:
        return x
    y = np.matmul(x, np.asarray(w, F32).T).astype(F32)
    return (y + np.asarray(b, F32)).astype(F32) if b is not None else y


def near_pool(q_tab, kv_tab, near, scale_dim, lq=(None, None), lk=(None, None), lv=(None, None)):
    """One self_attention pool (model.py:1281-1286 and its siblings): for every POI p,
    softmax(q . reshape(key, [d, K]) / sqrt(scale_dim)) @ value with q = Q[near[p][0]],
    keys/values = KV[near[p]] (through the optional Linear projections of
    transform_ingoing_outgoing, model.py:1934-1943). Returns [P, d]."""
    near = np.asarray(near, dtype=np.int64)
    x = np.asarray(kv_tab, F32)[near]                             # [P, K, d]
    P, K, d = x.shape
    q = _linear(np.asarray(q_tab, F32)[near[:, 0]], *lq).reshape(P, 1, d)
    keys = _linear(x, *lk).reshape(P, d, K)                       # reshape, not transpose
    vals = _linear(x, *lv)
    scale = np.sqrt(F32(scale_dim)).astype(F32)                   # torch.sqrt(torch.tensor(E/4 | E/2))
    return (_softmax(np.matmul(q, keys) / scale) @ vals)[:, 0, :].astype(F32)


def _in_out_pools(p, near, d, lin=None):
    """(result_in, result_out) of the two-pool self_attention: result_out pools embed_outgoing with
    the query from embed_ingoing, result_in the reverse (model.py:1281-1295)."""
    ein, eout = p["embed_ingoing.weight"], p["embed_outgoing.weight"]
    none = (None, None)
    lq = lk = lv = lvin = none
    if lin:    # transform_ingoing_outgoing: query/key/value Linear; v_in uses query (model.py:1943)
        lq, lk, lv = ((p[n + ".weight"], p[n + ".bias"]) for n in ("query", "key", "value"))
        lvin = lq
    r_out = near_pool(ein, eout, near, d, lq, lk, lv)
    r_in = near_pool(eout, ein, near, d, lq, lk, lvin)
    return r_in, r_out


# table-based members of the New4 family: the [P, D] (history rows, target rows) NAIS_basic's
# attention runs over (each forward's cat(...) calls, model.py lines cited per member)
NEAR_FAMILY = ("New4", "New4_padding", "all_in_out", "nearPOI_embedding", "no_POI_emb",
               "transform_ingoing_outgoing", "only_area_not_inout", "transform_attn")


def family_tables(model, p, near, embed_size):
    near = np.asarray(near, dtype=np.int64)
    P = near.shape[0]
    cat = lambda *a: np.concatenate([np.asarray(x, F32)[:P] for x in a], -1).astype(F32)  # noqa: E731
    E = embed_size
    if model in ("New4", "New4_padding", "transform_ingoing_outgoing", "transform_attn"):
        # :1212-1236, :1351-1375, :1865-1889, :2002-2026
        r_in, r_out = _in_out_pools(p, near, E / 4, lin=model == "transform_ingoing_outgoing")
        return cat(p["embed_history.weight"], r_in, r_out), cat(p["embed_target.weight"], r_out, r_in)
    if model == "all_in_out":                                             # :1492-1517
        r_in, r_out = _in_out_pools(p, near, E / 4)
        a, b = p["embed_history_ingoing.weight"], p["embed_history_outgoing.weight"]
        return cat(a, b, r_in, r_out), cat(b, a, r_out, r_in)
    if model == "nearPOI_embedding":                                      # :1622-1647, :1680-1686
        e = p["embed_near.weight"]
        r = near_pool(e, e, near, E / 2)
        a, b = p["embed_history_ingoing.weight"], p["embed_history_outgoing.weight"]
        return cat(a, b, r), cat(b, a, r)
    if model == "no_POI_emb":                                             # :1743-1760, :1797-1812
        r_in, r_out = _in_out_pools(p, near, E / 2)
        return cat(r_in, r_out), cat(r_out, r_in)
    if model == "only_area_not_inout":                                    # :2141-2165, :2198-2218
        e = p["embed_area.weight"]
        r = near_pool(e, e, near, E / 2)
        return cat(p["embed_history.weight"], r), cat(p["embed_target.weight"], r)
    raise ValueError(model)


def new4_tables(p, near, embed_size):
    """model.py:1272-1295 + 1215-1222: ([P, D] history rows, [P, D] target rows)."""
    return family_tables("New4", p, near, embed_size)


def _with_tables(p, xh, xt):
    q = dict(p)
    q["embed_history.weight"], q["embed_target.weight"] = xh, xt
    return q


def forward_new4(p, near, embed_size, user_history, target_item, beta=0.5):
    xh, xt = new4_tables(p, near, embed_size)
    return _sigmoid(attention_basic(_with_tables(p, xh, xt), user_history, target_item, beta))


def catalog_scores_new4(p, near, embed_size, history, num_pois, beta=0.5, model="New4", chunk=1024):
    """validation.py:254-272 (get_NAIS_batch_test_region candidates, chunked forward)."""
    xh, xt = family_tables(model, p, near, embed_size)
    if model != "transform_attn":
        return catalog_scores_basic(_with_tables(p, xh, xt), history, num_pois, beta)
    # the reference's 1024-row chunks matter here: a one-item history couples the rows of a chunk
    cand = complement_candidates(history, num_pois)
    hist = np.asarray(history, dtype=np.int64)
    out = np.empty(len(cand), dtype=F32)
    for s in range(0, len(cand), chunk):
        tg = cand[s:s + chunk]
        uh = np.broadcast_to(hist, (len(tg), len(hist)))
        out[s:s + chunk] = _sigmoid(attention_dot(p, xh, xt, uh, tg, embed_size, beta))
    return cand, out


def attention_dot(p, xh, xt, user_history, target_item, embed_size, beta=0.5):
    """transform_attn.attention_network (model.py:2015-2055): q = query(t), k = key(h_j),
    v = value(h_j) (nn.Linear over the full rows, Dropout on k = identity in eval),
    logit_j = sum(q * k_j) / sqrt(E); the same masked, beta-smoothed exp pooling, applied to v;
    prediction = sum_j w_j (v_j . t).

    Restated with torch's shapes: result2 is already [b, n], so exp_A.squeeze(dim=-1)
    (model.py:2042) turns a one-item history ([b, 1]) into [b], and `exp_A * mask` then broadcasts
    to [b, b]: for n == 1 every row's weight sums exp over ALL b rows of the call,
    pred_r = (v_r . t_r) * mask_r * S / (mask_r * S)^beta with S = sum_r' exp(logit_r')."""
    history = np.asarray(xh, F32)[user_history]
    target = np.asarray(xt, F32)[target_item]
    b = target.shape[0]
    t3 = target.reshape(b, 1, -1)
    q = _linear(t3, p["query.weight"], p["query.bias"])
    k = _linear(history, p["key.weight"], p["key.bias"])
    v = _linear(history, p["value.weight"], p["value.bias"])
    r2 = ((q * k).sum(axis=-1, dtype=F32) / np.sqrt(F32(embed_size)).astype(F32)).astype(F32)
    with np.errstate(over="ignore", invalid="ignore"):
        exp_a = np.exp(r2).astype(F32)
        if exp_a.shape[-1] == 1:
            exp_a = exp_a[..., 0]                                 # squeeze(dim=-1)
        mask = (user_history != target_item.reshape(-1, 1))
        exp_a = (exp_a * mask).astype(F32)                        # [b, n] or [b, b]
        exp_sum = np.power(exp_a.sum(axis=-1, dtype=F32), F32(beta)).astype(F32)
        attn = (exp_a.T / exp_sum).T.astype(F32).reshape(b, -1, 1)
        result = (v * attn).astype(F32)
        pred = np.einsum("bnd,bd->bn", result, target, dtype=F32).sum(axis=-1, dtype=F32)
    return pred.astype(F32)


def family_logits(model, p, xh, xt, user_history, target_item, embed_size, beta=0.5):
    if model == "transform_attn":
        return attention_dot(p, xh, xt, user_history, target_item, embed_size, beta)
    return attention_basic(_with_tables(p, xh, xt), user_history, target_item, beta)


def forward_family(model, p, near, embed_size, user_history, target_item, beta=0.5):
    xh, xt = family_tables(model, p, near, embed_size)
    return _sigmoid(family_logits(model, p, xh, xt, user_history, target_item, embed_size, beta))
