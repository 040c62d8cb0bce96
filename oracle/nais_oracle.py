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


def _softmax(x):
    x = np.asarray(x, dtype=F32)
    e = np.exp(x - x.max(axis=-1, keepdims=True)).astype(F32)
    return (e / e.sum(axis=-1, keepdims=True, dtype=F32)).astype(F32)


def new4_tables(p, near, embed_size):
    """model.py:1272-1295 + 1215-1222: ([P, D] history rows, [P, D] target rows)."""
    near = np.asarray(near, dtype=np.int64)
    ein = p["embed_ingoing.weight"].astype(F32)[near]           # [P, K, d4]
    eout = p["embed_outgoing.weight"].astype(F32)[near]
    P, K, d4 = ein.shape
    scale = np.sqrt(F32(embed_size / 4)).astype(F32)             # torch.sqrt(torch.tensor(E/4))
    q = ein[:, 0, :].reshape(P, 1, d4)
    k_out = eout.reshape(P, d4, K)                               # reshape, not transpose
    result_out = (_softmax(np.matmul(q, k_out) / scale) @ eout)[:, 0, :]
    q = eout[:, 0, :].reshape(P, 1, d4)
    k_in = ein.reshape(P, d4, K)
    result_in = (_softmax(np.matmul(q, k_in) / scale) @ ein)[:, 0, :]
    xh = np.concatenate([p["embed_history.weight"], result_in, result_out], -1).astype(F32)
    xt = np.concatenate([p["embed_target.weight"], result_out, result_in], -1).astype(F32)
    return xh, xt


def _with_tables(p, xh, xt):
    q = dict(p)
    q["embed_history.weight"], q["embed_target.weight"] = xh, xt
    return q


def forward_new4(p, near, embed_size, user_history, target_item, beta=0.5):
    xh, xt = new4_tables(p, near, embed_size)
    return _sigmoid(attention_basic(_with_tables(p, xh, xt), user_history, target_item, beta))


def catalog_scores_new4(p, near, embed_size, history, num_pois, beta=0.5):
    """validation.py:254-272 (get_NAIS_batch_test_region candidates, chunked forward)."""
    xh, xt = new4_tables(p, near, embed_size)
    return catalog_scores_basic(_with_tables(p, xh, xt), history, num_pois, beta)
