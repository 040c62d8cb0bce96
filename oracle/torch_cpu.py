"""TEST / BASELINE INFRASTRUCTURE ONLY -- never imported by the product package.

A torch-CPU restatement of the reference's full-catalog evaluation of NAIS_basic, used as the
CPU baseline of bench.py and pinned against the reference's own golden
outputs (tests/test_torch_cpu_baseline.py). It follows the reference's operations and their
order in plain torch ops on the CPU, with torch's intra-op threads:

  candidates   batches.py:52-65  complement of the CSR history, ascending; the history row
                                 repeated once per candidate (a [C, h] int64 matrix)
  forward      model.py:40-89    gather -> h * t -> attn_layer1 -> ReLU (Dropout off in eval)
                                 -> attn_layer2 -> exp -> mask -> sum -> pow(beta) -> divide ->
                                 weight the history rows -> bmm with t -> sum -> sigmoid
  loop         validation.py:9-27 1,024-candidate chunks, torch.cat, torch.topk(pred, k)
"""
from __future__ import annotations

import math

import numpy as np
import torch


class TorchNAIS:
    """NAIS_basic's eval-mode forward (model.py:40-89) on CPU tensors (or, `device`, on another
    torch device: the same ops through PyTorch's own kernels -- an independent checker of the
    HIP path at sizes the CPU cannot cover, tests/test_gpu_configs.py)."""

    def __init__(self, params, beta=0.5, device=None):
        t = lambda k: torch.as_tensor(np.ascontiguousarray(params[k]), dtype=torch.float32,
                                      device=device)
        self.eh, self.et = t("embed_history.weight"), t("embed_target.weight")
        self.w1, self.b1, self.w2 = t("attn_layer1.weight"), t("attn_layer1.bias"), t("attn_layer2.weight")
        self.beta = beta

    @torch.no_grad()
    def __call__(self, user_history, target_item):
        history = self.eh[user_history]                                   # model.py:64 (b, n, d)
        target = self.et[target_item]                                     # model.py:66
        b = len(target)
        target = target.reshape(b, 1, -1)
        x = history * target                                              # model.py:70
        r1 = torch.relu(torch.nn.functional.linear(x, self.w1, self.b1))  # model.py:71 (eval)
        r2 = torch.nn.functional.linear(r1, self.w2)                      # model.py:73
        e = torch.exp(r2).squeeze(-1)                                     # model.py:75-76
        e = e * (user_history != target_item.reshape(b, 1))               # model.py:77-78, 92-95
        s = torch.pow(torch.sum(e, dim=-1), self.beta)                    # model.py:79-80
        w = torch.divide(e.T, s).T.reshape(b, -1, 1)                      # model.py:82-83
        res = history * w                                                 # model.py:84
        pred = torch.bmm(res, target.reshape(b, -1, 1)).squeeze(-1)       # model.py:86-87
        return torch.sigmoid(torch.sum(pred, dim=-1))                     # model.py:88, 55


def candidates(history, num_pois):
    """batches.py:56-57: ascending complement, the history repeated per candidate."""
    keep = np.ones(num_pois, dtype=bool)
    keep[np.asarray(history, dtype=np.int64)] = False
    cand = np.nonzero(keep)[0]
    rows = np.repeat(np.asarray(history, dtype=np.int64)[None, :], len(cand), axis=0)
    return torch.from_numpy(rows), torch.from_numpy(cand)


def recommend_user(model, history, num_pois, k, chunk=1024):
    """validation.py:11-27 for one user: (top-k POI ids, their scores, #candidates)."""
    user_history, target_list = candidates(history, num_pois)
    n = math.ceil(len(user_history) / chunk)
    pred = torch.cat([model(user_history[chunk * i:chunk * (i + 1)],
                            target_list[chunk * i:chunk * (i + 1)]) for i in range(n)], dim=-1)
    vals, idx = torch.topk(pred, k)
    return target_list[idx].numpy(), vals.numpy(), len(target_list)


class TorchNAISRegionDistance:
    """NAIS_region_distance_Embedding's forward (model.py:246-297) on CPU tensors, in the
    reference's op order: [history | region] rows, dist = sigmoid(dist_layer(latlon * 100)),
    cat, attn_layer1, ReLU (no dropout in this variant), attn_layer2, exp, mask, sums."""

    def __init__(self, params, beta=0.5):
        t = lambda k: torch.as_tensor(np.ascontiguousarray(params[k]), dtype=torch.float32)
        self.eh, self.et, self.er = t("embed_history.weight"), t("embed_target.weight"), t("embed_region.weight")
        self.w1, self.b1, self.w2 = t("attn_layer1.weight"), t("attn_layer1.bias"), t("attn_layer2.weight")
        self.wd, self.bd = t("dist_layer.weight"), t("dist_layer.bias")
        self.beta = beta

    @torch.no_grad()
    def __call__(self, user_history, target_item, history_region, target_region, target_lat_long):
        history = torch.cat((self.eh[user_history], self.er[history_region]), -1)   # model.py:253-255
        target = torch.cat((self.et[target_item], self.er[target_region]), -1)      # model.py:257-259
        b = len(target)
        target = target.reshape(b, 1, -1)
        dist = torch.sigmoid(torch.nn.functional.linear(target_lat_long * 100, self.wd, self.bd))  # :265
        x = torch.cat((history * target, dist), dim=-1)                               # model.py:266-267
        r1 = torch.relu(torch.nn.functional.linear(x, self.w1, self.b1))              # model.py:268
        e = torch.exp(torch.nn.functional.linear(r1, self.w2)).squeeze(-1)            # model.py:269-280
        e = e * (user_history != target_item.reshape(b, 1))                          # model.py:282-283
        s = torch.pow(torch.sum(e, dim=-1), self.beta)                                # model.py:284-285
        w = torch.divide(e.T, s).T.reshape(b, -1, 1)                                  # model.py:287-288
        pred = torch.bmm(history * w, target.reshape(b, -1, 1)).squeeze(-1)           # model.py:289-292
        return torch.sigmoid(torch.sum(pred, dim=-1))


def region_distance_scores(model, history, num_pois, region_of, coords, chunk=2048):
    """validation.py:69-121 for one user (2,048-candidate chunks; latlon_mat entries of run.py:47-54
    formed on demand in float64, cast to float32): (candidates, scores)."""
    user_history, target_list = candidates(history, num_pois)
    region_of = torch.as_tensor(np.asarray(region_of, dtype=np.int64))
    c = torch.as_tensor(np.asarray(coords, dtype=np.float64))
    out = []
    for i in range(0, len(target_list), chunk):
        uh, tg = user_history[i:i + chunk], target_list[i:i + chunk]
        ll = torch.abs(c[tg].unsqueeze(1) - c[uh]).to(torch.float32)
        out.append(model(uh, tg, region_of[uh], region_of[tg], ll))
    return target_list.numpy(), torch.cat(out).numpy()
