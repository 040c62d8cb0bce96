"""CPU oracle for the NAIS training step (NAIS_basic and the two region variants) -- TEST
INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`/`scripts/bench_train.py`'s CPU leg use
this module; the product package never imports it.

Restates, in float64 numpy, one step of run.py:101-109 on a get_NAIS_batch batch
(batches.py:24-50):

* forward       model.py:57-89 (attention_network) with the Dropout of model.py:71 given as an
                explicit keep mask, then sigmoid (model.py:55)
* loss          nn.BCELoss (model.py:21): mean of -(y max(log p, -100) + (1-y) max(log(1-p), -100))
* backward      the chain rule of the same op sequence, written out by hand:
                BCELoss backward (p - y) / max(p (1 - p), 1e-12) / b, sigmoid backward, the
                bmm/sum, the beta-power normaliser, exp, the mask, attn_layer2, ReLU, Dropout,
                attn_layer1 and the two embedding gathers (index_add by POI id)
* adagrad       torch.optim.Adagrad's update (run.py:89)

Pinned against tests/golden/train_step.npz and train_step_region.npz (gradients from the
reference's own autograd, dropout off); histories may differ per row here (the reference's
general [b, n] input).
"""
from __future__ import annotations

import numpy as np

F64 = np.float64


def train_step_basic(p, hist, data, labels, beta=0.5, keep=None, drop_p=0.0):
    """Forward + backward of NAIS_basic. `p`: dict of parameter arrays keyed like the reference's
    state_dict ('embed_history.weight', ...). `keep`: optional [b, n, H] 0/1 dropout mask (the
    kept units are scaled by 1/(1-drop_p)). Returns dict(pred, logit, loss, grads={name: array})."""
    return train_step(p, hist, data, labels, beta=beta, keep=keep, drop_p=drop_p)


def train_step(p, hist, data, labels, hist_region=None, data_region=None, latlon=None, beta=0.5,
               keep=None, drop_p=0.0, dist_scale=100.0):
    """Forward + backward of NAIS_basic, NAIS_regionEmbedding (model.py:144-180: rows
    [E_hist | E_reg[region]] against [E_tgt | E_reg[region]], when `hist_region` / `data_region`
    are given) or NAIS_region_distance_Embedding (model.py:246-297: also the distance feature
    sigmoid(dist_layer(100 * latlon)) appended to h (.) t, when `latlon` [b, n, 2] is given), or
    NAIS_distance_Embedding (model.py:355-395: `latlon` without regions, dist_scale = 1000)."""
    EH = np.asarray(p["embed_history.weight"], F64)
    ET = np.asarray(p["embed_target.weight"], F64)
    W1 = np.asarray(p["attn_layer1.weight"], F64)
    b1 = np.asarray(p["attn_layer1.bias"], F64)
    w2 = np.asarray(p["attn_layer2.weight"], F64).reshape(-1)
    hist = np.asarray(hist, np.int64)
    data = np.asarray(data, np.int64)
    y = np.asarray(labels, F64)
    b, n = hist.shape
    H = W1.shape[0]
    region = hist_region is not None
    if region:
        ER = np.asarray(p["embed_region.weight"], F64)
        hist_region = np.asarray(hist_region, np.int64)
        data_region = np.asarray(data_region, np.int64)
        h = np.concatenate([EH[hist], ER[hist_region]], -1)          # model.py:151-153
        t = np.concatenate([ET[data], ER[data_region]], -1)          # model.py:155-157
    else:
        h = EH[hist]                                    # model.py:64  [b, n, D]
        t = ET[data]                                    # model.py:66  [b, D]
    x = h * t[:, None, :]                               # model.py:70
    if latlon is not None:                              # model.py:265-267
        Wd = np.asarray(p["dist_layer.weight"], F64)
        bd = np.asarray(p["dist_layer.bias"], F64)
        ll = np.asarray(latlon, F64) * dist_scale         # x100 (:265) / x1000 (:369)
        feat = 1.0 / (1.0 + np.exp(-(ll @ Wd.T + bd)))   # sigmoid(dist_layer(100 ll))
        x = np.concatenate([x, feat], -1)
    u = x @ W1.T + b1                                   # model.py:71 attn_layer1
    if keep is not None and drop_p > 0:
        m = np.asarray(keep, F64) * (1.0 / (1.0 - drop_p))   # Dropout (model.py:71)
    else:
        m = np.ones((b, n, H))
    v = u * m
    z = np.maximum(v, 0.0)                              # ReLU
    a = z @ w2                                          # model.py:73 attn_layer2 [b, n]
    mask = (hist != data[:, None]).astype(F64)          # model.py:92-95
    with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
        e = np.exp(a) * mask                            # model.py:75-78
        S = e.sum(-1)                                   # model.py:79
        Dn = S ** beta                                  # model.py:80
        w = e / Dn[:, None]                             # model.py:82
        s = np.einsum("bnd,bd->bn", h, t)               # h_j . t_c
        logit = (w * s).sum(-1) if n > 0 else np.zeros(b)   # model.py:84-88
        pred = 1.0 / (1.0 + np.exp(-logit))             # model.py:55
        lp = np.maximum(np.log(pred), -100.0)
        l1p = np.maximum(np.log(1.0 - pred), -100.0)
        loss = -np.mean(y * lp + (1.0 - y) * l1p)       # BCELoss (model.py:21)

        # ---- backward
        gp = (pred - y) / np.maximum(pred * (1.0 - pred), 1e-12) / b   # BCELoss backward
        g = gp * (1.0 - pred) * pred                    # sigmoid backward
        dw = g[:, None] * s                             # d/dw_cj
        ds = g[:, None] * w                             # d/ds_cj
        de = dw / Dn[:, None]                           # w = e / Dn
        dDn = -(dw * e).sum(-1) / Dn ** 2
        dS = dDn * beta * S ** (beta - 1.0)
        de = de + dS[:, None]
        da = de * mask * np.exp(a)                      # e = exp(a) * mask
        dz = da[..., None] * w2                         # attn_layer2 backward
        dv = dz * (v > 0)                               # ReLU backward
        du = dv * m                                     # Dropout backward
        dW1 = np.einsum("bnh,bnd->hd", du, x)
        db1 = du.sum((0, 1))
        dw2 = np.einsum("bn,bnh->h", da, z)
        dx = du @ W1
        D = h.shape[-1]
        dfeat = dx[..., D:]
        dx = dx[..., :D]
        dh = dx * t[:, None, :] + ds[..., None] * t[:, None, :]
        dt = (dx * h).sum(1) + (ds[..., None] * h).sum(1)
    I = EH.shape[1]
    gEH = np.zeros_like(EH)
    np.add.at(gEH, hist.reshape(-1), dh[..., :I].reshape(-1, I))
    gET = np.zeros_like(ET)
    np.add.at(gET, data, dt[:, :I])
    grads = {"embed_history.weight": gEH, "embed_target.weight": gET,
             "attn_layer1.weight": dW1, "attn_layer1.bias": db1,
             "attn_layer2.weight": dw2.reshape(1, -1)}
    if region:
        R = ER.shape[1]
        gER = np.zeros_like(ER)
        np.add.at(gER, hist_region.reshape(-1), dh[..., I:].reshape(-1, R))
        np.add.at(gER, data_region, dt[:, I:])
        grads["embed_region.weight"] = gER
    if latlon is not None:
        dpre = dfeat * feat * (1.0 - feat)              # sigmoid backward
        grads["dist_layer.weight"] = np.einsum("bnk,bnm->km", dpre, ll)
        grads["dist_layer.bias"] = dpre.sum((0, 1))
    return dict(pred=pred, logit=logit, loss=loss, grads=grads)


def adagrad(param, state_sum, grad, lr, step, lr_decay=0.0, weight_decay=0.0, eps=1e-10):
    """torch.optim.Adagrad (run.py:89) on float32 arrays; returns (param, state_sum).
    `step` is the optimizer's step count after incrementing (1 on the first step)."""
    f = np.float32
    g = np.asarray(grad, f)
    p = np.asarray(param, f)
    if weight_decay != 0:
        g = (g + f(weight_decay) * p).astype(f)
    clr = f(lr / (1 + (step - 1) * lr_decay))
    st = (np.asarray(state_sum, f) + g * g).astype(f)
    std = (np.sqrt(st) + f(eps)).astype(f)
    return (p - clr * (g / std)).astype(f), st
