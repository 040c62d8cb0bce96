"""TEST INFRASTRUCTURE: a full-catalog checker for every user of a job, built from PyTorch's own
kernels (rocBLAS GEMMs, a sparse CSR product) -- independent of this package's HIP code.

NAIS_basic's eval score (model.py:40-89) factorises over (history item j, candidate c): with
x = h_j * t_c (model.py:70), e_jc = exp(w2 . relu(W1 x + b1)) masked where j == c (model.py:71-78)
and s_jc = h_j . t_c, the user's logit is sum_j e_jc s_jc / (sum_j e_jc)^beta (model.py:79-88:
the weights e / S^beta applied to the history rows, then the bmm with t). This module forms e and
e*s per 512-column block in torch fp32 ops in that order, sums them per user with a sparse CSR
product (the CSR history as a U x P 0/1 matrix), applies sigmoid and keeps, per user, a running
top-`keep` over the whole catalog (history POIs excluded, validation.py:12-22) plus the checker's
score of every id in `probe_ids` (e.g. the build's own top-k). Only the summation order differs
from the reference's per-user loop; tests/test_torch_pairs_checker.py pins it to the numpy oracle
(and the region_distance form to oracle/torch_cpu.py's restatement of that variant).
"""
from __future__ import annotations

import numpy as np
import torch


@torch.no_grad()
def full_catalog_topk(p, indptr, indices, num_pois, keep, probe_ids, device, beta=0.5,
                      block=512, jchunk=12500, region_of=None, coords=None):
    """-> (top ids [U, keep] int64, their scores [U, keep] f32, scores at probe_ids [U, k] f32),
    all numpy; ties in the running top-k are broken by torch.topk (the comparison is tie-aware).
    With region_of and coords: NAIS_region_distance_Embedding (model.py:246-297) -- rows
    [E | embed_region[region]] (:253-259), x = [h * t | sigmoid(dist_layer(100 |ll|))] (:265-267)
    with ll the float64 coordinate difference cast to float32 (run.py:47-54), no dropout."""
    f = lambda k: torch.as_tensor(np.ascontiguousarray(p[k]), dtype=torch.float32, device=device)
    eh, et, w1, b1, w2 = (f(k) for k in ("embed_history.weight", "embed_target.weight",
                                         "attn_layer1.weight", "attn_layer1.bias", "attn_layer2.weight"))
    dist = coords is not None
    if region_of is not None:
        reg = torch.as_tensor(np.asarray(region_of, np.int64), device=device)
        er = f("embed_region.weight")
        eh = torch.cat([eh, er[reg]], 1)
        et = torch.cat([et, er[reg]], 1)
    if dist:
        cf = torch.as_tensor(np.asarray(coords, np.float64), device=device)
        wd, bd = f("dist_layer.weight"), f("dist_layer.bias")
    P = int(num_pois)
    U = len(indptr) - 1
    crow = torch.as_tensor(np.asarray(indptr, np.int64), device=device)
    col = torch.as_tensor(np.asarray(indices, np.int64), device=device)
    # the e / e*s rows of the distinct history POIs only (all of them at config 4; a few thousand
    # of config 5's 10^6)
    rows, rcol = torch.unique(col, return_inverse=True)
    J = rows.numel()
    A = torch.sparse_csr_tensor(crow, rcol, torch.ones(col.numel(), dtype=torch.float32, device=device),
                                size=(U, J))
    row_of = torch.repeat_interleave(torch.arange(U, device=device), crow[1:] - crow[:-1])
    by_col = torch.argsort(col)
    col_sorted = col[by_col]
    probe = torch.as_tensor(np.asarray(probe_ids, np.int64), device=device)
    at_probe = torch.full(probe.shape, float("nan"), dtype=torch.float32, device=device)
    top_v = torch.full((U, keep), -float("inf"), dtype=torch.float32, device=device)
    top_i = torch.full((U, keep), -1, dtype=torch.int64, device=device)
    for c0 in range(0, P, block):
        c1 = min(P, c0 + block)
        t = et[c0:c1]                                                  # [w, D]
        E = torch.empty(J, c1 - c0, dtype=torch.float32, device=device)
        ES = torch.empty_like(E)
        for j0 in range(0, J, jchunk):
            j1 = min(J, j0 + jchunk)
            jr = rows[j0:j1]
            h = eh[jr]
            x = h[:, None, :] * t[None, :, :]                          # model.py:70
            if dist:                                                   # model.py:265-267
                ll = torch.abs(cf[c0:c1][None, :, :] - cf[jr][:, None, :]).to(torch.float32)
                x = torch.cat([x, torch.sigmoid(torch.nn.functional.linear(ll * 100, wd, bd))], -1)
                del ll
            r1 = torch.relu(torch.nn.functional.linear(x, w1, b1))     # model.py:71
            e = torch.exp(torch.nn.functional.linear(r1, w2)).squeeze(-1)   # model.py:73-76
            self_ = (jr >= c0) & (jr < c1)                             # model.py:77-78: j == c
            if bool(self_.any()):
                q = torch.nonzero(self_).squeeze(1)
                e[q, jr[q] - c0] = 0.0
            E[j0:j1] = e
            ES[j0:j1] = e * (h @ t.T)
        S = A @ E                                                      # [U, w]
        N = A @ ES
        sc = torch.sigmoid(N / torch.pow(S, beta))
        a, b = torch.searchsorted(col_sorted, torch.tensor([c0, c1], device=device)).tolist()
        nz = by_col[a:b]
        sc[row_of[nz], col[nz] - c0] = -float("inf")                   # history POIs are not candidates
        inb = (probe >= c0) & (probe < c1)
        r, k = torch.nonzero(inb, as_tuple=True)
        at_probe[r, k] = sc[r, probe[r, k] - c0]
        ids = torch.arange(c0, c1, device=device).expand(U, -1)
        v, ix = torch.topk(torch.cat([top_v, sc], 1), keep, dim=1)
        top_i = torch.gather(torch.cat([top_i, ids], 1), 1, ix)
        top_v = v
        del E, ES, S, N, sc
    return top_i.cpu().numpy(), top_v.cpu().numpy(), at_probe.cpu().numpy()


def check_against_full_catalog(ids, scores, ref_top_i, ref_top_v, ref_at_ids, score_atol, tie_ulps):
    """The build's top-k lists [U, k] against the checker's full-catalog results:
      * the checker's score of each of the build's winners within score_atol of the build's;
      * no candidate of the whole catalog beats the build's weakest winner, in the checker's
        arithmetic, by more than tie_ulps ulps. The checker's top-`keep` (keep > k) suffices: it
        holds at least keep - k candidates that are not winners, each at least its keep-th score;
        once they are within the allowance, so is that keep-th score and with it every candidate
        outside the top-`keep`;
    -> (max |winner score diff|, users whose ids equal the checker's top-k as sets, max excess)."""
    k = ids.shape[1]
    assert ref_top_i.shape[1] > k
    assert not np.isnan(ref_at_ids).any(), "a winner's id was not scored by the checker"
    dw = np.abs(ref_at_ids - scores)
    assert dw.max() <= score_atol, (int(np.argmax(dw.max(1))), float(dw.max()))
    weakest = ref_at_ids.min(1)
    allow = tie_ulps * np.spacing(weakest.astype(np.float32))
    mine = np.zeros(ref_top_i.shape, bool)
    for i in range(k):
        mine |= ref_top_i == ids[:, i:i + 1]
    over = np.where(mine, -np.inf, ref_top_v - weakest[:, None])
    bad = over > allow[:, None]
    assert not bad.any(), (np.nonzero(bad.any(1))[0][:5].tolist(), float(over.max()))
    same = int(np.all(np.sort(ref_top_i[:, :k], 1) == np.sort(ids, 1), axis=1).sum())
    return float(dw.max()), same, float(over.max())
