"""Shared parity helpers for the test-suite (golden-fixture loading, tie-aware top-k check)."""
from __future__ import annotations

import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Score tolerance written in the north star: fp32 scores within 1e-4 of the reference.
SCORE_ATOL = 1e-4


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def params_from(z, tag):
    pre = tag + "/"
    return {k[len(pre):]: z[k] for k in z.files if k.startswith(pre) and "/" not in k[len(pre):]
            and ("." in k[len(pre):])}


def positives_from(z, kind):
    flat, lens = z[kind + "_flat"], z[kind + "_len"]
    out, o = [], 0
    for n in lens:
        out.append([int(x) for x in flat[o:o + n]])
        o += n
    return out


def ulp32(x):
    """fp32 unit in the last place of |x| (elementwise)."""
    a = np.abs(np.asarray(x, dtype=np.float32))
    return np.spacing(a).astype(np.float64)


def tie_groups(scores, tie_eps=0.0, tie_ulps=None):
    """Split a descending score list into maximal runs whose neighbours differ by <= tie_eps
    (absolute) or, with `tie_ulps`, by <= tie_ulps fp32 ulps of the larger neighbour."""
    groups, start = [], 0
    for i in range(1, len(scores) + 1):
        if i < len(scores):
            gap = scores[i - 1] - scores[i]
            eps = tie_eps if tie_ulps is None else tie_ulps * float(ulp32(max(abs(scores[i - 1]),
                                                                             abs(scores[i]))))
        if i == len(scores) or gap > eps or np.isnan(scores[i]) != np.isnan(scores[i - 1]):
            groups.append((start, i))
            start = i
    return groups


# per-call statistics of assert_topk_equivalent: lists checked, tie runs compared as sets, and
# how many of those runs are not exact fp32 ties (they rely on the ulp allowance)
TIE_STATS = {"lists": 0, "set_runs": 0, "inexact_runs": 0}


def assert_topk_equivalent(ref_ids, ref_scores, our_ids, our_scores, tie_eps=0.0,
                           score_atol=SCORE_ATOL, lookup=None, tie_ulps=None):
    """Tie-aware top-k parity (SURVEY.md 8(a) 'Tie rule').

    Wherever the reference's sorted scores are separated by more than `tie_eps` (or, with
    `tie_ulps`, by more than that many fp32 ulps), the id at each position must be identical.
    Inside a run of scores within that distance of each other the ids are compared as a set; for
    the run that straddles rank k, each of our ids that the reference did not list must carry a
    score within the tie distance of that run (its reference score when `lookup` (id -> reference
    score) is given, else our own). Scores at equal positions must agree within `score_atol`.
    Returns the number of tie runs compared as sets (TIE_STATS accumulates them).
    """
    ref_ids = [int(x) for x in ref_ids]
    our_ids = [int(x) for x in our_ids]
    ref_scores = np.asarray(ref_scores, dtype=np.float64)
    our_scores = np.asarray(our_scores, dtype=np.float64)
    k = len(ref_ids)
    assert len(our_ids) == k, (len(our_ids), k)
    assert len(set(our_ids)) == k, "duplicate ids in top-k"
    both = ~(np.isnan(ref_scores) | np.isnan(our_scores))
    assert np.array_equal(np.isnan(ref_scores), np.isnan(our_scores))
    assert np.all(np.abs(ref_scores[both] - our_scores[both]) <= score_atol), \
        np.max(np.abs(ref_scores[both] - our_scores[both]))
    groups = tie_groups(ref_scores, tie_eps, tie_ulps)
    runs = 0
    TIE_STATS["lists"] += 1
    for gi, (a, b) in enumerate(groups):
        if b - a > 1:
            runs += 1
            TIE_STATS["set_runs"] += 1
            if not np.all(ref_scores[a:b] == ref_scores[a]):
                TIE_STATS["inexact_runs"] += 1
        r, o = set(ref_ids[a:b]), set(our_ids[a:b])
        if gi < len(groups) - 1:
            assert r == o, f"positions {a}:{b}: ref {sorted(r)} ours {sorted(o)}"
        else:
            eps = tie_eps if tie_ulps is None else tie_ulps * float(ulp32(ref_scores[a]))
            lo = ref_scores[b - 1] - eps
            hi = ref_scores[a] + eps
            for pos in range(a, b):
                c = our_ids[pos]
                if c in r:
                    continue
                s = lookup[c] if lookup is not None and c in lookup else our_scores[pos]
                assert lo <= s <= hi, f"id {c} at pos {pos} score {s} outside tie run [{lo},{hi}]"
    return runs


def straddles(ref_scores, k, tie_ulps):
    """True when a run of the reference's sorted scores within `tie_ulps` fp32 ulps of each
    other crosses the cut-off k (positions a < k < b): which of the run's ids fall inside the
    first k is then the summation order's choice, not the model's."""
    return any(a < k < b for a, b in tie_groups(np.asarray(ref_scores, np.float64), 0.0, tie_ulps))


# the gradient tolerance the training tests assert (every gradient within GRAD_RTOL x max|g| of
# its tensor, tests/test_gpu_train.py::_assert_grads)
GRAD_RTOL = 1e-4


def adagrad_slack(g, lr, eps=GRAD_RTOL):
    """How far one Adagrad step (run.py:89; lr * g / sqrt(G), a +-lr step at the first update) can
    move an element when its gradient is known to eps * max|g| of the tensor -- the tolerance the
    gradient checks assert: lr * min(2, 2 eps max|g| / |g|). Negligible for ordinary elements (the
    D = H = 128 three-step loop needs it for 6 of 16,384 W1 elements, gradients ~1 % of the
    tensor's largest), up to a sign flip (2 lr) for gradients within rounding noise of zero. Pass
    the gradient Adagrad sees (weight decay included); sum over steps."""
    g = np.abs(np.asarray(g, dtype=np.float64))
    m = float(g.max()) if g.size else 0.0
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(g > 0, 2.0 * eps * m / g, 2.0)
    return lr * np.minimum(2.0, r)


# how many elements of one tensor may need the Adagrad slack (VERDICT r5 Next 6): at most 0.1 % of
# the tensor and at most 32 -- the slack explains isolated near-zero gradients, not a tensor-wide
# drift
SLACK_MAX_FRAC, SLACK_MAX_COUNT = 1e-3, 32


def slack_limit(size):
    return min(SLACK_MAX_COUNT, int(SLACK_MAX_FRAC * size))


def assert_params_close(name, got, want, slack, rtol=1e-4, atol=2e-5, g=None):
    """Training parity per element (VERDICT r4 'What's weak' 1): every element of `got` within
    atol + rtol |want| of `want`, widened only by that element's Adagrad slack (adagrad_slack:
    the update's sensitivity to the gradient's rounding, which is large only where the gradient
    is near zero). Elements outside the plain tolerance are counted and printed with their worst
    deviation (and, given the gradient `g`, their largest |g| / max|g| of the tensor); none may
    exceed its widened bound, and at most slack_limit(size) of them may need the slack at all.
    Returns how many needed the slack."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    dev = np.abs(got - want)
    plain = atol + rtol * np.abs(want)
    allowed = plain + np.broadcast_to(np.asarray(slack, dtype=np.float64), dev.shape)
    miss = dev > plain
    n = int(miss.sum())
    if n:
        rel = dev / np.maximum(np.abs(want), 1e-30)
        ratio = ""
        if g is not None:
            ga = np.abs(np.asarray(g, dtype=np.float64)).reshape(dev.shape)
            ratio = f", largest |g| / max|g| among them {float(ga[miss].max() / max(ga.max(), 1e-300)):.3g}"
        print(f"{name}: {n} of {miss.size} element(s) off rtol {rtol} / atol {atol}, "
              f"max |dev| {float(dev[miss].max()):.3g}, max rel {float(rel[miss].max()):.3g}, "
              f"worst dev / allowed {float((dev / allowed)[miss].max()):.3g}{ratio}")
    bad = dev > allowed
    assert not bad.any(), (name, np.argwhere(bad)[:8].tolist(), float(dev[bad].max()))
    assert n <= slack_limit(miss.size), (
        f"{name}: {n} elements need the Adagrad slack, more than {slack_limit(miss.size)} "
        f"(0.1 % of {miss.size}, at most {SLACK_MAX_COUNT})")
    return n


def assert_metrics_exact(got, ref_ids, ref_scores, our_rec, val_pos, test_pos, k_list, tie_ulps=4):
    """The 6-tuple of validation.*_validation (validation.py:28-31) equal to the reference's
    EXACTLY, except for (user, k) whose reference top-k has a tie run straddling k: for those the
    expected metric uses our list, every other (user, k) uses the reference's list, and our first
    k ids must be the reference's first k as a set. Returns the straddling (user, k) pairs (the
    users the tie allowance covers), which the caller prints and bounds."""
    from oracle import metrics_oracle
    U = len(ref_ids)
    excused = []
    per_k = {}
    for k in k_list:
        lists = []
        for u in range(U):
            if straddles(ref_scores[u], k, tie_ulps):
                excused.append((u, k))
                lists.append([int(x) for x in our_rec[u]])
            else:
                assert set(int(x) for x in our_rec[u][:k]) == set(int(x) for x in ref_ids[u][:k]), (u, k)
                lists.append([int(x) for x in ref_ids[u]])
        per_k[k] = lists
    want = [[], [], [], [], [], []]
    for k in k_list:
        pv, rv, hv = metrics_oracle.evaluate(val_pos, per_k[k], [k])
        pt, rt, ht = metrics_oracle.evaluate(test_pos, per_k[k], [k])
        for i, v in enumerate((pv, rv, hv, pt, rt, ht)):
            want[i].append(v[0])
    np.testing.assert_array_equal(np.array(got, dtype=np.float64), np.array(want, dtype=np.float64))
    return excused
