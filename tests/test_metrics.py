"""CPU: the vectorised ranking metrics (poi_recommendation_models_amd.eval_metrics) against the
loop restatement of eval_metrics.py:36-69 (oracle/metrics_oracle.py) -- bit-identical floats on
random lists, including empty / duplicated positives, duplicated and ragged recommendations,
k beyond the list length, and the reference's ZeroDivisionError cases."""
import numpy as np
import pytest

from oracle import metrics_oracle
from poi_recommendation_models_amd import eval_metrics


def _case(seed, U=300, P=500, K=50):
    rng = np.random.default_rng(seed)
    pred = [list(rng.choice(P, K, replace=False)) for _ in range(U)]
    act = []
    for u in range(U):
        n = int(rng.integers(0, 6))
        a = list(rng.choice(P, n)) + ([pred[u][int(rng.integers(K))]] if rng.random() < 0.6 else [])
        if n and rng.random() < 0.2:
            a.append(a[0])                          # duplicate positive
        act.append(a)
    return act, pred


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_metrics_bit_identical(seed):
    act, pred = _case(seed)
    k_list = [1, 5, 10, 15, 20, 25, 30, 60]
    got = eval_metrics.evaluate_mp(act, pred, k_list)
    ref = metrics_oracle.evaluate(act, pred, k_list)
    for g, r in zip(got, ref):
        assert g == r                               # exact float equality, list by list


def test_metrics_duplicates_ragged_and_single_functions():
    act, pred = _case(5, U=80, K=20)
    pred[3] = pred[3][:7]                           # ragged
    pred[4] = pred[4][:10] + pred[4][:10]           # repeated ids count once per prefix
    act[4] = [pred[4][0], pred[4][1]]
    for k in (1, 3, 7, 10, 20, 40):
        assert eval_metrics.precision_at_k(act, pred, k) == metrics_oracle.precision_at_k(act, pred, k)
        assert eval_metrics.recall_at_k(act, pred, k) == metrics_oracle.recall_at_k(act, pred, k)
        assert eval_metrics.hitrate_at_k(act, pred, k) == metrics_oracle.hitrate_at_k(act, pred, k)


def test_metrics_zero_division_like_reference():
    with pytest.raises(ZeroDivisionError):
        eval_metrics.recall_at_k([[], []], [[1, 2], [3, 4]], 2)
    with pytest.raises(ZeroDivisionError):
        eval_metrics.hitrate_at_k([[], []], [[1, 2], [3, 4]], 2)
    with pytest.raises(ZeroDivisionError):
        eval_metrics.precision_at_k([], [], 2)
