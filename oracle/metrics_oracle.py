"""CPU oracle for the ranking metrics -- TEST INFRASTRUCTURE ONLY.

Restates eval_metrics.py:36-69 (precision/recall/hit@k) in plain Python to check the
host-side metrics of the product package. Only tests/ import it.
"""
from __future__ import annotations


def precision_at_k(actual, predicted, topk):                 # eval_metrics.py:36-44
    s = 0.0
    for i in range(len(predicted)):
        s += len(set(actual[i]) & set(predicted[i][:topk])) / float(topk)
    return s / len(predicted)


def recall_at_k(actual, predicted, topk):                    # eval_metrics.py:46-56
    s, users = 0.0, 0
    for i in range(len(predicted)):
        a = set(actual[i])
        if len(a) != 0:
            s += len(a & set(predicted[i][:topk])) / float(len(a))
            users += 1
    return s / users


def hitrate_at_k(actual, predicted, topk):                   # eval_metrics.py:58-69
    s, users = 0.0, 0
    for i in range(len(predicted)):
        a = set(actual[i])
        if len(a) != 0:
            if len(a & set(predicted[i][:topk])) > 0:
                s += 1
            users += 1
    return s / users


def evaluate(positive_list, recommended_list, k_list):       # eval_metrics.py:3-27
    return ([precision_at_k(positive_list, recommended_list, k) for k in k_list],
            [recall_at_k(positive_list, recommended_list, k) for k in k_list],
            [hitrate_at_k(positive_list, recommended_list, k) for k in k_list])
