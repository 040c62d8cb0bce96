"""Ranking metrics on the host (same names, arguments and results as eval_metrics.py:3-69).

The reference fans each metric out to a `multiprocessing.Pool(len(k_list))` (eval_metrics.py:9-25),
forking 3 x len(k_list) processes per call; the values are the same when computed in-process,
which is what `evaluate_mp` does here. Errors match: recall/hit divide by the number of users
with a non-empty positive list (ZeroDivisionError when there is none, eval_metrics.py:56,69).
"""
from __future__ import annotations


def evaluate_mp(positive_list, recommended_list, k_list):      # eval_metrics.py:3-27
    precision = [precision_at_k(positive_list, recommended_list, k) for k in k_list]
    print(precision)
    recall = [recall_at_k(positive_list, recommended_list, k) for k in k_list]
    print(recall)
    hit = [hitrate_at_k(positive_list, recommended_list, k) for k in k_list]
    print(hit)
    print("--------")
    return precision, recall, hit


def precision_at_k_per_sample(actual, predicted, topk):        # eval_metrics.py:29-34
    num_hits = 0
    for place in predicted:
        if place in actual:
            num_hits += 1
    return num_hits / (topk + 0.0)


def precision_at_k(actual, predicted, topk):                   # eval_metrics.py:36-44
    sum_precision = 0.0
    num_users = len(predicted)
    for i in range(num_users):
        sum_precision += len(set(actual[i]) & set(predicted[i][:topk])) / float(topk)
    return sum_precision / num_users


def recall_at_k(actual, predicted, topk):                      # eval_metrics.py:46-56
    sum_recall, true_users = 0.0, 0
    for i in range(len(predicted)):
        act_set = set(actual[i])
        if len(act_set) != 0:
            sum_recall += len(act_set & set(predicted[i][:topk])) / float(len(act_set))
            true_users += 1
    return sum_recall / true_users


def hitrate_at_k(actual, predicted, topk):                     # eval_metrics.py:58-69
    sum_hit, true_users = 0.0, 0
    for i in range(len(predicted)):
        act_set = set(actual[i])
        if len(act_set) != 0:
            if len(act_set & set(predicted[i][:topk])) > 0:
                sum_hit += 1
            true_users += 1
    return sum_hit / true_users
