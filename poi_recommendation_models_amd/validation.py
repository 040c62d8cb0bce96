"""Drop-in evaluation loops (same signatures and 6-tuple result as validation.py:7-131).

Each function scores every user's full catalog (complement of the training history) on the
device with the fused NAIS kernel + radix-select top-k (`catalog.score_topk`), builds the same
`recommended_list` (args.topk POI ids per user, best first) and returns
(precision_v, recall_v, hit_v, precision_t, recall_t, hit_t) from `eval_metrics.evaluate_mp`.
The model must be one of this package's NAIS modules, on a ROCm device.

Multi-GPU is opt-in: pass `distributed=True` (or set NAIS_DISTRIBUTED_EVAL=1 for run.py's
unchanged call sites, run.py:112-116, 178-182, 259-263) inside a torch.distributed process group
of more than one rank (one process per GPU, as torchrun starts them). Every function then
evaluates cooperatively across the ranks (sharding.distributed_topk: column-sharded pairs route or
LPT user sharding) and returns the same 6-tuple on every rank; every rank must make the call. The
default is the single-process path even inside a process group, so a DDP script that validates on
rank 0 only does not block in a collective.
"""
from __future__ import annotations

import os

from . import eval_metrics
from .catalog import score_topk


def _distributed_world():
    try:
        import torch.distributed as dist
    except Exception:
        return 1
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size()


def _want_distributed(distributed):
    """distributed=None reads NAIS_DISTRIBUTED_EVAL (falls back to one process, with a warning,
    when no group of > 1 rank exists); distributed=True requires such a group."""
    if distributed is None:     # the env opt-in: single-process when there is no group to use
        if os.environ.get("NAIS_DISTRIBUTED_EVAL", "0") != "1":
            return False
        if _distributed_world() <= 1:
            import warnings
            warnings.warn("NAIS_DISTRIBUTED_EVAL=1 without a process group of > 1 rank: "
                          "evaluating in this process")
            return False
        return True
    if not distributed:
        return False
    if _distributed_world() <= 1:
        raise RuntimeError("distributed evaluation needs an initialised process group of > 1 rank")
    return True


def _recommend_ids(model, args, num_users, train_matrix, distributed=None, **kw):
    model.eval()                                               # validation.py:8
    dist_eval = _want_distributed(distributed)
    if dist_eval:
        from .sharding import distributed_topk
        ids, _ = distributed_topk(model, train_matrix, num_users, args.topk, **kw)
    else:
        ids, _ = score_topk(model, train_matrix, range(num_users), args.topk, **kw)
    nan_t = model._last_nan
    if dist_eval:
        # each rank counted the NaN scores of its own share: one count for the whole job,
        # printed once (model.py:53-54 prints per forward call in one process)
        import torch.distributed as dist
        nan_t = nan_t.clone()
        dist.all_reduce(nan_t)
    nan = int(nan_t.item())
    if nan > 0 and type(model).__name__ == "NAIS_basic" and model.report_nan:
        if not dist_eval or dist.get_rank() == 0:
            print(nan)                                         # model.py:53-54
    return ids.cpu().numpy()


def recommend(model, args, num_users, train_matrix, distributed=None, **kw):
    """recommended_list of validation.py:9-27: per user, args.topk POI ids, best first."""
    return _recommend_ids(model, args, num_users, train_matrix, distributed, **kw).tolist()


def _metrics(test_positive, val_positive, recommended_list, k_list):
    precision_v, recall_v, hit_v = eval_metrics.evaluate_mp(val_positive, recommended_list, k_list)
    precision_t, recall_t, hit_t = eval_metrics.evaluate_mp(test_positive, recommended_list, k_list)
    return precision_v, recall_v, hit_v, precision_t, recall_t, hit_t


def NAIS_validation(model, args, num_users, test_positive, val_positive, train_matrix, k_list,
                    distributed=None):
    """validation.py:7-31 (NAIS_basic)."""
    rec = _recommend_ids(model, args, num_users, train_matrix, distributed)
    return _metrics(test_positive, val_positive, rec, k_list)


def NAIS_region_validation(model, args, num_users, test_positive, val_positive, train_matrix,
                           businessRegionEmbedList, k_list, distributed=None):
    """validation.py:34-59 (NAIS_regionEmbedding)."""
    rec = _recommend_ids(model, args, num_users, train_matrix, distributed,
                         region_of=businessRegionEmbedList)
    return _metrics(test_positive, val_positive, rec, k_list)


def NAIS_region_distance_validation(model, args, num_users, test_positive, val_positive,
                                    train_matrix, businessRegionEmbedList, latlon_mat, k_list,
                                    poi_coords=None, distributed=None):
    """validation.py:62-131 (NAIS_region_distance_Embedding).

    The reference reads (|dlat|, |dlng|) from a P x P x 2 float64 `latlon_mat` (run.py:47-54,214).
    Pass `poi_coords` ([P, 2] lat/lng, the coordinates latlon_mat was built from) to have the
    kernel form the same float64 differences on the fly instead -- bit-identical, and the only
    option at P >= ~50k where the matrix does not fit. `latlon_mat=None` requires poi_coords.
    `args.powerlaw_weight` is read but unused, as at validation.py:66.
    """
    _ = args.powerlaw_weight
    if poi_coords is not None:
        rec = _recommend_ids(model, args, num_users, train_matrix, distributed,
                             region_of=businessRegionEmbedList, coords=poi_coords)
    else:
        rec = _recommend_ids(model, args, num_users, train_matrix, distributed,
                             region_of=businessRegionEmbedList, latlon_mat=latlon_mat)
    return _metrics(test_positive, val_positive, rec, k_list)


def new4_validation(model, args, num_users, test_positive, val_positive, train_matrix,
                    businessRegionEmbedList, k_list, nearPOI, distributed=None):
    """validation.py:254-280 (New4): the context tables are built once (the reference rebuilds
    them in every 1,024-candidate chunk), then every user's catalog is scored with the basic
    kernels. Differs from the reference only where it breaks: with <= 1,024 candidates the
    reference's chunk loop reads `pred` before assigning it (validation.py:264-266); here such
    users are scored normally."""
    model.eval()
    model.extended_tables(nearPOI)
    rec = _recommend_ids(model, args, num_users, train_matrix, distributed)
    return _metrics(test_positive, val_positive, rec, k_list)
