"""Drop-in evaluation loops (same signatures and 6-tuple result as validation.py:7-131).

Each function scores every user's full catalog (complement of the training history) on the
device with the fused NAIS kernel + radix-select top-k (`catalog.score_topk`), builds the same
`recommended_list` (args.topk POI ids per user, best first) and returns
(precision_v, recall_v, hit_v, precision_t, recall_t, hit_t) from `eval_metrics.evaluate_mp`.
The model must be one of this package's NAIS modules, on a ROCm device.

Multi-GPU: when a torch.distributed process group with more than one rank is initialised (one
process per GPU, as torchrun starts them), every function here evaluates cooperatively across the
ranks (sharding.distributed_topk: column-sharded pairs route or LPT user sharding) and returns the
same 6-tuple on every rank, so run.py's call sites (run.py:112-116, 178-182, 259-263) stay as they
are. Every rank must make the call.
"""
from __future__ import annotations

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


def _recommend_ids(model, args, num_users, train_matrix, **kw):
    model.eval()                                               # validation.py:8
    if _distributed_world() > 1:
        from .sharding import distributed_topk
        ids, _ = distributed_topk(model, train_matrix, num_users, args.topk, **kw)
    else:
        ids, _ = score_topk(model, train_matrix, range(num_users), args.topk, **kw)
    nan = int(model._last_nan.item())
    if nan > 0 and type(model).__name__ == "NAIS_basic" and model.report_nan:
        print(nan)                                             # model.py:53-54
    return ids.cpu().numpy()


def recommend(model, args, num_users, train_matrix, **kw):
    """recommended_list of validation.py:9-27: per user, args.topk POI ids, best first."""
    return _recommend_ids(model, args, num_users, train_matrix, **kw).tolist()


def _metrics(test_positive, val_positive, recommended_list, k_list):
    precision_v, recall_v, hit_v = eval_metrics.evaluate_mp(val_positive, recommended_list, k_list)
    precision_t, recall_t, hit_t = eval_metrics.evaluate_mp(test_positive, recommended_list, k_list)
    return precision_v, recall_v, hit_v, precision_t, recall_t, hit_t


def NAIS_validation(model, args, num_users, test_positive, val_positive, train_matrix, k_list):
    """validation.py:7-31 (NAIS_basic)."""
    rec = _recommend_ids(model, args, num_users, train_matrix)
    return _metrics(test_positive, val_positive, rec, k_list)


def NAIS_region_validation(model, args, num_users, test_positive, val_positive, train_matrix,
                           businessRegionEmbedList, k_list):
    """validation.py:34-59 (NAIS_regionEmbedding)."""
    rec = _recommend_ids(model, args, num_users, train_matrix, region_of=businessRegionEmbedList)
    return _metrics(test_positive, val_positive, rec, k_list)


def NAIS_region_distance_validation(model, args, num_users, test_positive, val_positive,
                                    train_matrix, businessRegionEmbedList, latlon_mat, k_list,
                                    poi_coords=None):
    """validation.py:62-131 (NAIS_region_distance_Embedding).

    The reference reads (|dlat|, |dlng|) from a P x P x 2 float64 `latlon_mat` (run.py:47-54,214).
    Pass `poi_coords` ([P, 2] lat/lng, the coordinates latlon_mat was built from) to have the
    kernel form the same float64 differences on the fly instead -- bit-identical, and the only
    option at P >= ~50k where the matrix does not fit. `latlon_mat=None` requires poi_coords.
    `args.powerlaw_weight` is read but unused, as at validation.py:66.
    """
    _ = args.powerlaw_weight
    if poi_coords is not None:
        rec = _recommend_ids(model, args, num_users, train_matrix, region_of=businessRegionEmbedList,
                        coords=poi_coords)
    else:
        rec = _recommend_ids(model, args, num_users, train_matrix, region_of=businessRegionEmbedList,
                        latlon_mat=latlon_mat)
    return _metrics(test_positive, val_positive, rec, k_list)


def new4_validation(model, args, num_users, test_positive, val_positive, train_matrix,
                    businessRegionEmbedList, k_list, nearPOI):
    """validation.py:254-280 (New4): the context tables are built once (the reference rebuilds
    them in every 1,024-candidate chunk), then every user's catalog is scored with the basic
    kernels. Differs from the reference only where it breaks: with <= 1,024 candidates the
    reference's chunk loop reads `pred` before assigning it (validation.py:264-266); here such
    users are scored normally."""
    model.eval()
    model.extended_tables(nearPOI)
    rec = _recommend_ids(model, args, num_users, train_matrix)
    return _metrics(test_positive, val_positive, rec, k_list)
