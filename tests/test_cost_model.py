"""CPU test of the pairs route's table / gather CU split (catalog.auto_table_cus): the splits the
measured A/Bs picked (CU split) and the shader-engine granularity."""
import types

import numpy as np

import pytest
import torch

from poi_recommendation_models_amd import catalog
from poi_recommendation_models_amd.catalog import auto_table_cus


def _model(d, h, precision):
    return types.SimpleNamespace(attn_layer1=types.SimpleNamespace(weight=torch.empty(h, d)),
                                 precision=precision)


@pytest.mark.parametrize("precision,prior,want", [
    ("fp16x6", False, 152),   # config 4, the bench default: work queues, 8-CU steps (round 4)
    ("fp16x3", False, 128),   # round 1's split
    ("fp16x6", True, 128),    # the prior doubles the gathered bytes
    ("fp32", False, 192),     # round 3: exact-fp32 tables need the CUs (gather 78 GB/s per CU at 64)
])
def test_config4_splits(precision, prior, want):
    assert auto_table_cus(_model(64, 64, precision), 100_000, 100_000, 5_030_351, 256, prior) == want


def test_config5_split_is_table_heavy():
    # one rank's column shard of the 8-GPU job: 1M distinct history POIs x 125k columns
    assert auto_table_cus(_model(128, 128, "fp16x6"), 1_000_000, 125_000, 20_076_322, 256,
                          block_bytes=1_000_000 * 512 * 8) == 232


@pytest.mark.parametrize("ncu", [64, 128, 256, 304])
def test_split_in_shader_engine_steps(ncu):
    for prior in (False, True):
        for prec in ("fp16x6", "fp16x3"):
            n = auto_table_cus(_model(64, 64, prec), 50_000, 60_000, 1_000_000, ncu, prior)
            # engine-sized steps unless both kernels run as work queues (x6n tables, no prior)
            step = max(1, ncu // 8)
            if prec == "fp16x6" and not prior and catalog.PAIR_WORK_QUEUE:
                step = min(catalog.PAIR_SPLIT_STEP, step)
            assert n % step == 0 and ncu // 4 <= n <= ncu - step


def test_fixed_grid_routes_keep_engine_steps():
    """a job whose gather or table launch keeps a fixed grid (the score-row gather for
    k > 256 or rows_only, transform_attn's nais_dot_pair_table) must not get an 8-CU split step."""
    n = auto_table_cus(_model(64, 64, "fp16x6"), 100_000, 100_000, 5_030_351, 256, False,
                       work_queues=False)
    assert n % 32 == 0, n
    assert n == 160          # the classic engine-sized optimum at config 4


def test_distance_variants_take_the_x6n_steps():
    """din = D + 2 for the distance variants: the split model keys on D (config 4's 152 / 104);
    a non-native width keys on the padded width the kernels run (66 -> 128)."""
    m = _model(66, 64, "fp16x6")
    m.VARIANT = 2            # NAIS_VARIANT_REGION_DISTANCE: D = 64, + the f32 distance K-step
    assert auto_table_cus(m, 100_000, 100_000, 5_030_351, 256, False) == 160
    m.VARIANT = 0            # NAIS_basic at D = 66: padded to 128, twice the table FLOPs
    n = auto_table_cus(m, 100_000, 100_000, 5_030_351, 256, False)
    assert n % 8 == 0 and n > 152


@pytest.mark.parametrize("precision,D,H,mode,want", [
    ("fp16x6", 64, 64, "table", "x6n"),
    ("fp16x6", 64, 64, "direct", "x6n"),
    ("fp16x6_pairsplit", 64, 64, "table", "x6n"),     # pair_table_impl: both fp16x6 -> x6b
    ("fp16x6_pairsplit", 64, 64, "direct", "x3"),     # score_catalog: pairsplit -> launch_catalog_x6
    ("fp16x6", 64, 200, "table", "x6n"),              # 128 < H <= 256 runs on x6n
    ("fp16x6", 128, 256, "direct", "x6n"),
    ("fp16x6", 16, 64, "table", "x3b"),               # D = 16: no x6n instance
    ("fp16x3", 64, 64, "table", "x3b"),
    ("fp16x3_pairsplit", 64, 64, "direct", "x3"),
    ("fp32", 64, 64, "table", "catalog_score_kernel"),
    ("fp16x6", 8, 64, "table", "catalog_score_kernel"),
])
def test_bench_kernel_label_mirrors_dispatch(precision, D, H, mode, want):
    """bench.py's roofline names the kernel nais_kernels.hip dispatches."""
    import bench
    name = bench.table_kernel_name(precision, D, H, mode=mode)
    want = want if want.startswith("catalog") else f"catalog_score_{want}_kernel"
    assert name.split(" ")[0] == want


@pytest.mark.parametrize("world,want", [(1, 190), (2, 190), (4, 186), (8, 180)])
def test_bounded_route_splits_by_shard_width(world, want):
    """The bounded gather's three-term cost (catalog.bounded_gather_cu_seconds): one rank's column
    shard of config 4 (all 50,000 users, P / N columns) pays the per-user and insertion terms on
    fewer bytes, so narrow shards give the gather more CUs (measured best before the shorter
    load chains: 188 / 188 / 180 / 172-180 at N = 1 / 2 / 4 / 8, profiles/r6/split_world; the
    gather is ~7 % cheaper since, profiles/r6/chains_ab); N = 1 keeps 188 because a gather on
    exactly two whole XCDs (192 / 64) lost, profiles/r6/split_n1."""
    NC = (100_000 + world - 1) // world
    n = auto_table_cus(_model(64, 64, "fp16x6"), 100_000, NC, 5_030_351, 256, False,
                       100_000 * 512 * 8, gather_bytes=4, k=50, users=50_000)
    assert n == want


def test_bounded_route_config2_split():
    """Config 2 (10,000 users, h <= 100, 50,000 POIs): 234 / 22 (2-CU steps; 232 / 24 measured
    96.2 ms, profiles/r6/configs); the per-user term prices its short histories."""
    assert auto_table_cus(_model(64, 64, "fp16x6"), 49_999, 50_000, 505_318, 256, False,
                          49_999 * 512 * 8, gather_bytes=4, k=50, users=10_000) == 234


def test_bounded_gather_cost_fit():
    """The fit reproduces the measured launches within 3 %: config 4 at N = 1 and one rank of
    N = 8 (2.168 ms x 68 CUs, 2.28 ms x 80 CUs per launch, profiles/r6/chains_ab)."""
    from poi_recommendation_models_amd.catalog import bounded_gather_cu_seconds
    for NC, cu_ms in ((100_000, 2.168 * 68), (12_500, 2.28 * 80)):
        per_launch = bounded_gather_cu_seconds(5_030_351, NC, 50_000, 50) / np.ceil(NC / 512)
        assert abs(per_launch * 1e3 / cu_ms - 1) < 0.03, (NC, per_launch)


def test_region_distance_bounded_split():
    """bench.py's region_distance leg on the bounded route: 194 / 62 (measured 514.2 / 516.6 ms
    against 522.6 / 524.4 at 196 / 60 and 530 at 190 / 66, profiles/r6/rd_split)."""
    m = _model(66, 64, "fp16x6")
    m.VARIANT = 2            # NAIS_VARIANT_REGION_DISTANCE
    assert auto_table_cus(m, 100_000, 100_000, 5_030_351, 256, False, 100_000 * 512 * 8,
                          gather_bytes=4, k=50, users=50_000) == 194
