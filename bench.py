#!/usr/bin/env python3
"""Benchmark: full-catalog NAIS scoring + top-50, scored (user, POI) pairs/s (BASELINE.json metric).

Workload (BASELINE.json configs[3], the "100k POIs" metric config): synthetic Gowalla-scale
check-ins, 50k users x 100k POIs, d = H = 64, h_u ~ U{1..200}, k = 50, NAIS_basic.
Inputs (tables, CSR, user lists) are resident in HBM before the timed region.

Strategy "pairs" (default for config 4): a step = the WHOLE job -- every user's
complete catalog scored and its top-50 formed. The per-(history POI, candidate) terms are computed
once (nais_pair_table: the split-fp16 MFMA catalog kernel in table mode), every user's sums are
gathered from those tables (nais_pair_gather, HBM-bound), then top-50 (nais_topk_rows). N > 1:
rank r owns POIs [r*P/N, (r+1)*P/N) for all users (tables, gathers, local top-50), then one RCCL
all-gather of the [users, 50] blocks and a merge (sharding.distributed_topk_pairs) -- the total
work is fixed as N grows -> strong scaling.

Strategy "direct" (config 5, or --strategy direct): a step = `--users-per-step` users per GPU,
each user's catalog scored against its whole history by the fused kernel (nais_score_catalog) +
top-50; users sharded across ranks by LPT, tables replicated (RCCL broadcast) -> weak scaling.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix peak (dense), spec
PEAK_F16_MFMA_TFLOPS = 2500.0   # MI355X_MICROARCH.md: BF16/F16 MFMA dense peak, spec
# the fp16x3 path issues 3 f16 MFMA products per algorithmic fp32 product, so its roof in
# algorithmic (fp32-equivalent) FLOP/s is the f16 dense peak / 3
PEAKS = {"fp32": PEAK_FP32_MFMA_TFLOPS, "fp16x3": PEAK_F16_MFMA_TFLOPS / 3,
         "fp16x3_pairsplit": PEAK_F16_MFMA_TFLOPS / 3}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", type=int, default=4, choices=[4, 5],
                    help="4: 50k users x 100k POIs, d=H=64 (the metric config); 5: stress, 200k users x "
                         "1M POIs, d=H=128, tables sharded + all-gathered, timed on the first 4096 users")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--users-per-step", type=int, default=256)
    ap.add_argument("--num-users", type=int, default=50_000)
    ap.add_argument("--num-pois", type=int, default=100_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--h-max", type=int, default=200)
    ap.add_argument("--topk", type=int, default=50)
    ap.add_argument("--precision", default="fp16x3", choices=["fp32", "fp16x3", "fp16x3_pairsplit"])
    ap.add_argument("--no-fp32-leg", action="store_true",
                    help="skip the extra exact-fp32 timing reported under 'fp32_path'")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL on ROCm) for real runs; gloo to rehearse N>1 on one GPU")
    ap.add_argument("--strategy", default="auto", choices=["auto", "pairs", "direct"],
                    help="auto: pairs for config 4 (each (item, candidate) pair shared by ~50 users), "
                         "direct for config 5's 4096-user subset (sharing ~1)")
    return ap.parse_args()


def cpu_baseline(p, data, users, k, seconds):
    """The CPU restatement (oracle, numpy fp32 + BLAS threads) on a bounded user sample."""
    from oracle import nais_oracle
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        cores = os.cpu_count()
    pairs, t0, n = 0, time.perf_counter(), 0
    for u in users:
        cand, sc = nais_oracle.catalog_scores_basic(p, data.history(int(u)), data.num_pois)
        nais_oracle.topk_ids(cand, sc, k)
        pairs += len(cand)
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": pairs / dt, "unit": "pairs/s", "cores": int(cores), "kind": "port",
            "sample": f"{n} users of the same workload (complement candidates + chunked forward + "
                      f"top-{k}, oracle/nais_oracle.py numpy fp32), {pairs} pairs in {dt:.1f} s"}


def main():
    a = parse()
    if a.config == 5:
        a.num_users, a.num_pois, a.dim, a.hidden = 200_000, 1_000_000, 128, 128
        if a.users_per_step == 256:
            a.users_per_step = 64
        a.no_cpu_baseline = True   # the CPU leg is quoted on the metric config (4)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    import torch.distributed as dist
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from poi_recommendation_models_amd import _capi
    from poi_recommendation_models_amd.catalog import DeviceCSR
    from poi_recommendation_models_amd.model import NAIS_basic
    from poi_recommendation_models_amd.sharding import broadcast_module, shard_users
    from poi_recommendation_models_amd.synthetic import init_nais_params, make_checkins

    P, D, H, K = a.num_pois, a.dim, a.hidden, a.topk
    data = make_checkins(a.num_users, P, a.h_max, seed=2024)
    model = NAIS_basic(P, D, H, 0.5)
    p_host = None
    gather_ms = None
    if a.config == 5:
        # every rank materialises 1/N of each POI table, then one all-gather per table (RCCL ring
        # over xGMI); rows come from per-65536-row-chunk seeds so the table is N-independent
        from poi_recommendation_models_amd.sharding import load_sharded_tables
        model = model.to(dev).eval()
        mlp = init_nais_params(8, D, H, seed=7, emb_std=0.3, bias_std=0.1)

        def rows(name, s0, e0):
            out = torch.empty(max(e0 - s0, 0), D)
            c0 = s0 // 65536
            while c0 * 65536 < e0:
                g = torch.Generator().manual_seed(1000 * (name == "embed_target") + c0)
                chunk = torch.randn(65536, D, generator=g) * 0.3
                lo, hi = max(s0, c0 * 65536), min(e0, (c0 + 1) * 65536)
                out[lo - s0:hi - s0] = chunk[lo - c0 * 65536:hi - c0 * 65536]
                c0 += 1
            return out
        with torch.no_grad():
            for k in ("attn_layer1.weight", "attn_layer1.bias", "attn_layer2.weight"):
                dict(model.named_parameters())[k].copy_(torch.from_numpy(mlp[k]))
        if world > 1:
            torch.cuda.synchronize(dev)
            dist.barrier()
            t0 = time.perf_counter()
            load_sharded_tables(model, rows)
            torch.cuda.synchronize(dev)
            gather_ms = (time.perf_counter() - t0) * 1e3
        else:
            with torch.no_grad():
                model.embed_history.weight.copy_(rows("embed_history", 0, P))
                model.embed_target.weight.copy_(rows("embed_target", 0, P))
        if rank == 0:
            p_host = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    else:
        if rank == 0:
            p_host = init_nais_params(P, D, H, seed=7, emb_std=0.3, bias_std=0.1)
            model.load_state_dict({k: torch.from_numpy(v) for k, v in p_host.items()}, strict=False)
        model = model.to(dev).eval()
        if world > 1:   # replicate the POI tables + MLP over RCCL (xGMI), once
            broadcast_module(model, src=0)
    model.report_nan = False
    model.precision = a.precision
    csr = DeviceCSR.from_arrays(data.indptr, data.indices, P, dev)
    hist_len = data.hist_len()
    strategy = a.strategy if a.strategy != "auto" else ("pairs" if a.config == 4 else "direct")
    if strategy == "pairs":
        return bench_pairs(a, model, csr, data, hist_len, p_host, dev, rank, world, dist)
    subset = np.arange(4096) if a.config == 5 else None
    mine = shard_users(hist_len, P, world, users=subset)[rank]
    if a.config == 5:   # the fixed 4096-user subset is the whole timed job: steps cover it once
        a.steps = max(1, len(mine) // a.users_per_step)
        a.warmup = min(a.warmup, 1)
    rng = np.random.default_rng(100 + rank)
    rng.shuffle(mine)                      # every step is a representative sample of h_u
    B = a.users_per_step
    nsteps = a.warmup + a.steps
    steps = []
    for s in range(nsteps):
        us = np.take(mine, np.arange(s * B, (s + 1) * B), mode="wrap")
        c = (P - hist_len[us]) * hist_len[us]
        us = us[np.argsort(-c, kind="stable")]          # heavy users dispatched first
        steps.append((torch.from_numpy(us.astype(np.int32)).to(dev),
                      int((P - hist_len[us]).sum()),
                      int(((P - hist_len[us]) * hist_len[us]).sum())))
    lib = _capi.load()
    scores = torch.empty(B, P, dtype=torch.float32, device=dev)
    ids = torch.empty(B, K, dtype=torch.int32, device=dev)
    top = torch.empty(B, K, dtype=torch.float32, device=dev)
    cnt = torch.zeros(2, dtype=torch.int32, device=dev)
    gat_ids = torch.empty(world * B, K, dtype=torch.int32, device=dev) if world > 1 else None
    gat_sc = torch.empty(world * B, K, dtype=torch.float32, device=dev) if world > 1 else None
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def run(precision, nwarm, nsteps):
        """nwarm untimed + nsteps timed steps; returns (elapsed s, catalog ms list, topk ms list)."""
        model.precision = precision
        prm = model.nais_params()

        def step(s, ev=None):
            u_dev = steps[s][0]
            if ev is not None:
                ev[0].record(stream)
            _capi.check(lib.nais_score_catalog(prm, csr.indptr.data_ptr(), csr.indices.data_ptr(),
                                               u_dev.data_ptr(), B, None, None, None,
                                               scores.data_ptr(), P, cnt[0:1].data_ptr(), sh),
                        "score_catalog")
            if ev is not None:
                ev[1].record(stream)
            _capi.check(lib.nais_topk_rows(scores.data_ptr(), P, P, B, K, ids.data_ptr(),
                                           top.data_ptr(), cnt[1:2].data_ptr(), sh), "topk_rows")
            if ev is not None:
                ev[2].record(stream)
            if world > 1:   # the per-step exchange: every rank's top-k blocks
                if a.backend == "nccl":
                    dist.all_gather_into_tensor(gat_ids, ids)
                    dist.all_gather_into_tensor(gat_sc, top)
                else:
                    dist.all_gather(list(gat_ids.chunk(world)), ids)
                    dist.all_gather(list(gat_sc.chunk(world)), top)

        for s in range(nwarm):
            step(s)
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(nsteps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(nsteps):
            step(nwarm + i, evs[i])
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        return (el, [e[0].elapsed_time(e[1]) for e in evs], [e[1].elapsed_time(e[2]) for e in evs])

    elapsed, score_ms, topk_ms = run(a.precision, a.warmup, a.steps)
    pairs = sum(steps[a.warmup + i][1] for i in range(a.steps))
    work = sum(steps[a.warmup + i][2] for i in range(a.steps))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        pt = torch.tensor([pairs], dtype=torch.float64, device=dev)
        dist.all_reduce(pt)
        pairs_total = float(pt.item())
    else:
        pairs_total = float(pairs)

    flop_per_pair_item = 2 * D * H + 3 * H + 4 * D
    flops = work * flop_per_pair_item / a.steps          # algorithmic FLOP per catalog launch
    avg_score_s = float(np.mean(score_ms)) / 1e3
    achieved = flops / avg_score_s / 1e12
    peak = PEAKS[a.precision]
    traffic = None
    try:
        tj = json.load(open(a.traffic_json)).get(a.precision, {})
        if tj.get("users_per_launch") == B and tj.get("num_pois") == P and tj.get("dim") == D:
            traffic = tj.get("hbm_bytes_per_launch")
    except Exception:
        pass
    fp32_leg = None
    if world == 1 and not a.no_fp32_leg and a.precision != "fp32":
        n32 = min(a.steps, 3)
        el32, sm32, _ = run("fp32", 1, n32)
        p32 = sum(steps[1 + i][1] for i in range(n32))
        w32 = sum(steps[1 + i][2] for i in range(n32)) * flop_per_pair_item / n32
        ach32 = w32 / (float(np.mean(sm32)) / 1e3) / 1e12
        fp32_leg = {"precision": "fp32 (v_mfma_f32_32x32x2_f32, exact fp32)", "value": p32 / el32,
                    "unit": "pairs/s", "steps": n32, "achieved": ach32, "peak": PEAK_FP32_MFMA_TFLOPS,
                    "frac": ach32 / PEAK_FP32_MFMA_TFLOPS, "avg_launch_ms": float(np.mean(sm32))}
    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            cpu = cpu_baseline(p_host, data, mine[:64], K, a.cpu_seconds)
        out = {
            "metric": "scored (user,POI) pairs/sec full-catalog + top-50, %s POIs"
                      % ("100k" if a.config == 4 else "1M"),
            "value": pairs_total / elapsed,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if a.precision == "fp32" else
                     "fp32 (W1 x products as 3 fp16 MFMA products of power-of-two-scaled hi/lo splits, fp32 accumulate)",
            "data": "synthetic (seeded CSR check-ins, h~U{1..%d}; random-init weights N(0,0.3))" % a.h_max,
            "config": {
                "workload": ("config4 Gowalla-scale" if a.config == 4 else
                             "config5 stress (timed on the first 4096 users)") +
                            ": %d users x %d POIs, d=H=%d, full-catalog NAIS_basic score + top-%d"
                            % (a.num_users, P, D, K),
                "table_allgather_ms": gather_ms,
                "model": "NAIS_basic", "users_per_step_per_gpu": B, "num_pois": P,
                "embed_dim": D, "hidden": H, "h_max": a.h_max, "topk": K,
                "pairs_per_step_per_gpu": pairs / a.steps,
                "parallelism": f"users sharded (LPT) over {world} GPU(s), POI tables replicated",
            },
            "roofline": {
                "kernel": ("catalog_score_kernel" if a.precision == "fp32" else
                           "catalog_score_x3b_kernel" if (D <= 64 and H <= 64 and a.precision == "fp16x3")
                           else "catalog_score_x3_kernel") + " (nais_score_catalog)",
                "bound": "mfma",
                "achieved": achieved,
                "peak": peak,
                "peak_basis": ("fp32 MFMA dense" if a.precision == "fp32" else
                               "f16 MFMA dense 2.5 PF / 3 products per algorithmic fp32 product"),
                "unit": "TFLOP/s",
                "frac": achieved / peak,
                "traffic": traffic,
                "algorithmic_flop_per_launch": flops,
                "avg_launch_ms": avg_score_s * 1e3,
                "topk_avg_launch_ms": float(np.mean(topk_ms)),
            },
            "cpu_baseline": cpu,
            "fp32_path": fp32_leg,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_pairs(a, model, csr, data, hist_len, p_host, dev, rank, world, dist):
    """Whole-job steps through sharding.distributed_topk_pairs (the product path)."""
    from poi_recommendation_models_amd import catalog
    from poi_recommendation_models_amd.sharding import distributed_topk_pairs
    if os.environ.get("NAIS_PAIR_TABLE_CUS"):          # A/B knobs of the table/gather overlap
        catalog.PAIR_TABLE_CUS = int(os.environ["NAIS_PAIR_TABLE_CUS"])
    if os.environ.get("NAIS_PAIR_CU_LAYOUT"):
        catalog.PAIR_CU_LAYOUT = os.environ["NAIS_PAIR_CU_LAYOUT"]
    if os.environ.get("NAIS_PAIR_BLOCK_COLS"):
        catalog.PAIR_BLOCK_COLS = int(os.environ["NAIS_PAIR_BLOCK_COLS"])
    for knob in ("PAIR_FUSED_TOPK", "PAIR_LPT_ORDER"):
        if os.environ.get("NAIS_" + knob):
            setattr(catalog, knob, os.environ["NAIS_" + knob] == "1")
    if os.environ.get("NAIS_PAIR_TABLE_GATHER_FRAC"):
        catalog.PAIR_TABLE_GATHER_FRAC = float(os.environ["NAIS_PAIR_TABLE_GATHER_FRAC"])
    if os.environ.get("NAIS_PAIR_FIRST_TABLE_ALL_CUS"):
        catalog.PAIR_FIRST_TABLE_ALL_CUS = os.environ["NAIS_PAIR_FIRST_TABLE_ALL_CUS"] == "1"
    # NAIS_EMULATE_WORLD=N (one process): time rank 0's column shard of an N-GPU run (its tables,
    # gathers and local top-k; no collective) -- per-rank cost and strong-scaling headroom on one GPU
    emulate = int(os.environ.get("NAIS_EMULATE_WORLD", "1"))
    P, D, H, K = a.num_pois, a.dim, a.hidden, a.topk
    users = np.arange(a.num_users)
    group = None
    if world == 1:   # the same code path with a trivial process group is not needed: call direct
        from poi_recommendation_models_amd.catalog import _score_topk_pairs

        S_em = (a.num_pois + emulate - 1) // emulate

        def job(events=None):
            return _score_topk_pairs(model, csr, users, K, None, None, None, None, force=True,
                                     events=events, cols=(0, S_em) if emulate > 1 else None)
    else:
        def job(events=None):
            return distributed_topk_pairs(model, csr, users, K, group=group, events=events)

    def run(precision, nwarm, nsteps):
        model.precision = precision
        for _ in range(nwarm):
            job()
        evs = [[] for _ in range(nsteps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(nsteps):
            job(evs[i])
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        per, nl = {}, {}
        for step_ev in evs:
            for kind, e0, e1, launches in step_ev:
                if e0 is None:          # a setting, not a timed launch
                    per[kind] = launches
                    continue
                per.setdefault(kind, []).append(e0.elapsed_time(e1))
                nl[kind] = nl.get(kind, 0) + launches
        per["_launches"] = nl
        return el, per

    elapsed, per = run(a.precision, a.warmup, a.steps)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    pairs_job = float((P - hist_len[users]).sum())            # every user's whole catalog
    S = (P + world - 1) // world
    if emulate > 1 and world == 1:
        S = (P + emulate - 1) // emulate
        pairs_job /= emulate     # ~ the shard's share (value is then a per-rank rate estimate)
    c0, c1 = min(rank * S, P), min((rank + 1) * S, P)
    NC = c1 - c0
    entries = int(hist_len.sum())
    J = int(np.count_nonzero(np.bincount(data.indices, minlength=P)))
    # algorithmic work per step on this rank
    fused = catalog.PAIR_FUSED_TOPK and K <= 256
    Wb, st_w = catalog.PAIR_BLOCK_COLS, catalog.PAIR_STRIPE
    stripes = sum((min(Wb, NC - b) + st_w - 1) // st_w for b in range(0, NC, Wb))
    # table rows (8 B per history entry x column) + each stripe's CSR ids and row map (12 B per
    # entry) + score rows (4 B per user x column; the fused kernel writes only the top-k merges)
    gather_bytes = entries * NC * 8 + entries * 12 * stripes + (0 if fused else a.num_users * NC * 4)
    # the timed gather launches are the gather stream's: with PAIR_TABLE_GATHER_FRAC > 0 the table
    # stream gathers the tail users, so count only the gather stream's share of the entries
    gather_bytes *= per.get("gather_share", 1.0)
    flop_per_pair_item = 2 * D * H + 3 * H + 4 * D
    table_flops = J * NC * flop_per_pair_item
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    table_cus = per.get("table_cus", ncu) or ncu
    g_ms = sum(per.get("gather", [])) / a.steps
    t_ms = sum(per.get("table", [])) / a.steps
    k_ms = sum(per.get("topk", [])) / a.steps
    n_gl = max(1, per["_launches"].get("gather", 0) // a.steps)
    achieved = gather_bytes / (g_ms * 1e-3) / 1e9
    traffic = None
    try:
        tj = json.load(open(a.traffic_json)).get("pairs_gather_topk" if fused else "pairs_gather", {})
        if (tj.get("num_users") == a.num_users and tj.get("num_pois") == P and tj.get("world") == world
                and tj.get("block_cols") == catalog.PAIR_BLOCK_COLS):
            traffic = tj.get("hbm_bytes_per_launch")
    except Exception:
        pass
    fp32_leg = None
    if world == 1 and not a.no_fp32_leg and a.precision != "fp32":
        el32, per32 = run("fp32", 0, 1)
        t32 = sum(per32.get("table", []))
        fp32_leg = {"precision": "fp32 (v_mfma_f32_32x32x2_f32 tables, exact fp32)", "value": pairs_job / el32,
                    "unit": "pairs/s", "steps": 1, "table_ms": t32,
                    "table_tflops": table_flops / (t32 * 1e-3) / 1e12, "peak": PEAK_FP32_MFMA_TFLOPS}
        model.precision = a.precision
    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            rng = np.random.default_rng(100)
            cpu = cpu_baseline(p_host, data, rng.choice(users, 64, replace=False), K, a.cpu_seconds)
        out = {
            "metric": "scored (user,POI) pairs/sec full-catalog + top-50, 100k POIs",
            "value": pairs_job * a.steps / elapsed,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32" if a.precision == "fp32" else
                     "fp32 (W1 x products as 3 fp16 MFMA products of power-of-two-scaled hi/lo splits, fp32 accumulate)",
            "data": "synthetic (seeded CSR check-ins, h~U{1..%d}; random-init weights N(0,0.3))" % a.h_max,
            "config": {
                "workload": "config4 Gowalla-scale: %d users x %d POIs, d=H=%d, full-catalog NAIS_basic "
                            "score + top-%d; one step = every user's whole catalog" % (a.num_users, P, D, K),
                "model": "NAIS_basic", "strategy": "pairs", "num_users": a.num_users, "num_pois": P,
                "table_cus": table_cus, "cu_layout": catalog.PAIR_CU_LAYOUT,
                "block_cols": catalog.PAIR_BLOCK_COLS,
                "first_table_all_cus": catalog.PAIR_FIRST_TABLE_ALL_CUS,
                "table_gather_frac": catalog.PAIR_TABLE_GATHER_FRAC,
                "fused_topk": catalog.PAIR_FUSED_TOPK, "lpt_order": catalog.PAIR_LPT_ORDER,
                **({"emulated_world_shard": emulate} if emulate > 1 and world == 1 else {}),
                "embed_dim": D, "hidden": H, "h_max": a.h_max, "topk": K,
                "pairs_per_step": pairs_job, "history_entries": entries, "distinct_history_pois": J,
                "parallelism": f"POI columns sharded over {world} GPU(s) (all users per rank), "
                               "tables replicated, one all-gather + merge of the top-k blocks",
            },
            "roofline": {
                "kernel": "pair_gather_topk_kernel (nais_pair_gather_topk)" if fused else
                          "pair_gather_kernel (nais_pair_gather)",
                "bound": "hbm",
                "achieved": achieved,
                "peak": 8000.0,
                "unit": "GB/s",
                "frac": achieved / 8000.0,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": gather_bytes / n_gl,
                "avg_launch_ms": g_ms / n_gl,
                "launches_per_step": n_gl,
                "note": "algorithmic bytes per launch (one 256-column stripe for the fused kernel) = "
                        "sum_u h_u x columns x 8 B table reads + 12 B CSR id + row map per history "
                        "entry (+ 4 B score writes per user x column, non-fused); traffic = "
                        "rocprofv3 (2 x FETCH_SIZE + WRITE_SIZE) per launch, Infinity-Cache hits "
                        "included",
                "overlap": "tables on CUs [0, %d) and gathers on the other %d, side by side on "
                           "CU-masked streams (double-buffered tables)" % (table_cus, ncu - table_cus)
                           if table_cus < ncu else "serial",
                "table_kernel": {"name": "catalog_score_x3b_kernel in table mode (nais_pair_table)",
                                 "bound": "mfma", "ms_per_step": t_ms, "cus": table_cus,
                                 "frac_of_its_cus": (table_flops / (t_ms * 1e-3) / 1e12) /
                                                    (PEAKS[a.precision] * table_cus / ncu) if t_ms else None,
                                 "achieved_tflops": table_flops / (t_ms * 1e-3) / 1e12 if t_ms else None,
                                 "peak_tflops": PEAKS[a.precision],
                                 "frac": (table_flops / (t_ms * 1e-3) / 1e12) / PEAKS[a.precision] if t_ms else None},
                "topk_ms_per_step": k_ms,
            },
            "cpu_baseline": cpu,
            "fp32_path": fp32_leg,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
