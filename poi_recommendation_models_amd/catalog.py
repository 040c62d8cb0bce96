"""Full-catalog scoring + top-k on the device (the per-user body of validation.py:11-27).

`score_topk` replaces, for a whole set of users at once:
  get_NAIS_batch_test(train_matrix, u)   batches.py:52-65   (complement candidates, C_u x h int64 matrix, H2D)
  chunked model(user_history, target)    validation.py:14-22 (1,024-row forward chunks, NaN .item() per chunk)
  torch.topk(pred, k) + 50 .item()       validation.py:26-27
with one `nais_score_topk` call: the user's CSR row is read on the device, every POI of the
catalog is scored by the fused kernel (history POIs excluded), and a radix-select top-k runs
per user. Nothing per-candidate crosses PCIe.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _capi


class DeviceCSR:
    """train_matrix (scipy CSR, users x POIs) resident on the device as int64 indptr/indices."""

    def __init__(self, train_matrix, device):
        X = train_matrix.tocsr() if not hasattr(train_matrix, "indptr") else train_matrix
        if not X.has_sorted_indices:   # rows ascending (the batch builder binary-searches them)
            X = X.sorted_indices()
        self.shape = X.shape
        self.host_indptr = np.asarray(X.indptr, dtype=np.int64)
        self.host_indices = np.asarray(X.indices, dtype=np.int64)
        self.hist_len = np.diff(self.host_indptr)
        self.indptr = torch.from_numpy(self.host_indptr).to(device)
        self.indices = torch.from_numpy(self.host_indices).to(device)
        self.device = device
        self.key = (id(train_matrix), X.shape, X.nnz)

    @classmethod
    def from_arrays(cls, indptr, indices, num_pois, device):
        import scipy.sparse as sp
        X = sp.csr_matrix((np.ones(len(indices)), np.asarray(indices), np.asarray(indptr)),
                          shape=(len(indptr) - 1, num_pois))
        return cls(X, device)


_csr_cache: dict = {}
_ws_cache: dict = {}


def _user_array(users):
    """User ids as int64 numpy (an ndarray or range without a per-element Python round trip)."""
    if isinstance(users, (np.ndarray, range)):
        return np.asarray(users, dtype=np.int64).reshape(-1)
    return np.asarray(list(users), dtype=np.int64)


def device_csr(train_matrix, device) -> DeviceCSR:
    if isinstance(train_matrix, DeviceCSR):
        return train_matrix
    X = train_matrix
    key = (id(X), X.shape, X.nnz, str(device))
    hit = _csr_cache.get(key)
    if hit is None or hit[0] is not X:
        _csr_cache.clear()
        hit = (X, DeviceCSR(X, device))
        _csr_cache[key] = hit
    return hit[1]


def _workspace(device, nbytes):
    ws = _ws_cache.get(str(device))
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        _ws_cache[str(device)] = ws
    return ws


def lpt_order(users, hist_len, num_pois):
    """Users sorted by descending cost (P - h_u) * h_u: heaviest workgroups are dispatched first."""
    users = np.asarray(users, dtype=np.int64)
    h = hist_len[users]
    cost = (num_pois - h) * h
    return users[np.argsort(-cost, kind="stable")]


def _side_inputs(model, dev, region_of, coords, latlon_mat):
    reg = cor = llm = None
    if model.VARIANT in (_capi.VARIANT_REGION, _capi.VARIANT_REGION_DISTANCE):
        if region_of is None:
            raise ValueError("region variants need businessRegionEmbedList (POI -> region)")
        reg = torch.as_tensor(np.asarray(region_of, dtype=np.int64)).to(dev)
    if model.VARIANT in (_capi.VARIANT_REGION_DISTANCE, _capi.VARIANT_DISTANCE):
        if coords is not None:
            cor = torch.as_tensor(np.ascontiguousarray(coords, dtype=np.float64)).to(dev)
        elif latlon_mat is not None:
            llm = torch.as_tensor(np.ascontiguousarray(latlon_mat, dtype=np.float64)).to(dev)
        else:
            raise ValueError("region_distance needs poi coords (or the reference latlon_mat)")
    return reg, cor, llm


def score_catalog(model, train_matrix, users, region_of=None, coords=None, latlon_mat=None,
                  strategy="direct"):
    """Full score rows f32 [len(users), P] (history POIs = -1.0), via nais_score_catalog
    (strategy "direct") or the pair tables (strategy "pairs", nais_pair_*)."""
    if strategy == "pairs" or model._pairs_only:
        return _score_topk_pairs(model, train_matrix, users, 1, region_of, coords, latlon_mat,
                                 None, force=True, rows_only=True)
    dev = model._check_device()
    csr = device_csr(train_matrix, dev)
    P = model._item_tables()[0].shape[0]
    users = _user_array(users)
    u_dev = torch.from_numpy(users.astype(np.int32)).to(dev)
    reg, cor, llm = _side_inputs(model, dev, region_of, coords, latlon_mat)
    out = torch.empty(len(users), P, dtype=torch.float32, device=dev)
    nan = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = _capi.load().nais_score_catalog(model._score_params(), csr.indptr.data_ptr(),
                                         csr.indices.data_ptr(), u_dev.data_ptr(), len(users),
                                         _capi.ptr(reg), _capi.ptr(cor), _capi.ptr(llm),
                                         out.data_ptr(), P, nan.data_ptr(), _capi.stream_handle(dev))
    _capi.check(rc, "nais_score_catalog")
    model._last_nan = nan
    return out


# "pairs" strategy (include/nais.h): worth it when the listed users' history entries outnumber
# their distinct history POIs by this factor (each (item, candidate) pair is then reused by that
# many users on average); below it, the direct per-user kernels do less work.
PAIR_MIN_SHARING = 3.0
PAIR_MEMORY_FRACTION = 0.6      # of the device's free memory, for the tables + score rows


def score_topk(model, train_matrix, users, k, region_of=None, coords=None, latlon_mat=None,
               ordered=True, stream=None, prior=None, strategy=None, _on_caller_stream=False):
    """Top-k (ids int64 [len(users), k], scores f32) of every listed user over its complement
    candidates, ordered (score desc, POI id asc). Raises like torch.topk when a user has fewer
    than k candidates (validation.py:26).

    `prior` = (a, b, alpha, poi_coords): rank on the power-law-blended score
    f32((1-alpha) * score) + alpha * G / max G instead (run.py:537-539, powerLaw.py:86-92).

    `strategy` (default: the model's `catalog_strategy`, "auto"): "direct" runs the fused per-user
    kernels; "pairs" computes each (distinct history POI, candidate) term once and gathers every
    user's sums from those tables (nais_pair_*; with a prior also the pr_d(dist) table and each
    user's float64 product G, nais_pair_prior_*); "auto" picks "pairs" when the users' history
    entries outnumber their distinct POIs by PAIR_MIN_SHARING.

    `stream` (a raw hipStream_t handle): the whole call -- its allocations, uploads, kernels and
    the final reorder -- runs on that stream, which first waits for the caller's current stream;
    the current stream then waits for it before the results are returned. The pairs route then
    stays on that stream alone (no CU-masked side streams), so work the caller confined to a
    CU-masked stream stays on those CUs."""
    dev = model._check_device()
    if stream is not None:
        ext = torch.cuda.ExternalStream(stream, device=dev)
        cur = torch.cuda.current_stream(dev)
        ext.wait_stream(cur)
        with torch.cuda.stream(ext):
            out = score_topk(model, train_matrix, users, k, region_of, coords, latlon_mat, ordered,
                             None, prior, strategy, _on_caller_stream=True)
        cur.wait_stream(ext)
        for t in out:
            t.record_stream(cur)
        return out
    strategy = strategy or getattr(model, "catalog_strategy", "auto")
    if strategy not in ("auto", "direct", "pairs"):
        raise ValueError(f"unknown strategy {strategy!r}")
    if model._pairs_only:
        if prior is not None:
            raise NotImplementedError(f"{type(model).__name__}: no power-law prior on its catalog path")
        strategy = "pairs"
    if strategy != "direct":
        got = _score_topk_pairs(model, train_matrix, users, k, region_of, coords, latlon_mat,
                                stream, force=strategy == "pairs", prior=prior,
                                no_side_streams=_on_caller_stream)
        if got is not None:
            return got
    csr = device_csr(train_matrix, dev)
    P = model._item_tables()[0].shape[0]
    if csr.shape[1] != P:
        raise ValueError(f"train_matrix has {csr.shape[1]} POIs, model has {P}")
    users = _user_array(users)
    if len(users) == 0:
        return (torch.empty(0, k, dtype=torch.int64, device=dev),
                torch.empty(0, k, dtype=torch.float32, device=dev))
    if np.any(P - csr.hist_len[users] < k):
        raise RuntimeError("selected index k out of range")       # torch.topk's error
    order = lpt_order(users, csr.hist_len, P) if ordered else users
    u_dev = torch.from_numpy(order.astype(np.int32)).to(dev)
    reg, cor, llm = _side_inputs(model, dev, region_of, coords, latlon_mat)
    n = len(order)
    ids = torch.empty(n, k, dtype=torch.int32, device=dev)
    sc = torch.empty(n, k, dtype=torch.float32, device=dev)
    counters = torch.zeros(2, dtype=torch.int32, device=dev)
    lib = _capi.load()
    prm = model._score_params()
    pri, pri_coords = None, None
    if prior is not None:
        pa, pb, alpha, pc = prior
        pri_coords = torch.as_tensor(np.ascontiguousarray(pc, dtype=np.float64)).to(dev)
        prior_flags = _capi.PRIOR_FINITE if _prior_entries_finite(pa, pb) else 0
        pri = _capi.NaisPrior(float(pa), float(pb), float(alpha), pri_coords.data_ptr())
    nbytes = lib.nais_score_topk_workspace_size(prm, n, k, int(prior is not None))
    ws = _workspace(dev, nbytes)
    st = stream if stream is not None else _capi.stream_handle(dev)
    rc = lib.nais_score_topk(prm, csr.indptr.data_ptr(), csr.indices.data_ptr(), u_dev.data_ptr(),
                             n, k, _capi.ptr(reg), _capi.ptr(cor), _capi.ptr(llm),
                             None if pri is None else ctypes.byref(pri),
                             ids.data_ptr(), sc.data_ptr(), counters[0:1].data_ptr(),
                             counters[1:2].data_ptr(), ws.data_ptr(), ws.numel(), st)
    _capi.check(rc, "nais_score_topk")
    model._last_nan = counters[0:1]
    if ordered:
        inv = np.empty(n, dtype=np.int64)
        pos = {int(u): i for i, u in enumerate(order)}
        inv[:] = [pos[int(u)] for u in users]
        inv_t = torch.from_numpy(inv).to(dev)
        ids, sc = ids.index_select(0, inv_t), sc.index_select(0, inv_t)
    return ids.to(torch.int64), sc


# Column-block width of the pair tables. Serial (profiles/r1/pairs/): 8192 best of 1024 / 8192 /
# 100000. Overlapped (below; profiles/r1/overlap/): 1024 / 2048 / 3072 / 4096 / 8192 columns ->
# 606 / 610 / 619 / 627 / 665 ms per config-4 step (a shorter pipeline fill). With block 0's table
# on every CU (profiles/r1/blocks/): 1024 vs 2048 -> 579.8 vs 581.3 ms at N = 1, and on one rank's
# column shard of an 8-GPU run (12.5k columns) 512 / 1024 / 2048 -> 77.2 / 77.7 / 79.9 ms. With the
# fused top-k, longest-first users and no host syncs (profiles/r1/blocks2/): 256 / 512 / 1024 ->
# 545.9 / 546.0 / 548.0 ms at N = 1 and 71.5 / 72.3 / 73.3 ms on the 8-GPU shard, where 256 brings
# the tables (65.8 ms on half the CUs) close to the gathers (67.7 ms): 512 keeps a margin.
PAIR_BLOCK_COLS = 512
# Table (MFMA-bound) and gather (HBM-bound) phases of consecutive column blocks run side by side
# on CU-masked streams: tables on CUs [0, PAIR_TABLE_CUS), gathers on the rest (-1 = half the
# device's CUs, i.e. 4 of the 8 XCDs each; 0 = serial on the caller's stream). Double-buffered
# tables. Config-4 A/B at 8192 columns (profiles/r1/overlap/): serial 859-874 ms/step; 96 / 112 /
# 128 / 144 / 160 / 192 table CUs -> 694 / 695 / 665 / 794 / 772 / 1085 ms (splits off XCD
# boundaries lose; masks that interleave CU ids are not honoured -- both kernels then share
# every CU).
PAIR_TABLE_CUS = -1
PAIR_FIRST_TABLE_ALL_CUS = True   # block 0's table (nothing to overlap it with) on every CU
# (The mirror image -- the last block's gather on every CU behind its table -- was neutral: config 4
# 475.3 / 476.9 vs 475.5 / 475.7 ms, one rank of N = 8 76.0 / 76.7 vs 76.0 / 75.6 ms, interleaved on
# one box, profiles/r6/last_gather_ab; not kept.)
# Fused gather + running top-k (nais_pair_gather_topk): each user keeps its best k keys while the
# stripes stream by, so no [users, P] score rows are formed and no top-k pass reads them back
# (k <= 256, models without a post-gather score fixup).
PAIR_FUSED_TOPK = True
PAIR_LPT_ORDER = True   # users launched in decreasing history length
PAIR_STRIPE = 256       # columns per gather wave (nais_pairs.hip STRIPE)
PAIR_CU_LAYOUT = "contiguous"   # or "interleaved" (kept for the A/B)
# Overlapped fused route: the table stream finishes its blocks before the gather stream (config 4:
# 454 vs 537 ms on 128 CUs each), so after each block's table it also gathers that block for the
# tail of the (longest-first) user list holding this fraction of the history entries. Each user
# stays on one stream, so its running top-k still has one writer per launch. Off: the gathers are
# bound by the memory side, not by their CUs -- at 0 / 0.04 / 0.08 / 0.12 the job took 545.4 /
# 542.6 / 552.6 / 614.8 ms while the gather stream's own time fell only 539 -> 532 ms
# (profiles/r1/table_gather_frac/; results bit-identical, test_pairs_blocks_passes_bit_identical).
# Round 4 (the 16x16x32 tables now the faster stream at config 4): 0 / 0.03 / 0.05 / 0.08 ->
# 604 / 599 / 594 / 609 ms on one box (profiles/r4/tgf), but 0.05 on a box whose tables ran at
# 601 ms made the table stream the bound (607 ms, profiles/r4/tgf2): box to box the two streams
# trade places, so the share stays 0.
PAIR_TABLE_GATHER_FRAC = 0.0
# Table launches alternate over two streams with the same CU mask, so block b + 1's workgroups
# fill the CUs that block b's last, partial round of workgroups leaves idle (1,564 workgroups of
# one table block = 9.8 rounds over 160 CUs; one stream waits for the whole launch to drain).
PAIR_TABLE_STREAMS = int(os.environ.get("NAIS_PAIR_TABLE_STREAMS", "2"))
# Work-queue launches of the table (16x16x32 kernel) and fused-gather kernels (round 4): a resident
# round of workgroups takes items from a counter, so a stream's CU count need not be a multiple of
# the 32 shader engines (auto_table_cus then steps in PAIR_SPLIT_STEP CUs).
PAIR_WORK_QUEUE = os.environ.get("NAIS_PAIR_WORK_QUEUE", "1") != "0"
PAIR_SPLIT_STEP = 8
# Bounded gather + exact refine (round 6; include/nais.h nais_pair_bound_topk): the fused top-k
# from split16 tables -- the gather streams only their hi halves (4 bytes per history entry and
# candidate instead of 8), keeps per user the k best LOWER bounds of the exact scores and the
# candidates whose UPPER bound reaches the k-th of them, and a refine pass recomputes those
# candidates' exact sums from their (e, e*s) pairs in CSR order: the same lists, ids and score bits as the exact
# fused gather (tests/test_gpu_bounded.py compares every user). Every block's tables stay resident
# until the refine (J x P x 8 bytes: 80 GB at config 4), so the route is taken only when they fit
# the memory budget; otherwise the exact fused gather runs on double-buffered tables.
PAIR_BOUNDED = True
PAIR_SURV_CAP = 1024            # survivor keys per user (compacted by the current bound when full)
# the bounded gather / refine get each CSR entry's table row and each slot's history span (ABI 14:
# shorter chains of dependent loads); "0" passes NULL (A/B only). Per gather launch 2.272 -> 2.224
# ms at config 4, 2.48 -> 2.45 ms on one rank of N = 8, interleaved (profiles/r6/chains_ab)
PAIR_SHORT_CHAINS = os.environ.get("NAIS_PAIR_SHORT_CHAINS", "1") != "0"
PAIR_BOUNDED_STRIPE = 512       # columns per bounded-gather wave (nais_pairs.hip BSTRIPE)
_masked: dict = {}


def bounded_gather_cu_seconds(entries, NC, users, k):
    """CU-seconds of one job's bounded gathers (nais_pair_bound_topk, one launch per 512-column
    stripe), fitted on the measured launches (profiles/r6/split_world, profiles/r6/configs):
      entries x NC x 4 B / 90.4 GB/s   the hi words streamed (Infinity-Cache served)
      + 512 ns x users x launches      per user and launch: its lists in and out, its CSR rows
      + 68 ns x insertions             a user's running top-k takes ~k (1 + ln(NC / k)) of them
    Fitted first (722 ns per user and launch) on config 4 at N = 1 / 2 / 4 / 8 column shards (68
    gather CUs: 157.9 / 165.9 / 176.9 / 194.9 CU-ms per launch) and on config 2 (24 CUs: 21.4 CU-ms
    per launch for 10,000 users with h <= 100), within 1-3 %. Narrow shards and short histories pay
    the per-user terms on fewer bytes. The per-user term is latency: a chain of dependent loads at
    a few waves per SIMD. The per-entry rows, the per-slot spans and 4 rows in flight (4 waves per
    SIMD) brought it to 512 ns: config 4 2.168 ms x 68 CUs, N = 8 2.28 ms x 80 CUs per launch
    (profiles/r6/chains_ab)."""
    launches = np.ceil(NC / PAIR_BOUNDED_STRIPE)
    ins = k * (1.0 + np.log(max(float(NC), float(k)) / k))
    return entries * NC * 4.0 / 90.4e9 + 512e-9 * users * launches + 68e-9 * users * ins


def auto_table_cus(model, J, NC, entries, ncu, prior=False, block_bytes=None, work_queues=True,
                   gather_bytes=8, k=None, users=None):
    """CUs for the table stream (the rest gather), in steps of ncu / 8 (counts off a multiple of 32
    leave a shader engine short and lose -- DESIGN.md, CU split), from a cost model fitted
    on config 4 and config 5 (profiles/r1/cfg5p/, re-fitted in round 3 on the fp16x6 tables:
    629-664 ms on 160 CUs): tables at ~1.25e15 f16 FLOP/s (split-fp16) or
    1.3e14 FLOP/s (fp32) on the whole chip, scaling with their CUs; gathers at ~72 GB/s per CU up
    to 7.5 TB/s (round 3: measured 71 GB/s per CU at 96 gather CUs, 78 at 64, 59 at 128 where the
    memory side saturates; the round-1 figure of 60 kept the exact-fp32 leg at 160 table CUs). Picks the split that minimises the slower of the two streams (config 4: 160 of 256
    under fp16x6, config 5: 224). With the power-law prior the table stream also builds the float64
    pr_d table (~1.4e-11 s per pair on the whole chip, profiles/r2/legs_s4) and the gather stream
    reads it too (8 more bytes per history entry and column).

    `work_queues`: whether this job's table AND gather launches take the work counter (the x6n
    table kernel of the NAIS modules and the fused top-k gather). Only then may the
    split step finer than one CU per shader engine: a fixed-grid launch on a CU count off a
    multiple of 32 leaves an engine short and runs at the next lower multiple."""
    H, din = model.attn_layer1.weight.shape
    prec = getattr(model, "precision", "fp16x6")
    products = 1 if prec == "fp32" else (6 if prec.startswith("fp16x6") else 3)
    dist = getattr(model, "VARIANT", 0) in (_capi.VARIANT_REGION_DISTANCE, _capi.VARIANT_DISTANCE)
    D = din - 2 if dist else din
    D = next((w for w in (8, 16, 32, 64, 128) if w >= D), D)   # the padded width the kernels run
    gbytes = entries * NC * float(gather_bytes)   # 4 on the bounded route (hi words only)
    if prior:
        gbytes *= 2
    xcd = max(1, ncu // 8)
    # with work-queue launches the split may step finer than a CU per shader engine (x6n tables
    # and the fused gather; other table kernels keep the engine-sized steps)
    x6n = (PAIR_WORK_QUEUE and work_queues and products == 6 and D in (32, 64, 128) and H <= 128
           and not prior)
    step = min(PAIR_SPLIT_STEP, xcd) if x6n else xcd
    # round 4: 1.45e15 (config 4), 1.55e15 (config-5 shard); round 6: 1.47e15 -- the final tree's
    # config-4 tables ran 446.5 ms on 190 CUs (1.45e15 said 456.8), and 1.47e15 keeps every
    # measured best split: 190 / 190 / 186 / 180 at N = 1 / 2 / 4 / 8 (profiles/r6/split_n1,
    # split_world) and region_distance at 194 (profiles/r6/rd_split), where 1.45e15 chose 196
    rate = 1.47e15 if x6n else 1.25e15
    din_k = D + (2 if dist else 0)      # the width the kernels multiply (padded)
    t_tab = J * NC * 2.0 * H * din_k * products / (1.3e14 if products == 1 else rate)
    if x6n and dist:
        # the distance K-step: 2 v_mfma_f32_16x16x1_4b_f32 (32 cycles each) per PAIR of 16-hidden
        # blocks beside their 2 * 12 * D / 32 f16 MFMAs (16 cycles each): 1 + 16 / (3 D) matrix time
        t_tab *= 1.0 + 16.0 / (3.0 * D)
    if prior:
        t_tab += J * NC * 1.4e-11
    # gather rate per CU: ~72 GB/s while a block's e / e*s tables (block_bytes) mostly stay in the
    # 256 MB Infinity Cache (config 4: 410 MB), ~51 GB/s from HBM (config-5 shard: 4.1 GB; round 4,
    # 1.64 TB/s on 32 CUs)
    per_cu = 72e9 if block_bytes is None or block_bytes <= 512e6 else 51e9
    if gather_bytes == 4:
        # the bounded gather (hi words, 4 B per entry and column): 65-66 GB/s per CU measured at 64,
        # 68 and 80 gather CUs (config 4, round 6: 485.8 / 448.6 / 389.3 ms for 2.02 TB;
        # profiles/r6/bounded, split_ab), and 4-CU steps: 188 / 68 ran 471.4 ms against 476.9 /
        # 480.2 at 184 / 72 and 490.8 at 180 / 76 on one box (profiles/r6/split_ab)
        per_cu = 66e9
        if x6n:
            # 2-CU steps: config 4 at 190 / 66 ran 476.2 / 476.8 / 478.6 ms against 482.4-482.5 at
            # 188 / 68, interleaved on one box (profiles/r6/split_n1); one rank of N = 2 at 190
            # 239.0 / 239.3 vs 240.5 / 240.9 at 188, N = 4 at 186 even with 184, config 2 at 234
            # 95.8 / 96.2 vs 95.5 / 95.9 at 232 (profiles/r6/split_n1/step2)
            step = 2
        if users and k:
            # the three-term fit (bounded_gather_cu_seconds) as an effective per-CU rate: one
            # rank's narrow column shard (N = 8: best split 172-180 against 188 at N = 1,
            # profiles/r6/split_world) and short histories (config 2) pay more per byte
            per_cu = gbytes / bounded_gather_cu_seconds(entries, NC, users, k)
    cap = 7.5e12   # the memory side's rate for the gather, chip-wide
    best, best_t = ncu // 2, None
    for n in range((ncu // 4 + step - 1) // step * step, ncu - step + 1, step):
        g_pen = 1.0
        if gather_bytes == 4 and PAIR_CU_LAYOUT == "contiguous" and (ncu - 1) // xcd - n // xcd + 1 <= 2:
            # a bounded gather confined to two XCDs (contiguous CU ids) costs ~4 % more CU-time per
            # launch than one spanning three: config 4 at 192 / 64 151.5 CU-ms against 146.2 at
            # 190 / 66 (the job 497 vs 484 ms, profiles/r6/split_n1), region_distance at 196 / 60
            # 151.9 -- whose job ran 522.6 / 524.4 ms there against 514.2 / 516.6 at 194 / 62
            # (profiles/r6/rd_split)
            g_pen = 1.04
        t = max(t_tab * ncu / n, gbytes * g_pen / min(cap, (ncu - n) * per_cu))
        if best_t is None or t <= best_t:   # ties (gather-bound): the larger table share
            best, best_t = n, t
    return best


def _destroy_masked_streams():
    """Release the CU-masked streams before interpreter exit: left to the C++ static destructors
    they outlive the HIP runtime (a crash at exit under rocprofv3)."""
    if not _masked:
        return
    lib = _capi.load()
    for pair in _masked.values():
        for s in pair:
            s.synchronize()
            lib.nais_stream_destroy(s.cuda_stream)
    _masked.clear()


def _masked_streams(dev, table_cus):
    """(table stream, gather stream, second table stream) as torch ExternalStreams: the two table
    streams on one CU mask, the gather stream on the disjoint rest (cached)."""
    key = (str(dev), table_cus, PAIR_CU_LAYOUT)
    hit = _masked.get(key)
    if hit is not None:
        return hit
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    if PAIR_CU_LAYOUT == "contiguous":
        mine = set(range(table_cus))
    else:   # spread over the CU ids evenly
        mine = {int(i * n / table_cus) for i in range(table_cus)}
    words = (n + 31) // 32
    masks = []
    for sel in (mine, set(range(n)) - mine, mine):
        m = (ctypes.c_uint32 * words)()
        for c in sel:
            m[c // 32] |= 1 << (c % 32)
        masks.append(m)
    lib = _capi.load()
    out = []
    with torch.cuda.device(dev):
        for m in masks:
            h = ctypes.c_void_p()
            _capi.check(lib.nais_stream_create_cu_mask(m, words, ctypes.byref(h)), "nais_stream_create_cu_mask")
            out.append(torch.cuda.ExternalStream(h.value, device=dev))
    if not _masked:
        import atexit
        atexit.register(_destroy_masked_streams)
    _masked[key] = tuple(out)
    return _masked[key]


def _score_topk_pairs(model, train_matrix, users, k, region_of, coords, latlon_mat, stream, force,
                      rows_only=False, cols=None, events=None, prior=None, no_side_streams=False,
                      group=None, return_keys=False, tau_group=None):
    """Pairs strategy. `cols` = (c0, c1): score only POIs [c0, c1) (top-k ids are global POI ids;
    a column shard of sharding.distributed_topk_pairs). `events`: optional list that receives
    (kind, start, end) HIP events around every table / gather / top-k launch. `prior` = (a, b,
    alpha, poi_coords): rank on the power-law-blended score (score_topk); score rows + float64 G
    rows per pass, then nais_topk_blend_rows (the direct route's blend, same G bits).

    Column shards with a prior (`cols` and `group`, a torch.distributed group whose ranks own
    the other columns): every rank makes the same number of user passes (MIN all-reduce of the
    users one pass can hold), and each user's max G over ITS columns is MAX all-reduced before the
    blend, so every rank normalises by the whole catalog's max (run.py:55-59) -- one [users]
    int64 collective per pass. `return_keys`: also return the f64 blended score of each returned
    candidate (the merge key of sharding.distributed_topk_pairs).

    `tau_group` (a column shard's process group, no prior): on the bounded route every rank takes
    the route or none does (one MIN all-reduce), and before the refine the ranks exchange their
    lower-bound lists (sharding.global_kth_keys), so each refines only what can reach the GLOBAL
    top-k -- the refine then shrinks with the world size like the tables and gathers; the returned
    lists may be short (padding id -1), which the merge ranks last."""
    dev = model._check_device()
    csr = device_csr(train_matrix, dev)
    P = model._item_tables()[0].shape[0]
    if csr.shape[1] != P:
        raise ValueError(f"train_matrix has {csr.shape[1]} POIs, model has {P}")
    c0_all, c1_all = cols if cols is not None else (0, P)
    NC = c1_all - c0_all
    users = _user_array(users)
    n = len(users)
    if n == 0 or NC <= 0:
        return None
    if cols is None and np.any(P - csr.hist_len[users] < k):
        raise RuntimeError("selected index k out of range")       # torch.topk's error
    lib = _capi.load()
    st = stream if stream is not None else _capi.stream_handle(dev)
    torch_stream = torch.cuda.current_stream(dev)
    # longest histories first: a gather launch then ends on its shortest users (short tail)
    order = None
    if PAIR_LPT_ORDER and not rows_only and n > 1:
        order = np.argsort(-csr.hist_len[users], kind="stable")
    # one pinned, non-blocking upload of the launch order (and its inverse): no host sync here or
    # at the end of the job, which would idle the GPU between consecutive jobs
    up = np.concatenate([users if order is None else users[order],
                         np.argsort(order, kind="stable") if order is not None else np.zeros(0, np.int64)])
    up_dev = torch.from_numpy(up.astype(np.int32)).pin_memory().to(dev, non_blocking=True)
    u_all = up_dev[:n]
    reg, cor, llm = _side_inputs(model, dev, region_of, coords, latlon_mat)
    prm = model._score_params()
    rowmap = torch.empty(P, dtype=torch.int32, device=dev)
    items = torch.empty(P, dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = _workspace(dev, lib.nais_pair_rows_workspace_size(P))

    def timed(kind, fn, launches=1):
        if events is None:
            return fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch_stream)
        r = fn()
        e1.record(torch_stream)
        events.append((kind, e0, e1, launches))
        return r

    def rows(u_dev, m):
        _capi.check(lib.nais_pair_rows(csr.indptr.data_ptr(), csr.indices.data_ptr(), u_dev.data_ptr(),
                                       m, P, rowmap.data_ptr(), items.data_ptr(), cnt.data_ptr(),
                                       ws.data_ptr(), ws.numel(), st), "nais_pair_rows")
        return int(cnt.item())
    J = rows(u_all, n)
    entries = int(csr.hist_len[users].sum())
    if not force and (J == 0 or entries < PAIR_MIN_SHARING * J):
        return None
    usable = usable_device_bytes(dev)
    budget = int(usable * PAIR_MEMORY_FRACTION)
    from .model import _NAISDevice
    if prior is not None and (rows_only or model._pairs_only):
        raise NotImplementedError("the pairs route blends the prior over the rows of NAIS models only")
    if prior is not None and cols is not None and (c0_all, c1_all) != (0, P) and group is None:
        raise ValueError("a prior over a column shard needs the process group of the other shards "
                         "(the normaliser max G runs over the whole catalog)")
    fused = (PAIR_FUSED_TOPK and not rows_only and J > 0 and k <= 256 and prior is None
             and type(model)._pair_fixup is _NAISDevice._pair_fixup)
    # the bounded route needs the split16 tables of the NAIS modules' own table kernels
    bounded_ok = fused and PAIR_BOUNDED and type(model)._pair_table is _NAISDevice._pair_table
    if prior is not None:
        pa, pb, alpha, pc = prior
        pri_coords = torch.as_tensor(np.ascontiguousarray(pc, dtype=np.float64)).to(dev)
        prior_flags = _capi.PRIOR_FINITE if _prior_entries_finite(pa, pb) else 0
    pr_of = {}   # column-block table -> its float64 pr_d table (prior only)

    # work-queue counters (PAIR_WORK_QUEUE): one int32 per stream, each used stream-ordered; on
    # only for a split off the shader-engine steps (config 4 at 152 / 104: 598 ms vs 607 at the
    # classic 160 / 96; config-5 shard at 232 / 24: 17.3 s vs 18.2 at 224 / 32 -- profiles/r4/wq)
    wq_slots = torch.zeros(8, dtype=torch.int32, device=dev) if PAIR_WORK_QUEUE else None
    wq_of = {}
    wq_on = [False]

    def wq(stream_):
        if wq_slots is None or not wq_on[0]:
            return None
        h = int(stream_ or 0)
        if h not in wq_of:
            if len(wq_of) >= wq_slots.numel():   # one counter per stream
                raise RuntimeError("pairs route: more streams than work-queue counters")
            wq_of[h] = wq_slots.data_ptr() + 4 * len(wq_of)
        return wq_of[h]

    def table(tab, c0, w, stream_):
        if isinstance(tab, tuple):   # the bounded route's split16 tables (hi words, ex pairs)
            _capi.check(lib.nais_pair_table_split(prm, items.data_ptr(), J, c0, w, _capi.ptr(reg),
                                                  _capi.ptr(cor), _capi.ptr(llm), tab[0].data_ptr(),
                                                  tab[1].data_ptr(), ld, wq(stream_), stream_),
                        "nais_pair_table_split")
            return
        model._pair_table(lib, prm, items, J, c0, w, reg, cor, llm, tab[0].data_ptr(),
                          tab[1].data_ptr(), ld, stream_, work=wq(stream_))
        if prior is not None:
            _capi.check(lib.nais_pair_prior_table(pri_coords.data_ptr(), P, items.data_ptr(), J, c0, w,
                                                  float(pa), float(pb), pr_of[id(tab)].data_ptr(), ld,
                                                  stream_), "nais_pair_prior_table")
    # users per pass: their score rows (+ float64 G rows with a prior) take at most half the
    # budget (fused: no score rows)
    row_bytes = 4 * NC + (8 * NC if prior is not None else 0)
    per_pass = n if (rows_only or fused) else max(1, min(n, (budget // 2) // row_bytes))
    if prior is not None and group is not None:     # the same passes (and collectives) on every rank
        from .sharding import agree_min
        per_pass = agree_min(per_pass, dev, group)
    if events is not None:    # the plan of this call, for the bench record
        npass = (n + per_pass - 1) // per_pass
        events.extend((name, None, None, v) for name, v in (
            ("passes", npass), ("users_per_pass", per_pass), ("distinct_rows", J),
            ("usable_bytes", usable), ("budget_bytes", budget)))
    keys_out = torch.empty(n, k, dtype=torch.float64, device=dev) if return_keys else None
    ids_out = torch.empty(n, k, dtype=torch.int32, device=dev)
    sc_out = torch.empty(n, k, dtype=torch.float32, device=dev)
    counters = torch.zeros(2, dtype=torch.int32, device=dev)
    for b0 in range(0, n, per_pass):
        m = min(per_pass, n - b0)
        u_dev = u_all[b0:b0 + m]
        if b0 > 0 or m < n:
            J = rows(u_dev, m)
        bnd = [False]   # this pass takes the bounded route (decided once the tables are sized)

        def gather_launches(w):   # one fused-gather kernel per 256-column (bounded: 512) stripe
            stripe = PAIR_BOUNDED_STRIPE if bnd[0] else PAIR_STRIPE
            return (w + stripe - 1) // stripe if fused else 1
        if fused:
            keys = torch.empty(m, k, dtype=torch.int64, device=dev)
            kcount = torch.zeros(m, dtype=torch.int32, device=dev)

            def gather(tab, c0, w, stream_, a=0, b=None):   # launch slots [a, b) of u_dev
                b = m if b is None else b
                if b <= a:
                    return
                if bnd[0]:
                    _capi.check(lib.nais_pair_bound_topk(
                        tab[0].data_ptr(), ld, rowmap.data_ptr(), csr.indptr.data_ptr(), csr.indices.data_ptr(),
                        u_dev.data_ptr() + 4 * a, b - a, c0, w, float(model.beta), k,
                        lokeys.data_ptr() + 8 * k * a, locount.data_ptr() + 4 * a,
                        surv.data_ptr() + 8 * PAIR_SURV_CAP * a, scount.data_ptr() + 4 * a, PAIR_SURV_CAP,
                        _capi.ptr(erows), spans.data_ptr() + 16 * a if spans is not None else None,
                        wq(stream_), stream_),
                        "nais_pair_bound_topk")
                    return
                _capi.check(lib.nais_pair_gather_topk(
                    tab[0].data_ptr(), tab[1].data_ptr(), ld, rowmap.data_ptr(), csr.indptr.data_ptr(),
                    csr.indices.data_ptr(), u_dev.data_ptr() + 4 * a, b - a, c0, w, float(model.beta), k,
                    keys.data_ptr() + 8 * k * a, kcount.data_ptr() + 4 * a, counters[0:1].data_ptr(),
                    wq(stream_), stream_), "nais_pair_gather_topk")
        else:
            scores = torch.empty(m, NC, dtype=torch.float32, device=dev)
            if prior is not None:
                G = torch.empty(m, NC, dtype=torch.float64, device=dev)
                gmax = torch.zeros(m, dtype=torch.int64, device=dev)

            def gather(tab, c0, w, stream_, a=0, b=None):
                _capi.check(lib.nais_pair_gather(
                    tab[0].data_ptr(), tab[1].data_ptr(), ld, rowmap.data_ptr(), csr.indptr.data_ptr(),
                    csr.indices.data_ptr(), u_dev.data_ptr(), m, c0, w, float(model.beta),
                    scores.data_ptr(), NC, c0_all, counters[0:1].data_ptr(), stream_), "nais_pair_gather")
                if prior is not None:
                    _capi.check(lib.nais_pair_prior_gather(
                        pr_of[id(tab)].data_ptr(), ld, rowmap.data_ptr(), csr.indptr.data_ptr(),
                        csr.indices.data_ptr(), u_dev.data_ptr(), m, c0, w, G.data_ptr(), NC, c0_all,
                        gmax.data_ptr(), prior_flags, stream_), "nais_pair_prior_gather")
        if J > 0:
            # two f32 tables (+ the f64 pr_d table with a prior) per buffer, <= budget / 4 each
            W = min(PAIR_BLOCK_COLS, (budget // 4) // ((16 if prior is not None else 8) * J))
            W = int(min(NC, max(256, W // 256 * 256)))
            # row pitch of the tables: a multiple of 4 floats (the gathers' 16-byte loads) even
            # when a narrow column shard makes the block width odd
            ld = (W + 3) // 4 * 4
            blocks = list(range(c0_all, c1_all, W))
            # bounded route: every block's split16 tables (2 x J x ld words each) resident, plus
            # the per-user lower-bound lists and survivor keys
            bnd[0] = bounded_ok and (len(blocks) * 3 * J * ld * 4 + m * (PAIR_SURV_CAP + k) * 8
                                     <= budget)
            if tau_group is not None and bounded_ok:   # the same route on every rank
                from .sharding import agree_min
                bnd[0] = bool(agree_min(int(bnd[0]), dev, tau_group))
            if bnd[0]:   # per block: the hi words [J, ld] and the exact (e, e*s) pairs [J, 2 ld]
                arena = (torch.empty(len(blocks), J, ld, dtype=torch.int32, device=dev),
                         torch.empty(len(blocks), J, 2 * ld, dtype=torch.int32, device=dev))
                lokeys = torch.empty(m, k, dtype=torch.int64, device=dev)
                locount = torch.zeros(m, dtype=torch.int32, device=dev)
                surv = torch.empty(m, PAIR_SURV_CAP, dtype=torch.int64, device=dev)
                scount = torch.zeros(m, dtype=torch.int32, device=dev)
                # the gathers' load chains shortened (include/nais.h, ABI 14): each CSR entry's
                # table row, and each slot's (history start, length)
                erows = spans = None
                if PAIR_SHORT_CHAINS:
                    erows = rowmap.index_select(0, csr.indices)
                    hb_ = csr.indptr.index_select(0, u_dev.to(torch.int64))
                    spans = torch.stack([hb_, csr.indptr.index_select(0, u_dev.to(torch.int64) + 1) - hb_],
                                        1).contiguous()
                if events is not None:
                    events.append(("bounded", None, None, 1))
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            # both streams run as work queues only with the NAIS modules' own table kernel and
            # the fused gather (the score-row gather and nais_dot_pair_table keep fixed grids)
            wq_both = fused and type(model)._pair_table is _NAISDevice._pair_table
            table_cus = (auto_table_cus(model, J, NC, entries, ncu, prior is not None, J * ld * 8,
                                        work_queues=wq_both, gather_bytes=4 if bnd[0] else 8, k=k,
                                        users=m)
                         if PAIR_TABLE_CUS < 0 else PAIR_TABLE_CUS)
            wq_on[0] = table_cus % max(1, ncu // 8) != 0
            if events is not None:
                events.append(("table_cus", None, None, table_cus))
                events.append(("block_cols", None, None, W))
            overlap = (0 < table_cus < ncu and len(blocks) > 1 and stream is None
                       and not no_side_streams)
            tabs = ([] if bnd[0] else [torch.empty(2, J, ld, dtype=torch.float32, device=dev)
                                       for _ in range(2 if overlap else 1)])
            if prior is not None:
                pr_of.update({id(t): torch.empty(J, ld, dtype=torch.float64, device=dev) for t in tabs})
            if overlap:
                ts, gs, ts2 = _masked_streams(dev, table_cus)
                tss = (ts, ts2) if PAIR_TABLE_STREAMS > 1 else (ts,)
                first_all = PAIR_FIRST_TABLE_ALL_CUS
                if first_all:      # block 0's table alone, on the caller's stream (all CUs)
                    w0 = min(W, c1_all - blocks[0])
                    tab0 = (arena[0][0], arena[1][0]) if bnd[0] else tabs[0]
                    timed("table", lambda: table(tab0, blocks[0], w0, st))
                for t_ in tss:
                    t_.wait_stream(torch_stream)
                gs.wait_stream(torch_stream)
                done_g = [None, None]
                done_tail = None   # the previous block's tail gather (another table stream)
                # launch slots [m1, m) are gathered on the table stream (PAIR_TABLE_GATHER_FRAC)
                m1 = m
                if fused and PAIR_TABLE_GATHER_FRAC > 0 and m > 1:
                    hl = csr.hist_len[up[b0:b0 + m]].astype(np.float64)
                    tail = np.cumsum(hl[::-1])[::-1]        # entries of slots [i, m)
                    m1 = int(np.searchsorted(-tail, -PAIR_TABLE_GATHER_FRAC * hl.sum(), side="left"))
                    m1 = min(max(m1, 1), m)
                if events is not None:
                    share = float(csr.hist_len[up[b0:b0 + m1]].sum()) / max(1.0, float(csr.hist_len[up[b0:b0 + m]].sum()))
                    events.append(("gather_share", None, None, share))
            for b, c0 in enumerate(blocks):
                w = min(W, c1_all - c0)
                tab = (arena[0][b], arena[1][b]) if bnd[0] else tabs[b % len(tabs)]
                if overlap:
                    tsb = tss[b % len(tss)]
                    if done_g[b % 2] is not None and not bnd[0]:
                        tsb.wait_event(done_g[b % 2])    # buffer free: its gather finished
                    if not (b == 0 and first_all):
                        e_t0, e_t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e_t0.record(tsb)
                        table(tab, c0, w, tsb.cuda_stream)
                        e_t1.record(tsb)
                        gs.wait_event(e_t1)
                        if events is not None:
                            events.append(("table", e_t0, e_t1, 1))
                    e_g0, e_g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e_g0.record(gs)
                    gather(tab, c0, w, gs.cuda_stream, 0, m1)
                    e_g1.record(gs)
                    done_g[b % 2] = e_g1
                    if events is not None:
                        events.append(("gather", e_g0, e_g1, gather_launches(w)))
                    if m1 < m:   # the tail users, behind this block's table on the table stream
                        # their running top-k keys were last merged by the previous block's tail
                        # gather, on the other table stream: order the two merges
                        if done_tail is not None and len(tss) > 1:
                            tsb.wait_event(done_tail)
                        gather(tab, c0, w, tsb.cuda_stream, m1, m)
                        done_tail = torch.cuda.Event()
                        done_tail.record(tsb)
                    continue
                timed("table", lambda: table(tab, c0, w, st))
                timed("gather", lambda: gather(tab, c0, w, st), gather_launches(w))
            if overlap:
                torch_stream.wait_stream(gs)
                for t_ in tss:
                    torch_stream.wait_stream(t_)
                for t in [*tabs, *pr_of.values(), *([wq_slots] if wq_slots is not None else []),
                          *((*arena, lokeys, locount, surv, scount,
                             *((erows, spans) if erows is not None else ())) if bnd[0] else ())]:
                    for t_ in (*tss, gs):   # not handed to the main stream early
                        t.record_stream(t_)
            if bnd[0]:   # the exact refine of every user's surviving candidates (all CUs)
                stats = torch.zeros(2, dtype=torch.int32, device=dev)
                tau_g = None
                if tau_group is not None:   # the k-th lower key over every rank's columns
                    from .sharding import global_kth_keys
                    tau_g = timed("tau_exchange", lambda: global_kth_keys(lokeys, locount, k, tau_group))
                timed("refine", lambda: _capi.check(lib.nais_pair_refine_topk(
                    arena[1].data_ptr(), 2 * J * ld, ld, W, rowmap.data_ptr(), csr.indptr.data_ptr(),
                    csr.indices.data_ptr(), u_dev.data_ptr(), m, c0_all, NC, float(model.beta), k,
                    lokeys.data_ptr(), locount.data_ptr(), surv.data_ptr(), scount.data_ptr(),
                    PAIR_SURV_CAP, tau_g.data_ptr() if tau_g is not None else None, keys.data_ptr(),
                    kcount.data_ptr(), counters[0:1].data_ptr(), stats.data_ptr(), _capi.ptr(erows), st),
                    "nais_pair_refine_topk"))
                model._last_bound_stats = stats
                del arena, lokeys, locount, surv, scount, erows, spans
            del tabs
            pr_of.clear()
            if not fused:
                model._pair_fixup(csr, u_dev, m, scores, c0_all, c1_all, st)
        else:
            scores.fill_(0.5)   # every listed user has an empty history: logit 0 (model.py:79-88)
        if rows_only:
            model._last_nan = counters[0:1]
            return scores
        if fused:
            timed("topk", lambda: _capi.check(lib.nais_topk_keys_finish(
                keys.data_ptr(), kcount.data_ptr(), m, k, ids_out[b0:b0 + m].data_ptr(),
                sc_out[b0:b0 + m].data_ptr(), counters[1:2].data_ptr(), st), "nais_topk_keys_finish"))
            del keys, kcount
            continue
        if prior is not None:
            if J == 0:      # empty histories: G = prod over nothing = 1.0 for every candidate
                G.fill_(1.0)
                gmax.fill_(int(np.array(1.0).view(np.int64)))
            if group is not None:   # normalise by the max over every rank's columns
                from .sharding import allreduce_gmax
                allreduce_gmax(gmax, group)
            timed("topk", lambda: _capi.check(lib.nais_topk_blend_rows_f64(
                scores.data_ptr(), NC, G.data_ptr(), NC, gmax.data_ptr(), NC, m, k, float(alpha),
                ids_out[b0:b0 + m].data_ptr(), sc_out[b0:b0 + m].data_ptr(),
                keys_out[b0:b0 + m].data_ptr() if return_keys else None, counters[1:2].data_ptr(),
                st), "nais_topk_blend_rows_f64"))
            del G, gmax
        else:
            timed("topk", lambda: _capi.check(lib.nais_topk_rows(
                scores.data_ptr(), NC, NC, m, k, ids_out[b0:b0 + m].data_ptr(), sc_out[b0:b0 + m].data_ptr(),
                counters[1:2].data_ptr(), st), "nais_topk_rows"))
        del scores
    model._last_nan = counters[0:1]
    ids = ids_out.to(torch.int64)
    if c0_all and not fused:        # the fused keys carry global POI ids already
        ids = torch.where(ids >= 0, ids + c0_all, ids)
    if order is not None:           # back to the caller's user order
        inv = up_dev[n:]
        ids, sc_out = ids.index_select(0, inv), sc_out.index_select(0, inv)
        if return_keys:
            keys_out = keys_out.index_select(0, inv)
    if return_keys:
        return ids, sc_out, keys_out
    return ids, sc_out


def usable_device_bytes(dev):
    """Bytes this process can still allocate on `dev`: the driver's free memory plus what torch's
    caching allocator holds reserved but unused. The pass split of the pairs route is sized from
    this, so it does not depend on how much of an earlier call's memory the allocator still caches
    (mem_get_info alone counts that as used: the prior route's 60 GB of score + G rows at config 4
    then fit one pass on a fresh process and needed two after a first job)."""
    # only cached segments with nothing allocated in them can serve a new large allocation (the
    # allocator releases them and retries when a request finds no block); the free pieces of partly
    # used segments ("inactive split" bytes) cannot, so they are not counted
    free = torch.cuda.mem_get_info(dev)[0]
    st = torch.cuda.memory_stats(dev)
    split = int(st.get("inactive_split_bytes.all.current", 0))
    cached = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev) - split
    return int(free + max(0, cached))


def _prior_entries_finite(a, b):
    """Every pr_d(d) = a * max(0.01, d)^b (powerLaw.py:86-88) is finite for 0 <= d <= half the
    earth's circumference (the range of powerLaw.dist), and with a > 0 every factor is >= +0, so a
    G product that reached +0.0 stays +0.0, sign bit included (nais_pair_prior_gather's
    NAIS_PRIOR_FINITE; the per-user prior_kernel's twin is prior_zero_exit in nais_kernels.hip)."""
    import math
    a, b = float(a), float(b)
    if not (math.isfinite(a) and math.isfinite(b) and a > 0.0):
        return False
    try:
        ends = (a * 0.01 ** b, a * (math.pi * 6371.0) ** b)
    except OverflowError:
        return False
    return all(math.isfinite(v) for v in ends)


def prior_rows(train_matrix, users, a, b, coords, device):
    """Power-law prior rows G [len(users), P] float64 (history POIs = -1) and the per-user max
    over candidates, via nais_powerlaw_prior (powerLaw.py:90-92, run.py:55-59)."""
    dev = torch.device(device)
    csr = device_csr(train_matrix, dev)
    P = csr.shape[1]
    users = _user_array(users)
    u_dev = torch.from_numpy(users.astype(np.int32)).to(dev)
    cor = torch.as_tensor(np.ascontiguousarray(coords, dtype=np.float64)).to(dev)
    out = torch.empty(len(users), P, dtype=torch.float64, device=dev)
    mx = torch.empty(len(users), dtype=torch.float64, device=dev)
    rc = _capi.load().nais_powerlaw_prior(cor.data_ptr(), P, csr.indptr.data_ptr(),
                                          csr.indices.data_ptr(), u_dev.data_ptr(), len(users),
                                          float(a), float(b), out.data_ptr(), P, mx.data_ptr(),
                                          _capi.stream_handle(dev))
    _capi.check(rc, "nais_powerlaw_prior")
    return out, mx
