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
# fp16x6 (the fp32-faithful default) issues 6 per algorithmic fp32 product
PRODUCTS = {"fp32": 1, "fp16x3": 3, "fp16x3_pairsplit": 3, "fp16x6": 6, "fp16x6_pairsplit": 6}
PEAKS = {k: (PEAK_FP32_MFMA_TFLOPS if v == 1 else PEAK_F16_MFMA_TFLOPS / v) for k, v in PRODUCTS.items()}
HBM_SPEC_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E peak (spec)
HBM_MEASURED_GBS = 6290.0      # MI355X_MICROARCH.md: float4 copy, measured
DTYPES = {
    "fp32": "fp32 (v_mfma_f32_32x32x2_f32: exact fp32 products, fp32 accumulate)",
    "fp16x6": "fp32-faithful: W1 x products as 6 f16 MFMA products of exact hi/mid/lo fp16 splits "
              "(dropped terms <= ~2^-33 relative, below fp32 rounding), fp32 accumulate; all other "
              "arithmetic fp32",
    "fp16x6_pairsplit": "fp32-faithful (fp16x6 arithmetic, per-pair split of x = h . t)",
    "fp16x3": "narrower than fp32: W1 x products as 3 f16 MFMA products of hi/lo splits (~2^-21)",
    "fp16x3_pairsplit": "narrower than fp32: fp16x3 arithmetic, per-pair split",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", type=int, default=4, choices=[2, 4, 5],
                    help="4: 50k users x 100k POIs, d=H=64 (the metric config); 2: 10k users x 50k POIs, "
                         "d=H=64, h<=100 (whole job, pairs route); 5: stress, 200k users x 1M POIs, "
                         "d=H=128, tables sharded + all-gathered, timed on the first 4096 users")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--users-per-step", type=int, default=256)
    ap.add_argument("--num-users", type=int, default=50_000)
    ap.add_argument("--num-pois", type=int, default=100_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--h-max", type=int, default=200)
    ap.add_argument("--topk", type=int, default=50)
    ap.add_argument("--precision", default="fp16x6", choices=sorted(PRODUCTS))
    ap.add_argument("--no-fp32-leg", action="store_true",
                    help="skip the secondary legs (fp32_path, fp16x3_path, prior_path, region_distance_path)")
    ap.add_argument("--leg-steps", type=int, default=3, help="timed steps of each secondary leg")
    ap.add_argument("--cpu-users", type=int, default=32,
                    help="CPU baseline sample: the first N users (after a 1-user warm-up)")
    ap.add_argument("--cpu-seconds", type=float, default=60.0, help="cap on the CPU sample's time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather-leg", action="store_true",
                    help="skip the standalone history-gather leg (nais_gather_rows, 2 GB table)")
    ap.add_argument("--no-train-leg", action="store_true",
                    help="skip the config-3 training-step leg (fused / drop-in / eager torch, D=H=64 and 128)")
    ap.add_argument("--no-self-check", action="store_true",
                    help="skip the oracle check of 2 bench users' top-50 after the timed steps")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL on ROCm) for real runs; gloo to rehearse N>1 on one GPU")
    ap.add_argument("--ab", action="store_true",
                    help="A/B runs only: read the pairs-route knobs from the environment (NAIS_PAIR_TABLE_CUS, "
                         "NAIS_PAIR_CU_LAYOUT, NAIS_PAIR_BLOCK_COLS, NAIS_PAIR_FUSED_TOPK, NAIS_PAIR_LPT_ORDER, "
                         "NAIS_PAIR_TABLE_GATHER_FRAC, NAIS_PAIR_FIRST_TABLE_ALL_CUS); the line records them")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="one process: time rank 0's column shard of an N-GPU pairs job (its tables, "
                         "gathers and local top-k; no collective)")
    ap.add_argument("--strategy", default="auto", choices=["auto", "pairs", "direct"],
                    help="auto: pairs for config 4 (each (item, candidate) pair shared by ~50 users), "
                         "direct for config 5's 4096-user subset (sharing ~1)")
    return ap.parse_args()


def cpu_threads():
    """CPUs this process may use: the affinity set, capped by a cgroup quota and OMP_NUM_THREADS
    (os.cpu_count() shows the whole machine on the GPU boxes)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except Exception:
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
    return max(1, n)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_baseline(p, data, users, k, seconds):
    """the torch-CPU restatement of the reference's evaluation loop
    (oracle/torch_cpu.py: candidate rows, 1,024-row forward chunks, torch.topk), all usable
    cores, a 1-user warm-up, then the listed users (the first 32) until `seconds` run out."""
    from oracle import torch_cpu
    threads = cpu_threads()
    torch.set_num_threads(threads)
    m = torch_cpu.TorchNAIS(p)
    torch_cpu.recommend_user(m, data.history(int(users[0])), data.num_pois, k)      # warm-up
    pairs, t0, n = 0, time.perf_counter(), 0
    for u in users:
        pairs += torch_cpu.recommend_user(m, data.history(int(u)), data.num_pois, k)[2]
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": pairs / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": f"users {int(users[0])}..{int(users[n - 1])} ({n} users, after a 1-user warm-up) "
                      f"of the same workload: complement candidate rows + 1,024-row forward chunks + "
                      f"torch.topk(50), oracle/torch_cpu.py (torch {torch.__version__} CPU, "
                      f"{threads} threads), {pairs} pairs in {dt:.1f} s"}


def torch_scorer(p, data):
    """(candidates, scores) of one user's whole catalog through oracle/torch_cpu.py (the
    reference's loop in torch CPU ops, pinned to the reference's outputs by
    tests/test_torch_cpu_baseline.py) -- ~4x faster than the numpy oracle on the same cores."""
    from oracle import torch_cpu
    m = torch_cpu.TorchNAIS(p)

    def scorer(u):
        rows, cand = torch_cpu.candidates(data.history(int(u)), data.num_pois)
        with torch.no_grad():
            ref = torch.cat([m(rows[c:c + 1024], cand[c:c + 1024]) for c in range(0, len(cand), 1024)])
        return cand.numpy(), ref.numpy()
    return scorer


def numpy_scorer(p, data):
    from oracle import nais_oracle

    def scorer(u):
        return nais_oracle.catalog_scores_basic(p, data.history(int(u)), data.num_pois, chunk=4096)
    return scorer


def spread_users(hist_len, n):
    """n users spread over the history lengths: shortest, longest and the quantiles between."""
    order = np.argsort(hist_len, kind="stable")
    pos = np.unique(np.round(np.linspace(0, len(order) - 1, n)).astype(np.int64))
    return [int(u) for u in order[pos]]


def self_check(p, data, users, ids, sc, k, scorer=None, oracle_name=None):
    """Oracle check of the timed path's output for a few users (test infrastructure): every
    returned id's oracle score within 1e-4 of ours, and the returned set equal to the oracle's
    top-k up to runs of scores within 4 fp32 ulps at the cut. `scorer(u)` -> (candidates, oracle
    scores); default NAIS_basic through the numpy oracle."""
    from oracle import nais_oracle
    if scorer is None:
        scorer, oracle_name = numpy_scorer(p, data), "oracle/nais_oracle.py (numpy)"
    t0 = time.perf_counter()
    out = {"users": [], "oracle": oracle_name, "max_abs_score_diff": 0.0, "topk_ok": True}
    for u in users:
        cand, ref = scorer(u)
        lut = dict(zip(cand.tolist(), ref.tolist()))
        got = np.array([lut[int(c)] for c in ids[u]])
        out["max_abs_score_diff"] = max(out["max_abs_score_diff"], float(np.max(np.abs(got - sc[u]))))
        rid, rsc = nais_oracle.topk_ids(cand, ref, k)
        cut = float(rsc[-1]) - 4 * float(np.spacing(np.float32(abs(rsc[-1]))))
        extra = set(ids[u].tolist()) - set(rid.tolist())
        ok = all(lut[c] >= cut for c in extra) and out["max_abs_score_diff"] <= 1e-4
        out["topk_ok"] = out["topk_ok"] and ok
        out["users"].append(int(u))
    out["h"] = [int(data.hist_len()[u]) for u in out["users"]]
    out["seconds"] = round(time.perf_counter() - t0, 1)
    return out


def merge_checks(*checks):
    """One self_check record from several (e.g. the numpy oracle on one user + torch_cpu on 8)."""
    checks = [c for c in checks if c]
    return {"users": sum((c["users"] for c in checks), []), "h": sum((c["h"] for c in checks), []),
            "oracle": " + ".join(f"{c['oracle']} on users {c['users']}" for c in checks),
            "max_abs_score_diff": max(c["max_abs_score_diff"] for c in checks),
            "topk_ok": all(c["topk_ok"] for c in checks),
            "seconds": round(sum(c["seconds"] for c in checks), 1)}


def prior_self_check(p, data, user, ids, sc, k, a_, b_, alpha):
    """The blended ranking of run.py:537-539 for one user: NAIS scores from the numpy oracle,
    G = powerLaw.predict per candidate (oracle/powerlaw_oracle.py, pure-Python float64),
    normalize (run.py:55-59), blend -- then the same checks as self_check on the blended f64 scores
    (relative 1e-6: the reference's libm and the device's differ by ulps in acos / pow)."""
    from oracle import nais_oracle, powerlaw_oracle
    t0 = time.perf_counter()
    hist = data.history(int(user))
    cand, pred = nais_oracle.catalog_scores_basic(p, hist, data.num_pois, chunk=4096)
    coords = [tuple(c) for c in np.asarray(data.place_coords, dtype=np.float64).tolist()]
    G = np.array([powerlaw_oracle.predict(a_, b_, coords, hist, int(c)) for c in cand])
    G = np.asarray(powerlaw_oracle.normalize(list(G)), dtype=np.float64)
    ref = powerlaw_oracle.blend(pred, G, alpha)
    lut = dict(zip(cand.tolist(), ref.tolist()))
    got = np.array([lut[int(c)] for c in ids[user]])
    diff = float(np.max(np.abs(got - sc[user].astype(np.float64))))
    rid, rsc = nais_oracle.topk_ids(cand, ref, k)
    cut = float(rsc[-1]) * (1 - 1e-6)
    extra = set(ids[user].tolist()) - set(rid.tolist())
    ok = all(lut[c] >= cut for c in extra) and diff <= 1e-4
    return {"users": [int(user)], "h": [len(hist)], "max_abs_score_diff": diff, "topk_ok": ok,
            "oracle": "oracle/nais_oracle.py + oracle/powerlaw_oracle.py (predict, normalize, blend)",
            "seconds": round(time.perf_counter() - t0, 1)}


def gather_rows_leg(dev, lib, traffic_json, rows=4_000_000, dim=128, m=4_000_000, reps=10):
    """The north star's HBM kernel on its own (nais_gather_rows = model.py:64's embedding gather):
    a 2 GB table (4M rows x d = 128, past the 256 MB Infinity Cache), 4M rows gathered in random
    permutation order (each row read once). Algorithmic bytes per launch = m x (8 B index + 4d B
    row read + 4d B row write); HIP events on the launch stream; frac against the 8 TB/s spec and
    the 6.29 TB/s measured copy ceiling (MI355X_MICROARCH.md); traffic from the committed
    FETCH_SIZE / WRITE_SIZE passes (profiles/traffic.json "gather_rows")."""
    from poi_recommendation_models_amd import _capi
    g = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(rows, dim, device=dev, generator=g)
    idx = torch.randperm(rows, device=dev, generator=g)[:m].contiguous()
    out = torch.empty(m, dim, device=dev)
    stream = torch.cuda.current_stream(dev)

    def launch():
        _capi.check(lib.nais_gather_rows(table.data_ptr(), rows, dim, idx.data_ptr(), m,
                                         out.data_ptr(), stream.cuda_stream), "nais_gather_rows")
    launch()
    torch.cuda.synchronize(dev)
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        launch()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms.append(e0.elapsed_time(e1))
    ok = bool(torch.equal(out, table.index_select(0, idx)))   # every gathered row, bit-exact
    algo = m * (8 + 8 * dim)
    avg = float(np.mean(ms))
    ach = algo / (avg * 1e-3) / 1e9
    traffic = None
    try:
        e = json.load(open(traffic_json)).get("gather_rows", {})
        if e.get("rows") == rows and e.get("dim") == dim and e.get("m") == m:
            traffic = e.get("hbm_bytes_per_launch")
    except Exception:
        pass
    del table, idx, out
    torch.cuda.empty_cache()
    return {"kernel": "gather_rows_kernel (nais_gather_rows)", "bound": "hbm", "unit": "GB/s",
            "achieved": ach, "peak": HBM_SPEC_GBS, "frac": ach / HBM_SPEC_GBS,
            "measured_hbm_peak": HBM_MEASURED_GBS, "frac_of_measured_hbm": ach / HBM_MEASURED_GBS,
            "traffic": traffic, "algorithmic_bytes_per_launch": algo, "avg_launch_ms": avg,
            "launches": reps, "table_bytes": rows * dim * 4, "rows_gathered": m, "dim": dim,
            "index_pattern": "random permutation (each row read once)", "rows_bit_exact": ok}


class EagerNAIS(torch.nn.Module):
    """The reference's NAIS_basic training forward (model.py:57-89: gather, h * t, attn_layer1,
    Dropout, ReLU, attn_layer2, exp, mask, pow(beta), divide, bmm, sigmoid) in eager PyTorch ops
    with autograd -- what run.py:101-109 runs when handed a ROCm device. Baseline timing only."""

    def __init__(self, src):
        super().__init__()
        cp = lambda t: torch.nn.Parameter(t.detach().clone())
        self.eh, self.et = cp(src.embed_history.weight), cp(src.embed_target.weight)
        self.w1, self.b1 = cp(src.attn_layer1.weight), cp(src.attn_layer1.bias)
        self.w2 = cp(src.attn_layer2.weight)
        self.drop = torch.nn.Dropout(src.drop.p)
        self.beta = src.beta

    def forward(self, hist, tgt):
        F = torch.nn.functional
        h = F.embedding(hist, self.eh)
        t = F.embedding(tgt, self.et).reshape(len(tgt), 1, -1)
        r1 = torch.relu(self.drop(F.linear(h * t, self.w1, self.b1)))
        a = torch.exp(F.linear(r1, self.w2)).squeeze(-1) * (hist != tgt.reshape(-1, 1))
        s = torch.pow(a.sum(-1), self.beta)
        w = torch.divide(a.T, s).T.reshape(len(tgt), -1, 1)
        return torch.sigmoid(torch.bmm(h * w, t.reshape(len(tgt), -1, 1)).squeeze(-1).sum(-1))


def train_batches(P, n, num_ng, count, seed):
    """get_NAIS_batch-shaped batches (batches.py:24-50): n shuffled positives shared as the
    history of n * (1 + num_ng) rows [pos, neg x num_ng], labels 1 / 0."""
    r = np.random.default_rng(seed)
    out = []
    for _ in range(count):
        pos = r.choice(P, n, replace=False)
        neg = r.choice(np.setdiff1d(np.arange(P), pos), n * num_ng, replace=False)
        data = np.concatenate([pos.reshape(-1, 1), neg.reshape(n, num_ng)], 1).reshape(-1)
        labels = np.concatenate([np.ones((n, 1)), np.zeros((n, num_ng))], 1).reshape(-1)
        out.append((pos, data, labels.astype(np.float32)))
    return out


def train_leg(dev, D, H, P=100_000, n=204, num_ng=4, steps=50, warmup=5, check=True):
    """BASELINE config 3 (run.py:91-109): one NAIS_basic training step on a get_NAIS_batch batch
    of n * (1 + num_ng) = 1,020 rows x 204 history items, P = 100k POIs, dropout 0.5, Adagrad
    lr 0.01. ms per step of (1) the fused native step (NAISTrainer.step: forward + BCELoss +
    backward + Adagrad in one C-ABI call), (2) the drop-in loop run.py runs (model(...),
    loss_func, backward(), optim.Adagrad.step()), (3) the reference's op sequence in eager
    PyTorch + torch.optim.Adagrad on the same GPU. Self-check: one fused step from fresh
    parameters against oracle/train_oracle.py (float64) with the device's dropout mask injected:
    the loss within 1e-5 and every updated parameter (all P rows) within rtol 1e-4."""
    import scipy.sparse as sp
    from poi_recommendation_models_amd import _capi, optim
    from poi_recommendation_models_amd.model import NAIS_basic
    from poi_recommendation_models_amd.trainer import NAISTrainer
    torch.manual_seed(0)
    m = NAIS_basic(P, D, H, 0.5)
    with torch.no_grad():   # trained-like embedding scale: the attention is not uniform
        m.embed_history.weight.normal_(0, 0.3)
        m.embed_target.weight.normal_(0, 0.3)
    m = m.to(dev).train()
    m.drop.p = 0.5
    m.report_nan = False              # the reference prints NaN counts (a .item() sync per call)
    m.check_shared_history = False    # batches are get_NAIS_batch-shaped by construction
    host = train_batches(P, n, num_ng, 8, seed=1)
    bs = [(torch.as_tensor(np.repeat(h[None], len(d), 0)).to(dev), torch.as_tensor(d).to(dev),
           torch.as_tensor(l).to(dev)) for h, d, l in host]
    p0 = {k: v.detach().cpu().numpy().copy() for k, v in m.named_parameters()}

    def loop(fn):
        for i in range(warmup):
            fn(*bs[i % len(bs)])
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(steps):
            fn(*bs[i % len(bs)])
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / steps * 1e3

    out = {"what": "config3 NAIS_basic training step: %d rows x %d history items, P = %d, D = %d, "
                   "H = %d, dropout 0.5, Adagrad" % (n * (1 + num_ng), n, P, D, H),
           "steps": steps, "warmup": warmup}
    rows = np.repeat(np.arange(len(host)), n)
    X = sp.csr_matrix((np.ones(len(rows)), (rows, np.concatenate([np.sort(h) for h, _, _ in host]))),
                      shape=(len(host), P))
    # (1) fused step, from fresh parameters: its first step is the self-checked one
    tr = NAISTrainer(m, X, lr=0.01, num_ng=num_ng)
    seed = 20240611
    tr.step(bs[0][0][0], bs[0][1], bs[0][2], dropout_seed=seed)
    loss0 = tr.finish()
    p1 = {k: v.detach().cpu().numpy().copy() for k, v in m.named_parameters()}
    out["fused_ms_per_step"] = loop(lambda h, d, l: tr.step(h[0], d, l))
    tr.finish()
    # (2) the drop-in loop
    opt = optim.Adagrad(m.parameters(), lr=0.01)
    m.loss_func.check_input = False     # finite by construction (no single-item histories)

    def dropin(h, d, l):
        opt.zero_grad()
        m.loss_func(m(h, d), l).backward()
        opt.step()
    out["dropin_ms_per_step"] = loop(dropin)
    # (3) eager PyTorch, the reference's ops
    em = EagerNAIS(m).to(dev).train()
    eopt = torch.optim.Adagrad(em.parameters(), lr=0.01)
    bce = torch.nn.BCELoss()

    def eager(h, d, l):
        eopt.zero_grad()
        bce(em(h, d), l).backward()
        eopt.step()
    out["torch_eager_ms_per_step"] = loop(eager)
    out["fused_speedup_vs_eager"] = out["torch_eager_ms_per_step"] / out["fused_ms_per_step"]
    out["dropin_speedup_vs_eager"] = out["torch_eager_ms_per_step"] / out["dropin_ms_per_step"]
    if check:
        from oracle import train_oracle
        t0 = time.perf_counter()
        b = len(host[0][1])
        keep = torch.empty(b * n * H, dtype=torch.uint8, device=dev)
        _capi.check(_capi.load().nais_dropout_mask(seed, b, n, H, 0.5, keep.data_ptr(),
                                                   _capi.stream_handle(dev)), "nais_dropout_mask")
        keep = keep.view(b, n, H).cpu().numpy()
        h, d, l = host[0]
        r = train_oracle.train_step_basic(p0, np.repeat(h[None], b, 0), d, l, keep=keep, drop_p=0.5)
        # every element within atol 2e-5 + rtol 1e-4 of the oracle, widened only by its Adagrad
        # slack lr * min(2, 2e-4 max|g| / |g|): the first step's lr * g / |g| amplifies the
        # gradient's rounding (tolerance 1e-4 max|g|) where |g| is small against the tensor's
        # largest (tests/_helpers.py::adagrad_slack)
        bad, unexplained, worst_dev, over_limit, per_tensor = 0, 0, 0.0, 0, {}
        for k, v in p0.items():
            g = r["grads"][k].reshape(v.shape)
            want, _ = train_oracle.adagrad(v, np.zeros_like(v), g, 0.01, 1)
            dev = np.abs(p1[k].astype(np.float64) - want)
            plain = 2e-5 + 1e-4 * np.abs(want)
            ga = np.abs(g.astype(np.float64))
            with np.errstate(divide="ignore", invalid="ignore"):
                slack = 0.01 * np.minimum(2.0, np.where(ga > 0, 2e-4 * ga.max() / ga, 2.0))
            miss = dev > plain
            bad += int(miss.sum())
            unexplained += int((dev > plain + slack).sum())
            # as tests/_helpers.assert_params_close: at most 0.1 % of a tensor, and 32, may need
            # the slack
            over_limit += int(miss.sum()) > min(32, int(1e-3 * miss.size))
            if miss.any():
                worst_dev = max(worst_dev, float(dev[miss].max()))
                per_tensor[k] = {"count": int(miss.sum()), "size": int(miss.size),
                                 "max_g_ratio": float(ga[miss].max() / max(ga.max(), 1e-300))}
        out["self_check"] = {"oracle": "oracle/train_oracle.py (float64, dropout mask injected)",
                             "loss": loss0, "oracle_loss": float(r["loss"]),
                             "loss_ok": abs(loss0 - float(r["loss"])) <= 1e-5,
                             "params_off_rtol_1e-4": bad, "params_beyond_adagrad_slack": unexplained,
                             "slack_elements_by_tensor": per_tensor,
                             "tensors_over_slack_limit": over_limit,
                             "max_dev_off": worst_dev,
                             "params_ok": unexplained == 0 and over_limit == 0,
                             "seconds": round(time.perf_counter() - t0, 1)}
    del tr, opt, em, eopt, m
    torch.cuda.empty_cache()
    return out


def table_kernel_name(precision, D, H, variant="basic", mode="table"):
    """The catalog kernel nais_pair_table (mode "table") or nais_score_catalog (mode "direct")
    runs for this shape -- nais_kernels.hip's dispatch: pair_table_impl sends fp16x6 AND
    fp16x6_pairsplit to launch_catalog_x6b, the direct route sends fp16x6_pairsplit to
    launch_catalog_x6 (the per-pair split kernel); launch_catalog_x3b takes x6n for D in
    {32, 64, 128} at any H <= 256 when NPC = 3."""
    dist = variant in ("region_distance", "distance")
    if precision == "fp32" or D < 16:
        return "catalog_score_kernel"
    fp16x6 = precision.startswith("fp16x6")
    x6b = fp16x6 and (mode == "table" or precision == "fp16x6")
    if x6b and D in (32, 64, 128) and H <= 256:
        return ("catalog_score_x6n_kernel (16x16x32 f16 MFMA%s)"
                % (" + 16x16x1_4b f32 K-steps for the distance features" if dist else ""))
    if precision.endswith("pairsplit") and not x6b:
        return "catalog_score_x3_kernel"
    if (dist or fp16x6) and (D > 64 or H > 64):
        return "catalog_score_x3_kernel"
    return "catalog_score_x3b_kernel"


def self_launch(a):
    """--gpus N > 1 without a torchrun environment: start N fresh worker processes through
    torch.distributed.run (this process never touches the GPU) and return their exit code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__),
           *sys.argv[1:]]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def main():
    a = parse()
    if a.config == 2:
        a.num_users, a.num_pois, a.dim, a.hidden, a.h_max = 10_000, 50_000, 64, 64, 100
    if a.config == 5:
        a.num_users, a.num_pois, a.dim, a.hidden = 200_000, 1_000_000, 128, 128
        if a.users_per_step == 256:
            a.users_per_step = 64
        a.no_cpu_baseline = True   # the CPU leg is quoted on the metric config (4)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(self_launch(a))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
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
    strategy = a.strategy if a.strategy != "auto" else ("direct" if a.config == 5 else "pairs")
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
                dist.all_gather_into_tensor(gat_ids, ids)
                dist.all_gather_into_tensor(gat_sc, top)

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
            cpu = cpu_baseline(p_host, data, np.arange(a.cpu_users), K, a.cpu_seconds)
        out = {
            "metric": "scored (user,POI) pairs/sec full-catalog + top-50, %s POIs"
                      % {2: "50k", 4: "100k", 5: "1M"}[a.config],
            "value": pairs_total / elapsed,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": DTYPES[a.precision],
            "data": "synthetic (seeded CSR check-ins, h~U{1..%d}; random-init weights N(0,0.3))" % a.h_max,
            "config": {
                "workload": {2: "config2 synthetic", 4: "config4 Gowalla-scale"}.get(
                    a.config, "config5 stress (timed on the first 4096 users)") +
                            ": %d users x %d POIs, d=H=%d, full-catalog NAIS_basic score + top-%d"
                            % (a.num_users, P, D, K),
                "table_allgather_ms": gather_ms,
                "model": "NAIS_basic", "users_per_step_per_gpu": B, "num_pois": P,
                "embed_dim": D, "hidden": H, "h_max": a.h_max, "topk": K,
                "pairs_per_step_per_gpu": pairs / a.steps,
                "parallelism": f"users sharded (LPT) over {world} GPU(s), POI tables replicated",
            },
            "roofline": {
                "kernel": ("catalog_score_x3_kernel" if "pairsplit" in a.precision
                           else table_kernel_name(a.precision, D, H, mode="direct")) + " (nais_score_catalog)",
                "bound": "mfma",
                "achieved": achieved,
                "peak": peak,
                "peak_basis": ("fp32 MFMA dense" if a.precision == "fp32" else
                               "f16 MFMA dense 2.5 PF / %d products per algorithmic fp32 product"
                               % PRODUCTS[a.precision]),
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


PRIOR_A, PRIOR_B, PRIOR_ALPHA = 0.052, -1.37, 0.2   # a typical PowerLaw fit (a, b) and run.py's alpha


def bench_pairs(a, model, csr, data, hist_len, p_host, dev, rank, world, dist):
    """Whole-job steps through sharding.distributed_topk_pairs (the product path)."""
    from poi_recommendation_models_amd import catalog
    from poi_recommendation_models_amd.sharding import column_blocks, distributed_topk_pairs
    if a.ab:   # A/B knobs of the table/gather overlap, only when asked for (--ab)
        if os.environ.get("NAIS_PAIR_TABLE_CUS"):
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
    # --emulate-world N (one process): time rank 0's column shard of an N-GPU run (its tables,
    # gathers and local top-k; no collective) -- per-rank cost and strong-scaling headroom on one GPU
    emulate = a.emulate_world
    P, D, H, K = a.num_pois, a.dim, a.hidden, a.topk
    users = np.arange(a.num_users)
    group = None
    last = {}
    if world == 1:   # the same code path with a trivial process group is not needed: call direct
        from poi_recommendation_models_amd.catalog import _score_topk_pairs

        S_em = (a.num_pois + emulate - 1) // emulate

        def job(events=None):
            return _score_topk_pairs(model, csr, users, K, None, None, None, None, force=True,
                                     events=events, cols=(0, S_em) if emulate > 1 else None)
    else:
        def job(events=None):
            return distributed_topk_pairs(model, csr, users, K, group=group, events=events)

    def run(precision, nwarm, nsteps, fn=None):
        fn = fn or job
        model.precision = precision
        for _ in range(nwarm):
            fn()
        evs = [[] for _ in range(nsteps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(nsteps):
            last["out"] = fn(evs[i])
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        last["wall_ms"] = el / nsteps * 1e3
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        per, nl, span = {}, {}, {}
        for step_ev in evs:
            ref = next((e0 for _, e0, _, _ in step_ev if e0 is not None), None)
            spans = {}
            for kind, e0, e1, launches in step_ev:
                if e0 is None:          # a setting, not a timed launch
                    per[kind] = launches
                    continue
                spans.setdefault(kind, []).append((ref.elapsed_time(e0), ref.elapsed_time(e1)))
                nl[kind] = nl.get(kind, 0) + launches
                span.setdefault(kind, []).append(spans[kind][-1][1] - spans[kind][-1][0])
            # busy time of each kind = the union of its launch intervals: the table launches of
            # consecutive blocks overlap (two table streams, catalog.PAIR_TABLE_STREAMS)
            for kind, iv in spans.items():
                busy, end = 0.0, -1e30
                for lo, hi in sorted(iv):
                    if hi > end:
                        busy += hi - max(lo, end)
                        end = hi
                per.setdefault(kind, []).append(busy)
        per["_launches"] = nl
        # mean span of one launch (its own HIP events, on its own stream): what rocprofv3 reports
        # as a dispatch's duration, overlap with the other table stream included
        per["_span_ms"] = {kd: float(np.mean(v)) for kd, v in span.items()}
        return el, per

    elapsed, per = run(a.precision, a.warmup, a.steps)
    wall_ms = last["wall_ms"]
    head_out = last["out"]   # the legs below overwrite last["out"]
    ranks = None
    if world > 1:   # every rank's phase busy times (ms per step), gathered over the same group
        ph = ("table", "gather", "allgather", "merge", "topk")
        mine = torch.tensor([sum(per.get(kind, [])) / a.steps for kind in ph] + [wall_ms],
                            dtype=torch.float64, device=dev)
        allr = torch.empty(world * len(mine), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(allr, mine)
        allr = allr.view(world, -1).cpu().numpy()
        ranks = {"world_size_reported": dist.get_world_size(), "backend": dist.get_backend(),
                 "phases": ph + ("wall",),
                 "ms_per_step_by_rank": [[round(float(x), 3) for x in row] for row in allr],
                 "note": "busy time (union of launch intervals, HIP events) of each phase per step on "
                         "each rank; allgather = the two all_gather_into_tensor calls of the [users, 50] "
                         "blocks, merge = the top-k over world x 50 candidates; wall = this rank's own "
                         "timed region / steps (value uses the max over ranks)"}
    pairs_job = float((P - hist_len[users]).sum())            # every user's whole catalog
    if emulate > 1 and world == 1:
        c0, c1 = column_blocks(P, emulate)[0]
        pairs_job /= emulate     # ~ the shard's share (value is then a per-rank rate estimate)
    else:
        c0, c1 = column_blocks(P, world)[rank]
    NC = c1 - c0
    entries = int(hist_len.sum())
    J = int(np.count_nonzero(np.bincount(data.indices, minlength=P)))
    fused = catalog.PAIR_FUSED_TOPK and K <= 256
    Wb = catalog.PAIR_BLOCK_COLS

    def stripes_of(bounded):
        st_w = catalog.PAIR_BOUNDED_STRIPE if bounded else catalog.PAIR_STRIPE
        return sum((min(Wb, NC - b) + st_w - 1) // st_w for b in range(0, NC, Wb)), st_w
    flop_per_pair_item = 2 * D * H + 3 * H + 4 * D
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count

    def kernels(per, precision, flop_item=None, kname=None, steps=None):
        """(gather roofline dict, table roofline dict) of one leg's per-step event timings
        (`flop_item`: algorithmic FLOP per (pair, history item) when not NAIS_basic's; `steps`:
        the leg's timed steps when not a_steps[precision])."""
        ns = steps or a_steps[precision]
        bounded = bool(per.get("bounded"))
        stripes, st_w = stripes_of(bounded)
        # table rows (8 B per history entry x column; the bounded gather: 4 B, the hi words) + each
        # stripe's CSR ids and row map (12 B per entry) + score rows (4 B per user x column; the
        # fused kernels write only the top-k merges); with PAIR_TABLE_GATHER_FRAC > 0 only the
        # gather stream's share is timed
        gbytes = (entries * NC * (4 if bounded else 8) + entries * 12 * stripes
                  + (0 if fused else a.num_users * NC * 4))
        gbytes *= per.get("gather_share", 1.0)
        g_ms = sum(per.get("gather", [])) / ns
        t_ms = sum(per.get("table", [])) / ns
        n_gl = max(1, per["_launches"].get("gather", 0) // ns)
        table_cus = per.get("table_cus", ncu) or ncu
        tflops = J * NC * (flop_item or flop_per_pair_item)
        g_ach = gbytes / (g_ms * 1e-3) / 1e9 if g_ms else None
        t_ach = tflops / (t_ms * 1e-3) / 1e12 if t_ms else None
        gcus = ncu - table_cus if table_cus < ncu else ncu
        gather = {
            "kernel": ("pair_bound_topk_kernel (nais_pair_bound_topk)" if bounded else
                       "pair_gather_topk_kernel (nais_pair_gather_topk)" if fused else
                       "pair_gather_kernel (nais_pair_gather)"),
            "bound": "hbm", "achieved": g_ach, "peak": HBM_SPEC_GBS, "unit": "GB/s",
            "frac": g_ach / HBM_SPEC_GBS if g_ach else None,
            "frac_of_measured_hbm": g_ach / HBM_MEASURED_GBS if g_ach else None,
            "measured_hbm_peak": HBM_MEASURED_GBS,
            "served_from": ("Infinity Cache (MALL) mostly: the %d-column stripe of the tables "
                            "(J x %d x %d B ~ %.0f MB) fits the 256 MB MALL, so the memory side "
                            "delivers more than the HBM copy rate"
                            % (st_w, st_w, 4 if bounded else 8, J * st_w * (4 if bounded else 8) / 1e6)),
            "algorithmic_bytes_per_launch": gbytes / n_gl, "avg_launch_ms": g_ms / n_gl,
            "launches_per_step": n_gl, "ms_per_step": g_ms, "cus": gcus,
        }
        if bounded:
            gather["refine_ms_per_step"] = sum(per.get("refine", [])) / ns
            gather["route"] = ("bounded: split16 tables, the gather streams the hi words (e, e*s "
                               "truncated to 8 significant bits) and keeps per user the k best lower "
                               "bounds + the candidates whose upper bound reaches them; the refine "
                               "recomputes those exactly from hi + lo in CSR order (the exact "
                               "gather's bits, exact_gather_path.identical)")
        table = {
            "kernel": (kname or table_kernel_name(precision, D, H)) + " in table mode (nais_pair_table)",
            "bound": "mfma", "achieved": t_ach, "peak": PEAKS[precision], "unit": "TFLOP/s",
            "frac": t_ach / PEAKS[precision] if t_ach else None,
            "frac_of_its_cus": t_ach / (PEAKS[precision] * table_cus / ncu) if t_ach else None,
            "peak_basis": ("fp32 MFMA dense" if precision == "fp32" else
                           "f16 MFMA dense 2.5 PF / %d products per algorithmic fp32 product"
                           % PRODUCTS[precision]),
            "algorithmic_flop_per_step": tflops, "ms_per_step": t_ms, "cus": table_cus,
            "launches_per_step": per["_launches"].get("table", 0) // ns,
            # achieved = the step's FLOP / the union of the table launches' intervals; a launch's own
            # span is longer, since consecutive blocks overlap on the two table streams
            "avg_launch_ms": per.get("_span_ms", {}).get("table"),
            "busy_ms_per_launch": t_ms / max(1, per["_launches"].get("table", 0) // ns),
            "table_streams": catalog.PAIR_TABLE_STREAMS,
        }
        nlt = max(1, per["_launches"].get("table", 0) // ns)
        if table["avg_launch_ms"]:
            # the literal per-launch rate (FLOP of one launch / its own span): with two table
            # streams each launch shares its span with the other stream's, so the kernel's
            # throughput (`achieved`) is ~streams x this
            table["achieved_per_launch_span"] = tflops / nlt / (table["avg_launch_ms"] * 1e-3) / 1e12
            table["achieved_basis"] = ("achieved = FLOP per step / the union of the table launches' "
                                       "intervals (HIP events on both table streams)")
        return gather, table

    a_steps = {a.precision: a.steps}
    gather, table = kernels(per, a.precision)
    k_ms = sum(per.get("topk", [])) / a.steps
    # the roofline line is the kernel on the job's critical path (the longer of the two streams)
    dominant = table if (table["ms_per_step"] or 0) > (gather["ms_per_step"] or 0) else gather
    other = gather if dominant is table else table
    try:   # the PMC traffic of both kernels (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, profiles/)
        tj = json.load(open(a.traffic_json))
        gkey = ("pairs_bound_topk" if per.get("bounded") else
                "pairs_gather_topk" if fused else "pairs_gather")
        for dct, key in ((gather, gkey), (table, "pairs_table_" + a.precision)):
            e = tj.get(key, {})
            ok = (e.get("num_users") == a.num_users and e.get("num_pois") == P and e.get("world") == world
                  and e.get("block_cols") == catalog.PAIR_BLOCK_COLS
                  and e.get("precision", a.precision) == a.precision)
            dct["traffic"] = e.get("hbm_bytes_per_launch") if ok else None
            if ok and dct is table:
                dct["traffic_note"] = "per launch (one 512-column table block)"
    except Exception:
        pass
    for dct in (gather, table):
        dct.setdefault("traffic", None)
    dominant["note"] = ("gather: algorithmic bytes per launch (one %d-column stripe) = sum_u h_u x "
                        "columns x %d B table reads + 12 B CSR id + row map per history entry; table: "
                        % (stripes_of(bool(per.get("bounded")))[1], 4 if per.get("bounded") else 8) +
                        "SURVEY.md 8(d) FLOP per (pair, history item) x distinct history POIs x "
                        "columns; traffic = rocprofv3 (2 x FETCH_SIZE + WRITE_SIZE) per launch")
    dominant["overlap"] = ("tables on CUs [0, %d) and gathers on the other %d, side by side on "
                           "CU-masked streams (double-buffered tables)" % (table["cus"], ncu - table["cus"])
                           if table["cus"] < ncu else "serial")
    dominant["other_kernel"] = other
    dominant["topk_ms_per_step"] = k_ms
    legs = {}
    if world == 1 and per.get("bounded"):
        # the same job on the exact fused gather (float tables, 8 B per history entry and column):
        # its time, and the headline's lists against it -- the same ids and score bits
        catalog.PAIR_BOUNDED = False
        try:
            el_x, per_x = run(a.precision, 1, a.leg_steps)
        finally:
            catalog.PAIR_BOUNDED = True
        g_x, t_x = kernels(per_x, a.precision, steps=a.leg_steps)
        xi, xs = (t.cpu().numpy() for t in last["out"])
        hi_, hs_ = (t.cpu().numpy() for t in head_out)
        st = getattr(model, "_last_bound_stats", None)
        st = st.cpu().numpy() if st is not None else None
        legs["exact_gather"] = {
            "what": "the exact fused gather (pair_gather_topk_kernel on float e / e*s tables) on the "
                    "same job",
            "value": pairs_job * a.leg_steps / el_x, "unit": "pairs/s", "steps": a.leg_steps,
            "ms_per_step": el_x / a.leg_steps * 1e3, "gather": g_x, "table_ms_per_step": t_x["ms_per_step"],
            "identical": bool(np.array_equal(xi, hi_) and np.array_equal(xs.view(np.uint32), hs_.view(np.uint32))),
            "users": int(xi.shape[0]),
            "bounded_refined_per_user": None if st is None else float(st[0]) / max(1, a.num_users),
            "bounded_overflowed_users": None if st is None else int(st[1])}
    if world == 1 and not a.no_fp32_leg:
        for prec in ("fp32", "fp16x3"):
            if prec == a.precision:
                continue
            a_steps[prec] = a.leg_steps
            el_l, per_l = run(prec, 1, a.leg_steps)
            g_l, t_l = kernels(per_l, prec)
            leg_check = None
            if not a.no_self_check:   # 2 users of this leg's last job against the restatement
                li, ls = (t.cpu().numpy() for t in last["out"])
                leg_check = self_check(p_host, data, spread_users(hist_len, 2), li, ls, K,
                                       scorer=torch_scorer(p_host, data),
                                       oracle_name="oracle/torch_cpu.py")
            legs[prec] = {"precision": DTYPES[prec], "value": pairs_job * a.leg_steps / el_l,
                          "unit": "pairs/s", "steps": a.leg_steps, "warmup": 1,
                          "ms_per_step": el_l / a.leg_steps * 1e3,
                          "table_ms_per_step": t_l["ms_per_step"], "table_tflops": t_l["achieved"],
                          "table_peak_tflops": t_l["peak"], "table_cus": t_l["cus"],
                          "gather_ms_per_step": g_l["ms_per_step"], "self_check": leg_check}
        model.precision = a.precision
        def prior_job(events=None):
            return _score_topk_pairs(model, csr, users, K, None, None, None, None, force=True,
                                     events=events, prior=(PRIOR_A, PRIOR_B, PRIOR_ALPHA, data.place_coords))
        el_p, per_p = run(a.precision, 1, a.leg_steps, prior_job)
        pr_out = last["out"]
        legs["prior"] = {"value": pairs_job * a.leg_steps / el_p, "unit": "pairs/s", "steps": a.leg_steps,
                         "warmup": 1, "ms_per_step": el_p / a.leg_steps * 1e3,
                         # the plan of the timed jobs (identical every step: the pass split is sized
                         # from the memory this process can allocate, cached blocks included)
                         "plan": {key: per_p.get(key) for key in (
                             "passes", "users_per_pass", "block_cols", "distinct_rows", "table_cus",
                             "usable_bytes", "budget_bytes")},
                         "table_ms_per_step": sum(per_p.get("table", [])) / a.leg_steps,
                         "gather_ms_per_step": sum(per_p.get("gather", [])) / a.leg_steps,
                         "blend_topk_ms_per_step": sum(per_p.get("topk", [])) / a.leg_steps}
        if not a.no_self_check:   # a short-history user: the pure-Python prior is O(h x P)
            pu = int(np.argmin(np.abs(hist_len - 12)))
            legs["prior"]["self_check"] = prior_self_check(
                p_host, data, pu, pr_out[0].cpu().numpy(), pr_out[1].cpu().numpy(), K,
                PRIOR_A, PRIOR_B, PRIOR_ALPHA)
        legs["prior"]["what"] = ("the same job ranked on the power-law-blended score (run.py:537-539): "
                                 "pr_d(dist) pair table + float64 product gather per user, score rows, "
                                 "nais_topk_blend_rows; a, b, alpha = %g, %g, %g" % (PRIOR_A, PRIOR_B, PRIOR_ALPHA))
        from poi_recommendation_models_amd.model import NAIS_region_distance_Embedding
        from poi_recommendation_models_amd.synthetic import init_nais_params as _init
        rd = NAIS_region_distance_Embedding(P, D, H, 0.5, 1024, 1)
        p_rd = _init(P, D, H, seed=11, emb_std=0.3, bias_std=0.1, variant="region_distance", num_regions=1024)
        rd.load_state_dict({k: torch.from_numpy(v) for k, v in p_rd.items()}, strict=False)
        rd = rd.to(dev).eval()
        rd.report_nan = False
        rd.precision = a.precision
        def rd_job(events=None):
            return _score_topk_pairs(rd, csr, users, K, data.region_of, data.place_coords, None, None,
                                     force=True, events=events)
        el_rd, per_rd = run(a.precision, 1, a.leg_steps, rd_job)
        rd_out = last["out"]
        # SURVEY.md 8(d) FLOP per (pair, history item) with din = D + 2 (the distance columns)
        flop_rd = 2 * (D + 2) * H + 3 * H + 4 * D
        g_rd, t_rd = kernels(per_rd, a.precision, flop_item=flop_rd, steps=a.leg_steps,
                             kname=table_kernel_name(a.precision, D, H, "region_distance"))
        t_rd["algorithmic_flop_per_pair_item"] = flop_rd
        legs["region_distance"] = {"value": pairs_job * a.leg_steps / el_rd, "unit": "pairs/s",
                                   "steps": a.leg_steps, "warmup": 1,
                                   "ms_per_step": el_rd / a.leg_steps * 1e3,
                                   "roofline": t_rd, "gather": g_rd}
        if not a.no_self_check:   # 8 users spread over h against the torch restatement of
            from oracle import torch_cpu   # validation.py:69-121 (pinned to the reference's lists)
            trd = torch_cpu.TorchNAISRegionDistance(p_rd)
            legs["region_distance"]["self_check"] = self_check(
                p_rd, data, spread_users(hist_len, 8), rd_out[0].cpu().numpy(), rd_out[1].cpu().numpy(), K,
                scorer=lambda u: torch_cpu.region_distance_scores(
                    trd, data.history(int(u)), P, data.region_of, data.place_coords),
                oracle_name="oracle/torch_cpu.py (region_distance)")
        legs["region_distance"]["what"] = ("NAIS_region_distance_Embedding (model.py:246-297) on the same "
                                           "users / POIs: [h | region] rows, distance features from the POI "
                                           "coordinates, %s tables" % a.precision)
        del rd
    if world == 1 and not a.no_gather_leg:
        from poi_recommendation_models_amd import _capi
        legs["gather_rows"] = gather_rows_leg(dev, _capi.load(), a.traffic_json)
    if world == 1 and not a.no_train_leg:
        legs["train_step"] = {"D=H=%d" % d: train_leg(dev, d, d, check=not a.no_self_check)
                              for d in (64, 128)}
    check = None
    if emulate == 1 and not a.no_self_check and rank == 0:   # N > 1: the merged top-k
        ids, sc = (t.cpu().numpy() for t in head_out)
        # 8 users spread over h through the torch-CPU restatement, user 1 through the numpy oracle
        check = merge_checks(self_check(p_host, data, [1], ids, sc, K),
                             self_check(p_host, data, spread_users(hist_len, 8), ids, sc, K,
                                        scorer=torch_scorer(p_host, data),
                                        oracle_name="oracle/torch_cpu.py"))
    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            cpu = cpu_baseline(p_host, data, np.arange(a.cpu_users), K, a.cpu_seconds)
        out = {
            "metric": "scored (user,POI) pairs/sec full-catalog + top-50, %s POIs"
                      % {2: "50k", 4: "100k", 5: "1M"}[a.config],
            "value": pairs_job * a.steps / elapsed,
            "per_rank": ranks,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": DTYPES[a.precision],
            "data": "synthetic (seeded CSR check-ins, h~U{1..%d}; random-init weights N(0,0.3))" % a.h_max,
            "world_size": world,
            "backend": (a.backend if world > 1 else None),
            "config": {
                "workload": "%s: %d users x %d POIs, d=H=%d, full-catalog NAIS_basic score + top-%d; "
                            "one step = every user's whole catalog"
                            % ({2: "config2 synthetic", 4: "config4 Gowalla-scale"}.get(a.config, "config5 stress"), a.num_users, P, D, K),
                "model": "NAIS_basic", "strategy": "pairs", "precision": a.precision,
                "num_users": a.num_users, "num_pois": P,
                "table_cus": table["cus"], "cu_layout": catalog.PAIR_CU_LAYOUT,
                "block_cols": catalog.PAIR_BLOCK_COLS,
                "first_table_all_cus": catalog.PAIR_FIRST_TABLE_ALL_CUS,
                "table_streams": catalog.PAIR_TABLE_STREAMS,
                "table_gather_frac": catalog.PAIR_TABLE_GATHER_FRAC,
                "fused_topk": catalog.PAIR_FUSED_TOPK, "lpt_order": catalog.PAIR_LPT_ORDER,
                **({"emulated_world_shard": emulate} if emulate > 1 and world == 1 else {}),
                "embed_dim": D, "hidden": H, "h_max": a.h_max, "topk": K,
                "pairs_per_step": pairs_job, "history_entries": entries, "distinct_history_pois": J,
                "parallelism": f"POI columns sharded over {world} GPU(s) (all users per rank), "
                               "tables replicated, one all-gather + merge of the top-k blocks",
            },
            "roofline": dominant,
            "cpu_baseline": cpu,
            "self_check": check,
            "exact_gather_path": legs.get("exact_gather"),
            "fp32_path": legs.get("fp32"),
            "fp16x3_path": legs.get("fp16x3"),
            "prior_path": legs.get("prior"),
            "region_distance_path": legs.get("region_distance"),
            "gather_rows_path": legs.get("gather_rows"),
            "train_step_path": legs.get("train_step"),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
