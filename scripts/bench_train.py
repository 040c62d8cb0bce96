"""Config 3: one NAIS_basic training step -- get_NAIS_batch batch (batches.py:24-50,
n positives x (1 + 4 negatives) rows sharing the history), forward in train mode (dropout 0.5),
BCELoss, backward, Adagrad (run.py:101-109) -- timed on one GPU.

Legs (one JSON line):
  hip      NAIS_basic (train mode) + optim.Adagrad (row update), the reference's loop unchanged
  fused    NAISTrainer.step: forward + BCELoss + backward + Adagrad in one C-ABI call
  fused+batch  NAISTrainer.batch + step: get_NAIS_batch built on the device too (8(f2))
  kernels  the two training kernels alone (HIP events on the launch stream) with their MFMA
           FLOP rate: forward 2*H*D flops per pair, backward 3 x 2*H*D (u recompute, dx, dW1)
  torch    the reference's own op sequence (model.py:57-89 restated in eager PyTorch, autograd,
           torch.optim.Adagrad) on the same GPU -- what run.py does when given a ROCm device
  cpu      the oracle (float64 numpy restatement) for one step on the host (--cpu)
Batches are synthetic (seeded), built on the host and copied to the device before timing.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from poi_recommendation_models_amd import _capi, optim  # noqa: E402
from poi_recommendation_models_amd.model import NAIS_basic  # noqa: E402
from poi_recommendation_models_amd.trainer import NAISTrainer  # noqa: E402


def batches(P, n, num_ng, count, seed):
    r = np.random.default_rng(seed)
    out = []
    for _ in range(count):
        pos = r.choice(P, n, replace=False)
        cand = r.choice(P, n * num_ng + n, replace=False)
        neg = np.setdiff1d(cand, pos)[:n * num_ng]
        r.shuffle(neg)
        data = np.concatenate([pos.reshape(-1, 1), neg.reshape(n, num_ng)], 1).reshape(-1)
        labels = np.concatenate([np.ones((n, 1)), np.zeros((n, num_ng))], 1).reshape(-1)
        hist = np.repeat(pos.reshape(1, -1), len(data), 0)
        out.append((hist, data, labels.astype(np.float32)))
    return out


class TorchNAIS(torch.nn.Module):
    """model.py:8-97 (NAIS_basic) in eager PyTorch: the reference's path on the GPU."""

    def __init__(self, src):
        super().__init__()
        self.embed_history = torch.nn.Embedding.from_pretrained(src.embed_history.weight.detach().clone(), freeze=False)
        self.embed_target = torch.nn.Embedding.from_pretrained(src.embed_target.weight.detach().clone(), freeze=False)
        self.attn_layer1 = torch.nn.Linear(*reversed(src.attn_layer1.weight.shape))
        self.attn_layer2 = torch.nn.Linear(src.attn_layer2.weight.shape[1], 1, bias=False)
        self.attn_layer1.load_state_dict(src.attn_layer1.state_dict())
        self.attn_layer2.load_state_dict(src.attn_layer2.state_dict())
        self.drop = torch.nn.Dropout()
        self.beta = src.beta

    def forward(self, hist, tgt):
        h = self.embed_history(hist)
        t = self.embed_target(tgt).reshape(len(tgt), 1, -1)
        r1 = torch.relu(self.drop(self.attn_layer1(h * t)))
        a = torch.exp(self.attn_layer2(r1)).squeeze(-1) * (hist != tgt.reshape(-1, 1))
        s = torch.pow(a.sum(-1), self.beta)
        w = torch.divide(a.T, s).T.reshape(len(tgt), -1, 1)
        return torch.sigmoid(torch.bmm(h * w, t.reshape(len(tgt), -1, 1)).squeeze(-1).sum(-1))


def time_loop(fn, bs, warmup, steps):
    for i in range(warmup):
        fn(*bs[i % len(bs)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(*bs[i % len(bs)])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=100_000)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--H", type=int, default=64)
    ap.add_argument("--n", type=int, default=204)
    ap.add_argument("--num-ng", type=int, default=4)
    ap.add_argument("--dropout", type=float, default=0.5)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = NAIS_basic(a.P, a.D, a.H, 0.5)
    with torch.no_grad():   # trained-like scale so the attention is not uniform
        m.embed_history.weight.normal_(0, 0.3)
        m.embed_target.weight.normal_(0, 0.3)
    m = m.to(dev).train()
    m.drop.p = a.dropout
    m.report_nan = False            # the reference prints NaN counts with a .item() sync
    m.loss_func.check_input = False # finite by construction (no single-item histories)
    m.check_shared_history = False  # batches are get_NAIS_batch-shaped by construction
    host = batches(a.P, a.n, a.num_ng, 8, seed=1)
    bs = [(torch.as_tensor(h).to(dev), torch.as_tensor(d).to(dev), torch.as_tensor(l).to(dev))
          for h, d, l in host]
    b = bs[0][1].numel()
    opt = optim.Adagrad(m.parameters(), lr=0.01)

    def hip_step(hist, data, labels):
        opt.zero_grad()
        loss = m.loss_func(m(hist, data), labels)
        loss.backward()
        opt.step()

    out = {"config": {"workload": "config3 NAIS_basic training step", "num_pois": a.P, "embed": a.D,
                      "hidden": a.H, "history": a.n, "rows": b, "dropout": a.dropout},
           "data": "synthetic get_NAIS_batch-shaped batches (seeded)"}
    t = time_loop(hip_step, bs, a.warmup, a.steps)
    out["hip_ms_per_step"] = t * 1e3

    # ---- fused native step (same batches), then with device-side batch construction
    import scipy.sparse as sp
    rows = np.repeat(np.arange(len(host)), a.n)
    cols = np.concatenate([np.sort(h[0]) for h, _, _ in host])
    X = sp.csr_matrix((np.ones(len(cols)), (rows, cols)), shape=(len(host), a.P))
    tr = NAISTrainer(m, X, lr=0.01, num_ng=a.num_ng)
    out["fused_ms_per_step"] = time_loop(lambda h, d, l: tr.step(h[0], d, l), bs, a.warmup, a.steps) * 1e3
    users = [(u,) for u in range(len(host))]
    out["fused_with_batch_ms_per_step"] = time_loop(lambda u: tr.step(*tr.batch(u)), users, a.warmup,
                                                    a.steps) * 1e3
    tr.finish()

    # ---- kernels alone, on their own stream, HIP events
    lib = _capi.load()
    prm = m.nais_params()
    hist1, data1 = bs[0][0][0].contiguous(), bs[0][1]
    n = hist1.numel()
    pred = torch.empty(b, device=dev)
    saved = torch.empty(2 * b, device=dev)
    gp = torch.randn(b, device=dev) * 1e-3
    ws_bytes = lib.nais_train_workspace_size(prm, b, n)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    g = [torch.zeros_like(p) for p in m.parameters()]
    st = torch.cuda.Stream(dev)
    sh = st.cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def fwd():
        _capi.check(lib.nais_train_forward(prm, hist1.data_ptr(), n, data1.data_ptr(), b, a.dropout, 7,
                                           pred.data_ptr(), saved.data_ptr(), None, ws.data_ptr(),
                                           ws_bytes, sh), "fwd")

    def bwd():
        _capi.check(lib.nais_train_backward(prm, hist1.data_ptr(), n, data1.data_ptr(), b, a.dropout, 7,
                                            pred.data_ptr(), saved.data_ptr(), gp.data_ptr(),
                                            *[x.data_ptr() for x in g], ws.data_ptr(), ws_bytes, sh), "bwd")
    with torch.cuda.stream(st):
        for _ in range(3):
            fwd()
            bwd()
        ev[0].record(st)
        for _ in range(a.kernel_iters):
            fwd()
        ev[1].record(st)
        for _ in range(a.kernel_iters):
            bwd()
        ev[2].record(st)
    st.synchronize()
    f_ms = ev[0].elapsed_time(ev[1]) / a.kernel_iters
    b_ms = ev[1].elapsed_time(ev[2]) / a.kernel_iters
    pairs = b * n
    out["kernels"] = {"forward_ms": f_ms, "backward_ms": b_ms,
                      "forward_tflops": pairs * 2 * a.H * a.D / (f_ms * 1e-3) / 1e12,
                      "backward_tflops": pairs * 6 * a.H * a.D / (b_ms * 1e-3) / 1e12,
                      "peak_fp32_mfma_tflops": 157.3}

    if not a.no_torch:
        tm = TorchNAIS(m).to(dev).train()
        topt = torch.optim.Adagrad(tm.parameters(), lr=0.01)
        loss_f = torch.nn.BCELoss()

        def torch_step(hist, data, labels):
            topt.zero_grad()
            loss = loss_f(tm(hist, data), labels)
            loss.backward()
            topt.step()
        out["torch_eager_ms_per_step"] = time_loop(torch_step, bs, a.warmup, a.steps) * 1e3
        out["speedup_vs_torch_eager"] = out["torch_eager_ms_per_step"] / out["hip_ms_per_step"]
        out["fused_speedup_vs_torch_eager"] = out["torch_eager_ms_per_step"] / out["fused_ms_per_step"]

    if a.cpu:
        sys.path.insert(0, ROOT)
        from oracle import train_oracle
        p = {k: v.detach().cpu().numpy() for k, v in m.named_parameters()}
        h, d, l = host[0]
        t0 = time.perf_counter()
        train_oracle.train_step_basic(p, h, d, l)
        out["cpu_oracle_s_per_step"] = time.perf_counter() - t0
        out["cpu_oracle_threads"] = torch.get_num_threads()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
