"""Per-phase cycle split of the training backward kernel (the timing build scripts/probes/train_timing.hip:
  python scripts/build_ab.py timing=nais_train.hip@scripts/probes/train_timing.hip).
  NAIS_HIP_LIB=build_ab/timing.so python scripts/train_phases.py [--D 64 --H 64 --n 204]
Phases (s_memtime deltas summed over waves): 0 prologue, 1 u recompute + exp, 2 du/db1/dw2 + LDS
writes, 3 dx MFMA + dt, 4 dh reduce-scatter, 5 barrier, 6 dW1 MFMA, 7 barrier, 8 flush.
--fused: the trainer's fused step (NAISTrainer.step, u cache on) instead of the forward + backward
entry points; at D or H > 64 that runs the general backward (gm_backward_kernel), whose phases are
0 W1 + unit staging, 1 u cache, 2 du/db1/dw2, 3 dx MFMA, 4 history/target row grads, 5 dW1
rounds, 6 dW1 atomics, 7 history-row atomics, 8 flush."""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poi_recommendation_models_amd import _capi  # noqa: E402
from poi_recommendation_models_amd.model import NAIS_basic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--P", type=int, default=100_000)
ap.add_argument("--D", type=int, default=64)
ap.add_argument("--H", type=int, default=64)
ap.add_argument("--n", type=int, default=204)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--dropout", type=float, default=0.5)
ap.add_argument("--fused", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
lib = _capi.load()
lib.nais_debug_train_cycles.restype = ctypes.c_int32
lib.nais_debug_train_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int32]
m = NAIS_basic(a.P, a.D, a.H, 0.5).to(dev)
g = torch.Generator().manual_seed(0)
hist = torch.randperm(a.P, generator=g)[:a.n].to(dev)
data = torch.randperm(a.P, generator=g)[:5 * a.n].to(dev)
b, n = data.numel(), a.n
prm = m.nais_params()
pred = torch.empty(b, device=dev)
saved = torch.empty(2 * b, device=dev)
gp = torch.randn(b, device=dev) * 1e-3
ws_bytes = lib.nais_train_workspace_size(prm, b, n)
ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
grads = [torch.zeros_like(p) for p in m.parameters()]
s = torch.cuda.current_stream(dev).cuda_stream
if a.fused:
    import numpy as np
    import scipy.sparse as sp
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from bench_train import batches
    from poi_recommendation_models_amd.trainer import NAISTrainer
    with torch.no_grad():
        m.embed_history.weight.normal_(0, 0.3)
        m.embed_target.weight.normal_(0, 0.3)
    m.train()
    m.drop.p = a.dropout
    m.report_nan = False
    host = batches(a.P, a.n, 4, 4, seed=1)
    bs = [(torch.as_tensor(h[0]).to(dev), torch.as_tensor(d).to(dev), torch.as_tensor(l).to(dev))
          for h, d, l in host]
    rows = np.repeat(np.arange(len(host)), a.n)
    cols = np.concatenate([np.sort(h[0]) for h, _, _ in host])
    tr = NAISTrainer(m, sp.csr_matrix((np.ones(len(cols)), (rows, cols)), shape=(len(host), a.P)), lr=0.01)
    for i in range(3):
        tr.step(*bs[i % len(bs)])
    buf = (ctypes.c_ulonglong * 16)()
    torch.cuda.synchronize()
    lib.nais_debug_train_cycles(buf, 1)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for i in range(a.iters):
        tr.step(*bs[i % len(bs)])
    ev[1].record()
    torch.cuda.synchronize()
    lib.nais_debug_train_cycles(buf, 0)
    tr.finish()
    tot = sum(buf[:9])
    names = ["staging", "ucache", "du", "dx", "row_grads", "dW1_rounds", "dW1_atomics", "hist_atomics", "flush"]
    print(json.dumps({"fused_ms_per_step": ev[0].elapsed_time(ev[1]) / a.iters,
                      "split": {nm: round(buf[i] / tot, 4) for i, nm in enumerate(names)},
                      "total_cycles_per_step": tot / a.iters}))
    sys.exit(0)
_capi.check(lib.nais_train_forward(prm, hist.data_ptr(), n, data.data_ptr(), b, a.dropout, 7, pred.data_ptr(),
                                   saved.data_ptr(), None, ws.data_ptr(), ws_bytes, s), "fwd")
buf = (ctypes.c_ulonglong * 16)()
torch.cuda.synchronize()
lib.nais_debug_train_cycles(buf, 1)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(a.iters):
    _capi.check(lib.nais_train_backward(prm, hist.data_ptr(), n, data.data_ptr(), b, a.dropout, 7,
                                        pred.data_ptr(), saved.data_ptr(), gp.data_ptr(),
                                        *[x.data_ptr() for x in grads], ws.data_ptr(), ws_bytes, s), "bwd")
ev[1].record()
torch.cuda.synchronize()
lib.nais_debug_train_cycles(buf, 0)
tot = sum(buf[:9])
names = ["prologue", "u+exp", "du+lds", "dx+dt", "dh_rs", "barrier1", "dW1", "barrier2", "flush"]
print(json.dumps({"backward_ms": ev[0].elapsed_time(ev[1]) / a.iters,
                  "split": {nm: round(buf[i] / tot, 4) for i, nm in enumerate(names)},
                  "total_cycles_per_launch": tot / a.iters}))
