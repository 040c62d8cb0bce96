"""Adagrad on the device kernels (`nais_adagrad`, `nais_adagrad_rows`): a drop-in for the
`torch.optim.Adagrad(model.parameters(), lr=args.lr, weight_decay=args.lamda)` of run.py:89.

Same constructor, same per-parameter state ('step', 'sum') and the same update as torch's
Adagrad (torch/optim/adagrad.py, single-tensor form):
    g' = g + weight_decay * p ; sum += g' * g' ; p -= clr * g' / (sqrt(sum) + eps),
    clr = lr / (1 + (step - 1) * lr_decay).
Row update: with weight_decay == 0, a row of an embedding table whose gradient is zero is left
bit-identical by that update (sum += 0, p -= 0). NAIS_basic's training backward records which
rows of embed_history / embed_target it wrote (the batch's history and targets); for those
tables this optimizer updates only those rows (2 x (n + b) x d floats instead of 2 x P x d).
Parameters without such a record, or any parameter when weight_decay != 0, get the dense update.
"""
from __future__ import annotations

import torch
from torch.autograd.graph import increment_version

from . import _capi


class Adagrad(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-2, lr_decay=0, weight_decay=0, initial_accumulator_value=0,
                 eps=1e-10, row_update=True):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if lr_decay < 0.0:
            raise ValueError(f"Invalid lr_decay value: {lr_decay}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if initial_accumulator_value < 0.0:
            raise ValueError(f"Invalid initial_accumulator_value value: {initial_accumulator_value}")
        if eps < 0.0:
            raise ValueError(f"Invalid epsilon value: {eps}")
        defaults = dict(lr=lr, lr_decay=lr_decay, eps=eps, weight_decay=weight_decay,
                        initial_accumulator_value=initial_accumulator_value, row_update=row_update)
        super().__init__(params, defaults)
        for group in self.param_groups:
            for p in group["params"]:
                st = self.state[p]
                st["step"] = torch.tensor(0.0)
                st["sum"] = torch.full_like(p, group["initial_accumulator_value"],
                                            memory_format=torch.preserve_format)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _capi.load()
        for group in self.param_groups:
            for p in group["params"]:
                rows = getattr(p, "_nais_rows", None)
                if rows is not None:
                    p._nais_rows = None
                if p.grad is None:
                    continue
                if p.device.type != "cuda" or p.dtype != torch.float32 or not p.is_contiguous():
                    raise RuntimeError("optim.Adagrad: parameters must be contiguous float32 on the "
                                       "ROCm device")
                if p.grad.is_sparse:
                    raise RuntimeError("optim.Adagrad: sparse gradients are not supported")
                st = self.state[p]
                st["step"] += 1
                step = float(st["step"])
                clr = group["lr"] / (1 + (step - 1) * group["lr_decay"])
                g = p.grad.contiguous()
                s = st["sum"]
                stream = _capi.stream_handle(p.device)
                if isinstance(rows, list) and group["row_update"] and group["weight_decay"] == 0 and p.dim() == 2:
                    # sorted with repeats (the kernel skips an entry equal to its predecessor):
                    # torch.unique would size its output on the host, one sync per table per step
                    r = torch.sort(torch.cat([x.reshape(-1) for x in rows])).values
                    _capi.check(lib.nais_adagrad_rows(p.data_ptr(), s.data_ptr(), g.data_ptr(),
                                                      p.shape[1], r.data_ptr(), r.numel(), clr,
                                                      group["eps"], stream), "nais_adagrad_rows")
                else:
                    _capi.check(lib.nais_adagrad(p.data_ptr(), s.data_ptr(), g.data_ptr(), p.numel(),
                                                 clr, group["weight_decay"], group["eps"], stream),
                                "nais_adagrad")
                # the kernels write p through its raw pointer; bump its version counter as an
                # in-place torch op would, so version-keyed caches (model._score_params' padded
                # copies) see the update
                increment_version(p)
        return loss
