"""Drop-in NAIS modules whose forward runs the gfx950 HIP kernels through the C-ABI.

Constructor signatures, sub-module names (hence state_dict keys), initialisation and forward
signatures follow the reference:

* `NAIS_basic(item_num, embed_size, hidden_size, beta)`                               model.py:8-97
* `NAIS_regionEmbedding(item_num, embed_size, hidden_size, beta, region_embed_size)`   model.py:99-187
* `NAIS_region_distance_Embedding(item_num, embed_size, hidden_size, beta,
                                  region_embed_size, dist_embed_size)`                model.py:189-304
* `NAIS_distance_Embedding(item_num, embed_size, hidden_size, beta,
                           region_embed_size, dist_embed_size)`                       model.py:306-408
* `NAIS_region_distance_disentangled_Embedding(item_num, embed_size, hidden_size, beta,
                                               region_embed_size, dist_embed_size)`   model.py:409-541
* `New4(item_num, embed_size, hidden_size, beta, region_embed_size)`                  model.py:1169-1306
  and the rest of its family with the same signature: `New4_padding` (:1308), `all_in_out`
  (:1447), `nearPOI_embedding` (:1578), `no_POI_emb` (:1707), `transform_ingoing_outgoing`
  (:1822), `transform_attn` (:1959, dot-product core), `only_area_not_inout` (:2100)

`forward` evaluates attention_network + sigmoid on the device in one fused kernel
(`nais_forward`); there is no CPU path: inputs must live on the ROCm device that holds the
parameters, otherwise a RuntimeError is raised. In eval mode Dropout is the identity (as under
`model.eval()` in every reference validation loop).

Training (run.py:91-109): `NAIS_basic.forward` in train mode runs
`nais_train_forward` (Dropout(p) on W1 x + b1, model.py:71) inside an autograd Function whose
backward is `nais_train_backward`, so the reference's loop -- forward, `loss_func`, `backward()`,
optimizer step -- runs unchanged. The batch must be get_NAIS_batch's shape (batches.py:24-50):
every row shares one history (checked; per-row histories raise). The region variants train on
the same autograd Function (`nais_train_forward_ex` / `nais_train_backward_ex`, region rows and
the distance layer included); NAIS_basic at embed_dim <= 64 / hidden <= 64 takes the fused MFMA
kernels, every other shape (run.py's default factor_num = hidden_dim = 128) a general kernel.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import _capi


class BCELoss(nn.BCELoss):
    """nn.BCELoss (model.py:21) that raises like the reference's CPU BCELoss ("all elements of
    input should be between 0 and 1") when a prediction is NaN or outside [0, 1] -- e.g. the NaN
    row of a single-item history equal to its target (model.py:92-95) -- instead of reaching the
    ROCm kernel's device-side assert, which aborts the process. The check costs one device->host
    sync; `check_input = False` skips it when the caller guarantees finite predictions."""

    check_input = True

    def forward(self, input, target):
        if self.check_input and input.is_cuda and \
                bool(((input < 0) | (input > 1) | torch.isnan(input)).any()):
            raise RuntimeError("all elements of input should be between 0 and 1")
        return super().forward(input, target)


# embedding widths the scoring kernels are compiled for (MFMA K tiles); others are zero-padded
NATIVE_WIDTHS = (8, 16, 32, 64, 128)


class _NAISDevice(nn.Module):
    """Shared plumbing: parameter struct for the C-ABI, device checks, NaN reporting."""

    VARIANT = _capi.VARIANT_BASIC
    report_nan = True  # model.py:50-54 prints the NaN count of every forward
    # arithmetic of the catalog scorer's W1 x products (include/nais.h NAIS_PRECISION_*):
    #   "fp16x6" (default) fp32-faithful split-fp16 MFMA: hi/mid/lo pieces represent every fp32
    #            operand exactly, 6 products per fp32 product (dropped terms <= ~2^-33 relative,
    #            below fp32's own product rounding), fp32 accumulation;
    #   "fp32"   exact fp32 MFMA (a k-ordered fmaf chain);
    #   "fp16x3" 2 pieces / 3 products (~2^-21 relative per product: narrower than fp32, kept for
    #            A/B); "*_pairsplit" split x = h (.) t per pair instead of A_j = W1 diag(h_j).
    # nais_forward (the general model.forward path) is always fp32.
    precision = "fp16x6"
    # full-catalog strategy of catalog.score_topk / the validation drop-ins: "auto" (pair tables
    # when the users' history entries outnumber their distinct POIs 3:1, else per user),
    # "direct" or "pairs" (include/nais.h)
    catalog_strategy = "auto"

    def _check_device(self, *tensors):
        dev = self.attn_layer1.weight.device
        if dev.type != "cuda":
            raise RuntimeError(f"{type(self).__name__}: the NAIS path runs only on a ROCm device "
                               f"(parameters are on {dev}); move the model with .to('cuda')")
        for t in tensors:
            if t is not None and t.device != dev:
                raise RuntimeError(f"{type(self).__name__}: input on {t.device}, parameters on {dev}")
        for n, p in self.named_parameters():
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise RuntimeError(f"{type(self).__name__}: parameter {n} must be contiguous float32")
        return dev

    def _item_tables(self):
        """(embed_history, embed_target) tables the kernels index by POI id."""
        return self.embed_history.weight, self.embed_target.weight

    # catalog hooks of the pairs strategy (catalog._score_topk_pairs): the (item, candidate) table
    # builder, a post-gather pass over the score rows, and whether the direct kernels apply
    _pairs_only = False

    def _pair_table(self, lib, prm, items, J, c0, w, reg, cor, llm, e, es, ld, stream, work=None):
        _capi.check(lib.nais_pair_table(prm, items.data_ptr(), J, c0, w, _capi.ptr(reg), _capi.ptr(cor),
                                        _capi.ptr(llm), e, es, ld, work, stream), "nais_pair_table")

    def _pair_fixup(self, csr, users, m, scores, c0, c1, stream):
        pass

    def nais_params(self) -> _capi.NaisParams:
        """`nais_params_t` view of this module's parameters (device pointers, no copies)."""
        eh, et = self._item_tables()
        p = _capi.NaisParams()
        p.variant = self.VARIANT
        p.embed_dim = self.embed_size
        p.item_dim = eh.shape[1]
        p.region_dim = self.embed_region.weight.shape[1] if hasattr(self, "embed_region") else 0
        p.hidden = self.attn_layer1.weight.shape[0]
        p.din = self.attn_layer1.weight.shape[1]
        p.num_pois = eh.shape[0]
        p.num_regions = self.embed_region.weight.shape[0] if hasattr(self, "embed_region") else 0
        p.beta = float(self.beta)
        p.precision = {"fp32": _capi.PRECISION_FP32, "fp16x3": _capi.PRECISION_FP16X3,
                       "fp16x3_pairsplit": _capi.PRECISION_FP16X3_PAIRSPLIT,
                       "fp16x6": _capi.PRECISION_FP16X6,
                       "fp16x6_pairsplit": _capi.PRECISION_FP16X6_PAIRSPLIT}[self.precision]
        p.embed_history = eh.data_ptr()
        p.embed_target = et.data_ptr()
        p.embed_region = self.embed_region.weight.data_ptr() if hasattr(self, "embed_region") else None
        p.w1 = self.attn_layer1.weight.data_ptr()
        p.b1 = self.attn_layer1.bias.data_ptr()
        p.w2 = self.attn_layer2.weight.data_ptr()
        if hasattr(self, "dist_layer"):
            p.dist_w = self.dist_layer.weight.data_ptr()
            p.dist_b = self.dist_layer.bias.data_ptr()
        return p

    def _score_params(self) -> _capi.NaisParams:
        """`nais_params_t` for the scoring / forward kernels. Those are compiled for the embedding
        widths D in NATIVE_WIDTHS (the MFMA K tiles); any other D <= 128 (the reference builds
        Linear(embed_size, hidden_size) for any size, model.py:9-38) is served from zero-padded
        copies: the tables padded to the next native width (each half separately for the region
        variants' [E | region] rows), attn_layer1's columns placed at the padded positions, the
        distance columns after them. Exact: a padded dimension contributes 0 * x = 0 to W1 x and
        to h . t, and the per-wave power-of-two scales see the same maxima. The copies are rebuilt
        when a parameter changes (tensor version counter). Training reads the parameters as they
        are (the training kernels take any D, H <= 128)."""
        D = int(self.embed_size)
        if D in NATIVE_WIDTHS or D > NATIVE_WIDTHS[-1]:
            # above 128 the library's generic-shape kernels (nais_generic.hip, exact fp32) take the
            # parameters as they are, up to embed_size 256 (NAIS_E_UNSUPPORTED beyond)
            return self.nais_params()
        Dp = next(w for w in NATIVE_WIDTHS if w >= D)
        region = self.VARIANT in (_capi.VARIANT_REGION, _capi.VARIANT_REGION_DISTANCE)
        dist = self.VARIANT in (_capi.VARIANT_REGION_DISTANCE, _capi.VARIANT_DISTANCE)
        eh, et = self._item_tables()
        er = self.embed_region.weight if region else None
        w1 = self.attn_layer1.weight
        srcs = [t for t in (eh, et, er, w1) if t is not None]
        key = tuple((t.data_ptr(), t._version) for t in srcs)
        cache = self.__dict__.get("_pad_cache")
        if cache is None or cache[0] != key:
            with torch.no_grad():
                H = w1.shape[0]
                w1p = torch.zeros(H, Dp + (2 if dist else 0), dtype=w1.dtype, device=w1.device)
                if region:
                    if eh.shape[1] * 2 != D:
                        raise ValueError(f"region variants need an even embed_size (got {D}): the "
                                         "[history | region] rows are 2 * int(embed_size / 2) wide")
                    half, hp = D // 2, Dp // 2
                    pad = lambda t: torch.nn.functional.pad(t, (0, hp - half)).contiguous()
                    tabs = (pad(eh), pad(et), pad(er))
                    w1p[:, :half] = w1[:, :half]
                    w1p[:, hp:hp + half] = w1[:, half:D]
                else:
                    pad = lambda t: torch.nn.functional.pad(t, (0, Dp - D)).contiguous()
                    tabs = (pad(eh), pad(et), None)
                    w1p[:, :D] = w1[:, :D]
                if dist:
                    w1p[:, Dp:Dp + 2] = w1[:, D:D + 2]
            cache = (key, tabs, w1p)
            self.__dict__["_pad_cache"] = cache
        _, (ehp, etp, erp), w1p = cache
        p = self.nais_params()
        p.embed_dim = Dp
        p.item_dim = ehp.shape[1]
        p.din = w1p.shape[1]
        p.embed_history, p.embed_target, p.w1 = ehp.data_ptr(), etp.data_ptr(), w1p.data_ptr()
        if region:
            p.region_dim = erp.shape[1]
            p.embed_region = erp.data_ptr()
        return p

    def _run_forward(self, history, target, history_region=None, target_region=None,
                     target_lat_long=None, sigmoid=True):
        if self.training:
            if not sigmoid:
                raise NotImplementedError(
                    f"{type(self).__name__}: training-mode attention_network is not implemented; the "
                    "training path is the forward (SURVEY.md 8(f1)); call model.eval()")
            return self._train_forward(history, target, history_region, target_region, target_lat_long)
        dev = self._check_device(history, target, history_region, target_region, target_lat_long)
        if history.dim() != 2 or target.dim() != 1 or history.shape[0] != target.shape[0]:
            raise ValueError(f"history must be [b, n] and target [b]; got {tuple(history.shape)}, "
                             f"{tuple(target.shape)}")

        def idx(t):
            t = t.to(torch.int64)
            return t if t.dim() < 2 or t.stride(1) == 1 else t.contiguous()

        history, target = idx(history), idx(target).contiguous()
        b, n = history.shape
        ll, ll_ld = None, 0
        if self.VARIANT in (_capi.VARIANT_REGION, _capi.VARIANT_REGION_DISTANCE):
            if history_region is None or target_region is None:
                raise ValueError("region variants need history_region and target_region")
            history_region = idx(history_region)
            target_region = idx(target_region).contiguous()
            if tuple(history_region.shape) != (b, n) or tuple(target_region.shape) != (b,):
                raise ValueError("history_region must be [b, n] and target_region [b]")
        else:
            history_region = target_region = None
        if self.VARIANT in (_capi.VARIANT_REGION_DISTANCE, _capi.VARIANT_DISTANCE):
            if target_lat_long is None or tuple(target_lat_long.shape) != (b, n, 2):
                raise ValueError("target_lat_long must be [b, n, 2]")
            ll = target_lat_long.to(torch.float32)
            if not (ll.stride(2) == 1 and ll.stride(1) == 2):
                ll = ll.contiguous()
            ll_ld = ll.stride(0)
        out = torch.empty(b, dtype=torch.float32, device=dev)
        nan = torch.zeros(1, dtype=torch.int32, device=dev)
        lib = _capi.load()
        prm = self._score_params()
        rc = lib.nais_forward(prm, _capi.ptr(history) if n > 0 else None, b, n,
                              history.stride(0) if n > 0 else 0, _capi.ptr(target),
                              _capi.ptr(history_region) if (history_region is not None and n > 0) else None,
                              history_region.stride(0) if (history_region is not None and n > 0) else 0,
                              _capi.ptr(target_region), _capi.ptr(ll) if n > 0 else None, ll_ld,
                              out.data_ptr(), nan.data_ptr(),
                              _capi.FLAG_SIGMOID if sigmoid else 0, _capi.stream_handle(dev))
        _capi.check(rc, "nais_forward")
        self._last_nan = nan
        if self.report_nan and isinstance(self, NAIS_basic):
            c = int(nan.item())           # model.py:52 (.item() host sync, as in the reference)
            if c > 0:
                print(c)
        return out

    # check that every row of a training batch carries the same history (batches.py:30); set to
    # False to skip the check (one device->host sync per step) when the caller guarantees it
    check_shared_history = True

    def _train_param_names(self):
        """nais_train_grads_t fields of the parameters the training forward reads."""
        names = ["embed_history", "embed_target"]
        if self.VARIANT in (_capi.VARIANT_REGION, _capi.VARIANT_REGION_DISTANCE):
            names.append("embed_region")
        names += ["w1", "b1", "w2"]
        if self.VARIANT in (_capi.VARIANT_REGION_DISTANCE, _capi.VARIANT_DISTANCE):
            names += ["dist_w", "dist_b"]
        return names

    def _train_params(self):
        t = {"embed_history": self.embed_history.weight, "embed_target": self.embed_target.weight,
             "w1": self.attn_layer1.weight, "b1": self.attn_layer1.bias, "w2": self.attn_layer2.weight}
        if hasattr(self, "embed_region"):
            t["embed_region"] = self.embed_region.weight
        if hasattr(self, "dist_layer"):
            t["dist_w"], t["dist_b"] = self.dist_layer.weight, self.dist_layer.bias
        return [t[k] for k in self._train_param_names()]

    def _train_forward(self, history, target, history_region=None, target_region=None,
                       target_lat_long=None):
        dev = self._check_device(history, target, history_region, target_region, target_lat_long)
        if history.dim() != 2 or target.dim() != 1 or history.shape[0] != target.shape[0]:
            raise ValueError(f"history must be [b, n] and target [b]; got {tuple(history.shape)}, "
                             f"{tuple(target.shape)}")
        history = history.to(torch.int64)
        target = target.to(torch.int64).contiguous()
        b, n = history.shape
        if self.check_shared_history and b > 1 and n > 0 and \
                not bool((history == history[:1]).all()):
            raise NotImplementedError(
                f"{type(self).__name__}: the training step needs rows that share one history "
                "(get_NAIS_batch, batches.py:24-50); per-row histories are not supported")
        hist = history[0].contiguous() if b > 0 else history.new_empty(0)
        side = None
        if self.VARIANT in (_capi.VARIANT_REGION, _capi.VARIANT_REGION_DISTANCE):
            if history_region is None or target_region is None:
                raise ValueError("region variants need history_region and target_region")
            history_region = history_region.to(torch.int64)
            if tuple(history_region.shape) != (b, n) or tuple(target_region.shape) != (b,):
                raise ValueError("history_region must be [b, n] and target_region [b]")
            if self.check_shared_history and b > 1 and n > 0 and \
                    not bool((history_region == history_region[:1]).all()):
                raise NotImplementedError(f"{type(self).__name__}: history_region rows must be shared")
            ll = None
            if self.VARIANT == _capi.VARIANT_REGION_DISTANCE:
                if target_lat_long is None or tuple(target_lat_long.shape) != (b, n, 2):
                    raise ValueError("target_lat_long must be [b, n, 2]")
                ll = target_lat_long.to(torch.float32)
                if not (ll.stride(2) == 1 and ll.stride(1) == 2):
                    ll = ll.contiguous()
            hreg = history_region[0].contiguous() if b > 0 else history_region.new_empty(0)
            side = (hreg, target_region.to(torch.int64).contiguous(), ll)
        elif self.VARIANT == _capi.VARIANT_DISTANCE:
            if target_lat_long is None or tuple(target_lat_long.shape) != (b, n, 2):
                raise ValueError("target_lat_long must be [b, n, 2]")
            ll = target_lat_long.to(torch.float32)
            if not (ll.stride(2) == 1 and ll.stride(1) == 2):
                ll = ll.contiguous()
            side = (None, None, ll)
        drop = getattr(self, "drop", None)        # none in the two distance variants (model.py:268, 369)
        p = float(drop.p) if drop is not None and drop.training else 0.0
        seed = int(torch.randint(0, 2**62, (1,)).item())   # torch's CPU generator: manual_seed applies
        pred, nan = _NAISTrainStep.apply(self, hist, target, p, seed, side, *self._train_params())
        self._last_nan = nan
        if self.report_nan and isinstance(self, NAIS_basic):
            c = int(nan.item())                              # model.py:50-54 (NAIS_basic only)
            if c > 0:
                print(c)
        return pred

    def get_mask(self, user_history, target_item):            # model.py:92-95
        target_item = target_item.reshape([len(target_item), 1])
        return user_history != target_item

    def loss_function(self, prediction, label):              # model.py:96-97
        return self.loss_func(prediction, label)


class _NAISTrainStep(torch.autograd.Function):
    """pred = sigmoid(attention_network(...)) of a shared-history batch with dropout; backward
    through nais_train_backward_ex (gradients of every parameter the variant's forward reads:
    the module's `_train_params()`)."""

    @staticmethod
    def forward(ctx, module, hist, target, p, seed, side, *weights):
        dev = weights[0].device
        b, n = target.shape[0], hist.shape[0]
        lib = _capi.load()
        prm = module.nais_params()
        # the general kernels' u cache (D or H beyond the fused kernels' shapes): the forward leaves
        # each pair's u / s / logit for this Function's backward instead of it recomputing them
        ub = lib.nais_train_ucache_size(prm, b, n)
        ucache = torch.empty(ub, dtype=torch.uint8, device=dev) if ub else None
        sd = _train_side(side, ucache)
        pred = torch.empty(b, dtype=torch.float32, device=dev)
        saved = torch.empty(2 * max(b, 1), dtype=torch.float32, device=dev)
        nan = torch.zeros(1, dtype=torch.int32, device=dev)
        ws_bytes = lib.nais_train_workspace_size(prm, b, n)
        ws = torch.empty(max(ws_bytes, 4), dtype=torch.uint8, device=dev)
        _capi.check(lib.nais_train_forward_ex(prm, sd, _capi.ptr(hist) if n else None, n,
                                              _capi.ptr(target) if b else None, b, p, seed,
                                              pred.data_ptr(), saved.data_ptr(), nan.data_ptr(),
                                              ws.data_ptr(), ws_bytes, _capi.stream_handle(dev)),
                    "nais_train_forward_ex")
        ctx.module, ctx.p, ctx.seed, ctx.side, ctx.ucache = module, p, seed, side, ucache
        ctx.save_for_backward(hist, target, pred, saved)
        ctx.mark_non_differentiable(nan)
        return pred, nan

    @staticmethod
    def backward(ctx, gpred, _gnan):
        hist, target, pred, saved = ctx.saved_tensors
        m = ctx.module
        names = m._train_param_names()
        params = m._train_params()
        g = [torch.zeros_like(t) for t in params]
        grads = _capi.NaisTrainGrads()
        for name, t in zip(names, g):
            setattr(grads, name, t.data_ptr())
        b, n = target.shape[0], hist.shape[0]
        dev = params[0].device
        gpred = gpred.to(torch.float32).contiguous()
        lib = _capi.load()
        prm = m.nais_params()
        ws_bytes = lib.nais_train_workspace_size(prm, b, n)
        ws = torch.empty(max(ws_bytes, 4), dtype=torch.uint8, device=dev)
        _capi.check(lib.nais_train_backward_ex(prm, _train_side(ctx.side, ctx.ucache),
                                               _capi.ptr(hist) if n else None,
                                               n, _capi.ptr(target) if b else None, b, ctx.p, ctx.seed,
                                               pred.data_ptr(), saved.data_ptr(), gpred.data_ptr(),
                                               grads, ws.data_ptr(), ws_bytes, _capi.stream_handle(dev)),
                    "nais_train_backward_ex")
        # rows of the embedding tables this step can have touched (for optim.Adagrad's row update)
        _note_rows(m.embed_history.weight, hist)
        _note_rows(m.embed_target.weight, target)
        if "embed_region" in names:
            _note_rows(m.embed_region.weight, torch.cat([ctx.side[0], ctx.side[1]]))
        return (None, None, None, None, None, None, *g)


def _train_side(side, ucache=None):
    sd = _capi.NaisTrainSide()
    if side is not None:
        hreg, treg, ll = side
        sd.hist_region, sd.target_region = _capi.ptr(hreg), _capi.ptr(treg)
        if ll is not None:
            sd.target_lat_long, sd.latlon_ld = ll.data_ptr(), ll.stride(0)
    if ucache is not None:
        sd.ucache, sd.ucache_bytes = ucache.data_ptr(), ucache.numel()
    return sd


def _note_rows(param, rows):
    """Record rows whose gradient this backward wrote; consumed (reset) by optim.Adagrad.step.
    Without such a consumer (e.g. torch.optim.Adagrad) the record degrades to "dense" after a few
    backward calls instead of growing."""
    lst = getattr(param, "_nais_rows", None)
    if isinstance(lst, str):
        return
    if lst is None:
        lst = []
        param._nais_rows = lst
    if len(lst) >= 16:
        param._nais_rows = "dense"
        return
    lst.append(rows)


class NAIS_basic(_NAISDevice):
    VARIANT = _capi.VARIANT_BASIC

    def __init__(self, item_num, embed_size, hidden_size, beta):
        super().__init__()
        self.embed_size = embed_size
        self.item_num = item_num
        self.beta = beta
        self.hidden_size = hidden_size
        self.embed_history = nn.Embedding(item_num, self.embed_size)
        self.embed_target = nn.Embedding(item_num, self.embed_size)
        self.relu = nn.ReLU()
        self.sigmoid = nn.Sigmoid()
        self.loss_func = BCELoss()
        self.drop = nn.Dropout()
        self.attn_layer1 = nn.Linear(self.embed_size, self.hidden_size)
        self.attn_layer2 = nn.Linear(self.hidden_size, 1, bias=False)
        self._init_weight_()

    def _init_weight_(self):                                  # model.py:30-38
        nn.init.normal_(self.embed_history.weight, std=0.01)
        nn.init.normal_(self.embed_target.weight, std=0.01)
        for m in self.modules():
            if isinstance(m, nn.Linear) and m.bias is not None:
                m.bias.data.zero_()

    def forward(self, history, target):                       # model.py:40-55
        return self._run_forward(history, target)

    def attention_network(self, user_history, target_item):   # model.py:57-89 (logits)
        return self._run_forward(user_history, target_item, sigmoid=False)


class NAIS_regionEmbedding(_NAISDevice):
    VARIANT = _capi.VARIANT_REGION

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size):
        super().__init__()
        self.embed_size = embed_size
        self.item_num = item_num
        self.beta = beta
        self.hidden_size = hidden_size
        self.embed_history = nn.Embedding(item_num, int(embed_size / 2))
        self.embed_target = nn.Embedding(item_num, int(embed_size / 2))
        self.embed_region = nn.Embedding(region_embed_size, int(embed_size / 2))
        self.relu = nn.ReLU()
        self.sigmoid = nn.Sigmoid()
        self.loss_func = BCELoss()
        self.attn_layer1 = nn.Linear(embed_size, hidden_size)
        self.attn_layer2 = nn.Linear(hidden_size, 1, bias=False)
        self.drop = nn.Dropout()
        self._init_weight_()

    def _init_weight_(self):                                  # model.py:121-130
        nn.init.normal_(self.embed_history.weight, std=0.01)
        nn.init.normal_(self.embed_target.weight, std=0.01)
        nn.init.normal_(self.embed_region.weight, std=0.01)
        for m in self.modules():
            if isinstance(m, nn.Linear) and m.bias is not None:
                m.bias.data.zero_()

    def forward(self, history, target, history_region, target_region):   # model.py:132-142
        return self._run_forward(history, target, history_region, target_region)

    def attention_network(self, user_history, target_item, history_region, target_region):
        return self._run_forward(user_history, target_item, history_region, target_region,
                                 sigmoid=False)


class NAIS_region_distance_Embedding(_NAISDevice):
    VARIANT = _capi.VARIANT_REGION_DISTANCE

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size, dist_embed_size):
        super().__init__()
        self.DEVICE = torch.device('cuda' if torch.cuda.is_available() else 'cpu')
        self.embed_size = embed_size
        self.item_num = item_num
        self.beta = beta
        self.hidden_size = hidden_size
        self.embed_history = nn.Embedding(item_num, int(embed_size / 2))
        self.embed_target = nn.Embedding(item_num, int(embed_size / 2))
        self.embed_region = nn.Embedding(region_embed_size, int(embed_size / 2))
        self.embed_distance = nn.Embedding(dist_embed_size, embed_size)   # unused, as in model.py:204
        self.relu = nn.ReLU()
        self.tanh = nn.Tanh()
        self.sigmoid = nn.Sigmoid()
        self.loss_func = BCELoss()
        self.attn_layer1 = nn.Linear(embed_size + 2, hidden_size)
        self.attn_layer2 = nn.Linear(hidden_size, 1, bias=False)
        self.dist_layer = nn.Linear(2, 2)
        self._init_weight_()

    def _init_weight_(self):                                  # model.py:219-229
        nn.init.normal_(self.embed_history.weight, std=0.01)
        nn.init.normal_(self.embed_target.weight, std=0.01)
        nn.init.normal_(self.embed_region.weight, std=0.01)
        nn.init.normal_(self.embed_distance.weight, std=0.01)
        for m in self.modules():
            if isinstance(m, nn.Linear) and m.bias is not None:
                m.bias.data.zero_()

    def forward(self, history, target, history_region, target_region, target_lat_long):  # :231-244
        return self._run_forward(history, target, history_region, target_region, target_lat_long)

    def attention_network(self, user_history, target_item, history_region, target_region,
                          target_lat_long_tensor):
        return self._run_forward(user_history, target_item, history_region, target_region,
                                 target_lat_long_tensor, sigmoid=False)


class NAIS_distance_Embedding(_NAISDevice):
    """NAIS_basic + the distance feature sigmoid(dist_layer(1000 * (|dlat|, |dlng|))) appended to
    h (.) t (model.py:306-408); the regions of forward() are accepted and ignored, as in the
    reference. Validated by NAIS_region_distance_validation (run.py:431)."""
    VARIANT = _capi.VARIANT_DISTANCE

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size, dist_embed_size):
        super().__init__()
        self.DEVICE = torch.device('cuda' if torch.cuda.is_available() else 'cpu')
        self.embed_size = embed_size
        self.item_num = item_num
        self.beta = beta
        self.hidden_size = hidden_size
        self.embed_history = nn.Embedding(item_num, embed_size)
        self.embed_target = nn.Embedding(item_num, embed_size)
        self.relu = nn.ReLU()
        self.sigmoid = nn.Sigmoid()
        self.loss_func = BCELoss()
        self.attn_layer1 = nn.Linear(embed_size + 2, hidden_size)
        self.attn_layer2 = nn.Linear(hidden_size, 1, bias=False)
        self.dist_layer = nn.Linear(2, 2)
        self._init_weight_()

    def _init_weight_(self):                                  # model.py:329-337
        nn.init.normal_(self.embed_history.weight, std=0.01)
        nn.init.normal_(self.embed_target.weight, std=0.01)
        for m in self.modules():
            if isinstance(m, nn.Linear) and m.bias is not None:
                m.bias.data.zero_()

    def forward(self, history, target, history_region, target_region, target_distance):  # :339-353
        return self._run_forward(history, target, target_lat_long=target_distance)

    def attention_network(self, user_history, target_item, target_lat_long_tensor):     # :355-395
        return self._run_forward(user_history, target_item, target_lat_long=target_lat_long_tensor,
                                 sigmoid=False)


class NAIS_region_distance_disentangled_Embedding(_NAISDevice):
    """NAIS_region_distance_disentangled_Embedding (model.py:409-541): an item attention MLP and a
    region attention MLP (region rows embed_size wide), both shifted by a learned multiple of the
    target-history distance, normalised separately and summed (`nais_disent_forward`).
    forward(history, target, history_region, target_region, target_distance) with
    target_distance [b, n] f32 as run.py:326-333 builds it (`pair_distances` does that on the
    device). Eval arithmetic; the model has no dropout. The reference's evaluation call for it
    (run.py:353) does not match NAIS_region_distance_validation, so there is no catalog path."""

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size, dist_embed_size):
        super().__init__()
        self.embed_size = embed_size
        self.item_num = item_num
        self.beta = beta
        self.hidden_size = hidden_size
        self.embed_history = nn.Embedding(item_num, embed_size)
        self.embed_target = nn.Embedding(item_num, embed_size)
        self.embed_region = nn.Embedding(region_embed_size, embed_size)
        self.embed_distance = nn.Embedding(dist_embed_size, embed_size)
        self.relu = nn.ReLU()
        self.sigmoid = nn.Sigmoid()
        self.loss_func = BCELoss()
        self.attn_layer1 = nn.Linear(embed_size, hidden_size)
        self.attn_layer2 = nn.Linear(hidden_size, 1, bias=False)
        self.region_attn_layer1 = nn.Linear(embed_size, hidden_size)
        self.region_attn_layer2 = nn.Linear(hidden_size, 1, bias=False)
        self._init_weight_()

    def _init_weight_(self):                                  # model.py:436-444
        for e in (self.embed_history, self.embed_target, self.embed_region, self.embed_distance):
            nn.init.normal_(e.weight, std=0.01)
        for m in self.modules():
            if isinstance(m, nn.Linear) and m.bias is not None:
                m.bias.data.zero_()

    def disent_params(self):
        p = _capi.NaisDisentParams()
        p.embed_dim, p.hidden = self.embed_size, self.attn_layer1.weight.shape[0]
        p.num_pois, p.num_regions = self.embed_history.weight.shape[0], self.embed_region.weight.shape[0]
        p.beta = float(self.beta)
        for name, t in (("embed_history", self.embed_history.weight), ("embed_target", self.embed_target.weight),
                        ("embed_region", self.embed_region.weight), ("embed_distance", self.embed_distance.weight),
                        ("w1", self.attn_layer1.weight), ("b1", self.attn_layer1.bias),
                        ("w2", self.attn_layer2.weight), ("region_w1", self.region_attn_layer1.weight),
                        ("region_b1", self.region_attn_layer1.bias), ("region_w2", self.region_attn_layer2.weight)):
            setattr(p, name, t.data_ptr())
        return p

    def forward(self, history, target, history_region, target_region, target_distance):   # :446-455
        if self.training:
            raise NotImplementedError(f"{type(self).__name__}: training mode is not implemented on the "
                                      "HIP path; call model.eval()")
        dev = self._check_device(history, target, history_region, target_region, target_distance)
        if history.dim() != 2 or target.dim() != 1 or history.shape[0] != target.shape[0]:
            raise ValueError(f"history must be [b, n] and target [b]; got {tuple(history.shape)}, "
                             f"{tuple(target.shape)}")
        b, n = history.shape
        if tuple(history_region.shape) != (b, n) or tuple(target_region.shape) != (b,) or \
                tuple(target_distance.shape) != (b, n):
            raise ValueError("history_region and target_distance must be [b, n], target_region [b]")

        def rows(t, dtype):
            t = t.to(dtype)
            return t if n == 0 or t.stride(1) == 1 else t.contiguous()
        history, history_region = rows(history, torch.int64), rows(history_region, torch.int64)
        td = rows(target_distance, torch.float32)
        target = target.to(torch.int64).contiguous()
        target_region = target_region.to(torch.int64).contiguous()
        out = torch.empty(b, dtype=torch.float32, device=dev)
        nan = torch.zeros(1, dtype=torch.int32, device=dev)
        _capi.check(_capi.load().nais_disent_forward(
            self.disent_params(), _capi.ptr(history) if n else None, b, n, history.stride(0) if n else 0,
            _capi.ptr(target), _capi.ptr(history_region) if n else None, history_region.stride(0) if n else 0,
            _capi.ptr(target_region), _capi.ptr(td) if n else None, td.stride(0) if n else 0,
            out.data_ptr(), nan.data_ptr(), _capi.FLAG_SIGMOID, _capi.stream_handle(dev)),
            "nais_disent_forward")
        self._last_nan = nan
        return out


def pair_distances(coords, hist, target):
    """run.py:326-333 on the device: f32 [b, n] powerLaw.dist (km) between every target and
    history POI (`nais_pair_distances`). coords: float64 [P, 2] device tensor; hist [n], target [b]."""
    hist = hist.to(torch.int64).contiguous()
    target = target.to(torch.int64).contiguous()
    if coords.dtype != torch.float64 or coords.dim() != 2 or coords.shape[1] != 2 or coords.device.type != "cuda":
        raise ValueError("coords must be a float64 [P, 2] ROCm tensor")
    out = torch.empty(target.numel(), hist.numel(), dtype=torch.float32, device=coords.device)
    _capi.check(_capi.load().nais_pair_distances(coords.contiguous().data_ptr(), _capi.ptr(hist), hist.numel(),
                                                 _capi.ptr(target), target.numel(), out.data_ptr(),
                                                 _capi.stream_handle(coords.device)), "nais_pair_distances")
    return out


def _as_near(near_pois, dev, P):
    near = torch.as_tensor(np.asarray(near_pois) if not torch.is_tensor(near_pois) else near_pois,
                           dtype=torch.int64).to(dev).contiguous()
    if near.dim() != 2 or near.shape[0] != P or near.shape[1] < 1:
        raise ValueError(f"near_pois must be [{P}, K]")
    return near


class _NearPOIModel(_NAISDevice):
    """Device path of the table-based New4 family (model.py:1169-2228): each
    forward(history, target, near_pois, target_region) pools every POI's near-POI list
    (`nais_near_attention`), lays the pools and embedding columns out as two [P, embed_size] row
    tables (`nais_copy_columns`) and runs NAIS_basic's attention over them with the basic kernels
    (fused forward, full-catalog scorer, pair tables). The tables are cached per near_pois array
    and parameter version. Eval only; sub-modules the forward never reads (embed_region,
    query/key/value where unused, drop) are kept for state_dict parity.

    Subclasses give `_layout()`: (pools, history columns, target columns), where a pool is
    (name, query table, key/value table, width, scale_dim, (wq, bq, wk, bk, wv, bv) or None) and a
    column is a pool name or an embedding weight."""
    VARIANT = _capi.VARIANT_BASIC
    _ext = None

    def _layout(self):
        raise NotImplementedError

    def _emb(self, *names_and_dims):
        for name, d in names_and_dims:
            setattr(self, name, nn.Embedding(self.item_num, int(d)))

    def _common(self, item_num, embed_size, hidden_size, beta, proj_dim):
        self.embed_size = embed_size
        self.item_num = item_num
        self.beta = beta
        self.hidden_size = hidden_size
        self.relu = nn.ReLU()
        self.sigmoid = nn.Sigmoid()
        self.loss_func = BCELoss()
        self.softmax = nn.Softmax(dim=-1)
        self.attn_layer1 = nn.Linear(embed_size, hidden_size)
        self.attn_layer2 = nn.Linear(hidden_size, 1, bias=False)
        self.query = nn.Linear(int(proj_dim), int(proj_dim))
        self.key = nn.Linear(int(proj_dim), int(proj_dim))
        self.value = nn.Linear(int(proj_dim), int(proj_dim))
        self.drop = nn.Dropout()

    def _init_weight_(self):                                  # e.g. model.py:1197-1209
        for name, m in self.named_children():
            if isinstance(m, nn.Embedding):
                nn.init.normal_(m.weight, std=0.01)
                if m.padding_idx is not None:
                    with torch.no_grad():
                        m.weight[m.padding_idx].fill_(0)
        for m in self.modules():
            if isinstance(m, nn.Linear) and m.bias is not None:
                m.bias.data.zero_()

    def _build_tables(self, near, xh, xt):
        lib, st = _capi.load(), _capi.stream_handle(near.device)
        P, D, K = self.item_num, self.embed_size, near.shape[1]
        pools, hcols, tcols = self._layout()
        done = {}
        for name, qt, kvt, d, sd, lin in pools:
            out = torch.empty(P, d, device=near.device)
            ptrs = [None] * 6 if lin is None else [t.data_ptr() for t in lin]
            _capi.check(lib.nais_near_attention(qt.data_ptr(), kvt.data_ptr(), P, d, near.data_ptr(), K,
                                                *ptrs, float(sd), out.data_ptr(), d, st),
                        "nais_near_attention")
            done[name] = out
        for dst, cols in ((xh, hcols), (xt, tcols)):
            c0 = 0
            for c in cols:
                src = done[c] if isinstance(c, str) else c
                _capi.check(lib.nais_copy_columns(src.data_ptr(), src.shape[1], P, src.shape[1],
                                                  dst.data_ptr(), D, c0, st), "nais_copy_columns")
                c0 += src.shape[1]
            if c0 != D:
                raise AssertionError(f"{type(self).__name__}: row layout width {c0} != {D}")
        return done

    def extended_tables(self, near_pois):
        """([P, D] history rows, [P, D] target rows) for this near-POI array (cached)."""
        dev = self._check_device()
        P, D = self.item_num, self.embed_size
        near = _as_near(near_pois, dev, P)
        ws = [p for p in self.parameters()]
        key = (near.data_ptr(), tuple(near.shape), tuple((w.data_ptr(), w._version) for w in ws))
        if self._ext is not None and self._ext[0] == key:
            return self._ext[1]
        xh = torch.empty(P, D, device=dev)
        xt = torch.empty(P, D, device=dev)
        self._build_tables(near, xh, xt)
        self._ext = (key, (xh, xt), near)
        return xh, xt

    def _item_tables(self):
        if self._ext is None:
            raise RuntimeError(f"{type(self).__name__}: call extended_tables(near_pois) (or forward) first")
        return self._ext[1]

    def forward(self, history, target, near_pois, target_region):   # e.g. model.py:1212-1222
        if self.training:
            raise NotImplementedError(f"{type(self).__name__}: training mode is not implemented on the HIP path")
        self.extended_tables(near_pois)
        return self._run_forward(history, target)


class New4(_NearPOIModel):
    """New4 (model.py:1169-1306): NAIS_basic's attention over POI rows extended with context
    vectors from each POI's near-POI list: history rows [E_hist | in | out], target rows
    [E_tgt | out | in] (model.py:1215-1236), in = pool of embed_ingoing queried by embed_outgoing
    and out the reverse (self_attention, model.py:1269-1295). Built in one call
    (`nais_new4_tables`)."""

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size):
        super().__init__()
        self._common(item_num, embed_size, hidden_size, beta, embed_size / 2)
        self._emb(("embed_ingoing", embed_size / 4), ("embed_outgoing", embed_size / 4),
                  ("embed_history", embed_size / 2), ("embed_target", embed_size / 2))
        self.embed_region = nn.Embedding(region_embed_size, int(embed_size / 2))
        self._init_weight_()

    def _build_tables(self, near, xh, xt):
        ws = (self.embed_history.weight, self.embed_target.weight, self.embed_ingoing.weight,
              self.embed_outgoing.weight)
        _capi.check(_capi.load().nais_new4_tables(*[w.data_ptr() for w in ws], self.item_num,
                                                  self.embed_size, near.data_ptr(), near.shape[1],
                                                  xh.data_ptr(), xt.data_ptr(),
                                                  _capi.stream_handle(near.device)), "nais_new4_tables")


def _in_out_layout(m, d, lin=None, lin_in=None):
    """The two pools of New4-style self_attention (model.py:1281-1295): out = pool of
    embed_outgoing queried by embed_ingoing[near[p][0]], in = the reverse."""
    ein, eout = m.embed_ingoing.weight, m.embed_outgoing.weight
    return [("out", ein, eout, int(d), d, lin), ("in", eout, ein, int(d), d, lin_in)]


def _lin(*layers):
    return tuple(t for l in layers for t in (l.weight, l.bias))


class New4_padding(_NearPOIModel):
    """New4_padding (model.py:1308-1445): New4 with (item_num + 1)-row tables, padding_idx=0;
    the forward is New4's (rows p < item_num of every table are read)."""

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size):
        super().__init__()
        self._common(item_num, embed_size, hidden_size, beta, embed_size / 2)
        for name, d in (("embed_ingoing", embed_size / 4), ("embed_outgoing", embed_size / 4),
                        ("embed_history", embed_size / 2), ("embed_target", embed_size / 2)):
            setattr(self, name, nn.Embedding(item_num + 1, int(d), padding_idx=0))
        self.embed_region = nn.Embedding(region_embed_size + 1, int(embed_size / 2), padding_idx=0)
        self._init_weight_()

    def _layout(self):
        E = self.embed_size
        return (_in_out_layout(self, E / 4), [self.embed_history.weight, "in", "out"],
                [self.embed_target.weight, "out", "in"])


class all_in_out(_NearPOIModel):
    """all_in_out (model.py:1447-1576): no per-role POI embedding; history rows
    [E_hist_in | E_hist_out | in | out], target rows [E_hist_out | E_hist_in | out | in]
    (model.py:1510-1517; the target rows read the embed_history_* tables too)."""

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size):
        super().__init__()
        self._common(item_num, embed_size, hidden_size, beta, embed_size / 2)
        self._emb(("embed_ingoing", embed_size / 4), ("embed_outgoing", embed_size / 4),
                  ("embed_history_ingoing", embed_size / 4), ("embed_history_outgoing", embed_size / 4),
                  ("embed_target_ingoing", embed_size / 4), ("embed_target_outgoing", embed_size / 4))
        self._init_weight_()

    def _layout(self):
        a, b = self.embed_history_ingoing.weight, self.embed_history_outgoing.weight
        return _in_out_layout(self, self.embed_size / 4), [a, b, "in", "out"], [b, a, "out", "in"]


class nearPOI_embedding(_NearPOIModel):
    """nearPOI_embedding (model.py:1578-1705): one pool of embed_near (width embed_size/2,
    model.py:1680-1686); history rows [E_hist_in | E_hist_out | r], target rows
    [E_hist_out | E_hist_in | r]."""

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size):
        super().__init__()
        self._common(item_num, embed_size, hidden_size, beta, embed_size / 2)
        self._emb(("embed_near", embed_size / 2),
                  ("embed_history_ingoing", embed_size / 4), ("embed_history_outgoing", embed_size / 4),
                  ("embed_target_ingoing", embed_size / 4), ("embed_target_outgoing", embed_size / 4))
        self._init_weight_()

    def _layout(self):
        e, E = self.embed_near.weight, self.embed_size
        a, b = self.embed_history_ingoing.weight, self.embed_history_outgoing.weight
        return [("r", e, e, E // 2, E / 2, None)], [a, b, "r"], [b, a, "r"]


class no_POI_emb(_NearPOIModel):
    """no_POI_emb (model.py:1707-1820): only the two pools, each embed_size/2 wide
    (model.py:1797-1812); history rows [in | out], target rows [out | in]."""

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size):
        super().__init__()
        self._common(item_num, embed_size, hidden_size, beta, embed_size / 4)
        self._emb(("embed_ingoing", embed_size / 2), ("embed_outgoing", embed_size / 2))
        self._init_weight_()

    def _layout(self):
        return _in_out_layout(self, self.embed_size / 2), ["in", "out"], ["out", "in"]


class transform_ingoing_outgoing(_NearPOIModel):
    """transform_ingoing_outgoing (model.py:1822-1957): New4 whose pools project through
    query / key / value (nn.Linear(embed_size/4)); the `in` pool's values go through `query`, as
    the reference writes it (model.py:1943)."""

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size):
        super().__init__()
        self._common(item_num, embed_size, hidden_size, beta, embed_size / 4)
        self._emb(("embed_ingoing", embed_size / 4), ("embed_outgoing", embed_size / 4),
                  ("embed_history", embed_size / 2), ("embed_target", embed_size / 2))
        self.embed_region = nn.Embedding(region_embed_size, int(embed_size / 2))
        self._init_weight_()

    def _layout(self):
        lin = _lin(self.query, self.key, self.value)
        lin_in = _lin(self.query, self.key, self.query)
        return (_in_out_layout(self, self.embed_size / 4, lin, lin_in),
                [self.embed_history.weight, "in", "out"], [self.embed_target.weight, "out", "in"])


class only_area_not_inout(_NearPOIModel):
    """only_area_not_inout (model.py:2100-2228): one pool of embed_area (embed_size/2,
    model.py:2198-2218); history rows [E_hist | r], target rows [E_tgt | r]."""

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size):
        super().__init__()
        self._common(item_num, embed_size, hidden_size, beta, embed_size / 2)
        self._emb(("embed_area", embed_size / 2), ("embed_history", embed_size / 2),
                  ("embed_target", embed_size / 2))
        self.embed_region = nn.Embedding(region_embed_size, int(embed_size / 2))
        self._init_weight_()

    def _layout(self):
        e, E = self.embed_area.weight, self.embed_size
        return ([("r", e, e, E // 2, E / 2, None)], [self.embed_history.weight, "r"],
                [self.embed_target.weight, "r"])


class transform_attn(_NearPOIModel):
    """transform_attn (model.py:1959-2098): New4's rows, but the NAIS MLP is replaced by a
    dot-product attention of projected rows (model.py:2030-2033): query/key/value are
    nn.Linear(embed_size). The projections act on one POI row each, so they run once per table
    build (`nais_linear_rows`: qt = xt Wq^T + bq, kh = xh Wk^T + bk, vh = xh Wv^T + bv) and the
    forward / catalog use the dot core (`nais_dot_forward`, `nais_dot_pair_table` + the shared
    `nais_pair_gather`). One-item histories keep the reference's batch coupling (include/nais.h).
    The catalog path is always the pairs strategy."""
    _pairs_only = True

    def __init__(self, item_num, embed_size, hidden_size, beta, region_embed_size):
        super().__init__()
        self._common(item_num, embed_size, hidden_size, beta, embed_size)
        self._emb(("embed_ingoing", embed_size / 4), ("embed_outgoing", embed_size / 4),
                  ("embed_history", embed_size / 2), ("embed_target", embed_size / 2))
        self.embed_region = nn.Embedding(region_embed_size, int(embed_size / 2))
        self._init_weight_()

    def _layout(self):
        return (_in_out_layout(self, self.embed_size / 4), [self.embed_history.weight, "in", "out"],
                [self.embed_target.weight, "out", "in"])

    def _build_tables(self, near, xh, xt):
        super()._build_tables(near, xh, xt)
        lib, st = _capi.load(), _capi.stream_handle(near.device)
        P, D = self.item_num, self.embed_size
        proj = []
        for src, lin in ((xt, self.query), (xh, self.key), (xh, self.value)):
            y = torch.empty(P, D, device=near.device)
            _capi.check(lib.nais_linear_rows(src.data_ptr(), D, P, D, lin.weight.data_ptr(),
                                             lin.bias.data_ptr(), D, y.data_ptr(), D, st), "nais_linear_rows")
            proj.append(y)
        self._proj = proj
        t = _capi.NaisDotTables()
        t.embed_dim, t.num_pois, t.beta, t.scale_dim = D, P, float(self.beta), float(D)
        t.xh, t.xt = xh.data_ptr(), xt.data_ptr()
        t.qt, t.kh, t.vh = (y.data_ptr() for y in proj)
        self._dot = t

    def dot_tables(self):
        """`nais_dot_tables_t` of the current tables (extended_tables must have run)."""
        self._item_tables()
        return self._dot

    def forward(self, history, target, near_pois, target_region):   # model.py:2002-2013
        if self.training:
            raise NotImplementedError("transform_attn: training mode is not implemented on the HIP path")
        self.extended_tables(near_pois)
        dev = self._check_device(history, target)
        if history.dim() != 2 or target.dim() != 1 or history.shape[0] != target.shape[0]:
            raise ValueError(f"history must be [b, n] and target [b]; got {tuple(history.shape)}, "
                             f"{tuple(target.shape)}")
        history = history.to(torch.int64)
        if history.dim() == 2 and history.shape[1] > 0 and history.stride(1) != 1:
            history = history.contiguous()
        target = target.to(torch.int64).contiguous()
        b, n = history.shape
        out = torch.empty(b, dtype=torch.float32, device=dev)
        nan = torch.zeros(1, dtype=torch.int32, device=dev)
        _capi.check(_capi.load().nais_dot_forward(
            self._dot, _capi.ptr(history) if n > 0 else None, b, n, history.stride(0) if n > 0 else 0,
            _capi.ptr(target), out.data_ptr(), nan.data_ptr(), _capi.FLAG_SIGMOID,
            _capi.stream_handle(dev)), "nais_dot_forward")
        self._last_nan = nan
        return out

    def _pair_table(self, lib, prm, items, J, c0, w, reg, cor, llm, e, es, ld, stream, work=None):
        _capi.check(lib.nais_dot_pair_table(self.dot_tables(), items.data_ptr(), J, c0, w, e, es, ld, stream),
                    "nais_dot_pair_table")

    def _pair_fixup(self, csr, users, m, scores, c0, c1, stream):
        _capi.check(_capi.load().nais_dot_single_fixup(
            self.dot_tables(), csr.indptr.data_ptr(), csr.indices.data_ptr(), users.data_ptr(), m, c0,
            c1 - c0, scores.data_ptr(), c1 - c0, c0, stream), "nais_dot_single_fixup")
