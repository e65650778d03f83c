"""Module-level GPU path: ``AssetPricingGAN.forward`` / ``get_weights`` and ``SimpleSDF.forward``
on CUDA tensors run the native HIP engine (fused MFMA towers, fused masked loss reductions,
persistent LSTM), not eager PyTorch ops.

Reference semantics: `/root/reference/src/model.py:485-594` (forward dict, get_weights) and
`:620-694` (SimpleSDF).

Everything is stream-ordered with torch's current stream: the engine runs on its own stream and
joins torch's stream with events on entry and exit (``Engine.join_from`` / ``join_to``; it never
queues work on torch's, possibly legacy NULL, stream). Parameters go
to the engine as one device-to-device copy of the flat fp32 vector (skipped when no parameter
changed since the last call), results come back as device-to-device copies into torch tensors,
and the dropout stream advances with a one-int kernel -- a forward / backward pair issues no
host synchronisation (a training step's only sync is the caller's ``.item()``). The engine keeps
its own copy of the panel (compacted valid rows) and re-uploads it only when the input tensors
changed.

Autograd (as the reference's modules, `/root/reference/src/model.py:553-563`):
  * ``loss`` -> the engine's analytic backward of the fused loss (``_EngineLoss``);
  * ``weights`` / ``portfolio_returns`` -> the raw SDF weights enter torch through ``_TowerW``
    (zero-mean normalisation and the portfolio sum are torch ops) whose backward is the engine's
    SDF tower backward from the incoming dL/dw (``Engine.xs_backward``, phase 1);
  * ``moments`` -> ``_TowerH``: the engine's moment tower backward from dL/dh (phase 2);
  * ``hidden`` (an initial (h0, c0) passed in) -> dL/d(h0, c0) from the LSTM backward.
So a caller's loss built from any output backpropagates to the parameters; combined losses
accumulate through the separate paths. The residual term (``residual_loss_factor``) is a torch
function of the differentiable weights, the engine computes the moment losses only (this also
gives the 'moment' phase's SDF gradient with a residual term).

Gradient scopes of ``loss`` per phase (what ``loss.backward()`` produces, as in autograd):
  * 'unconditional': SDF params <- engine phase-1 backward; moment params get no gradient.
  * 'conditional'  : SDF params <- phase-3 backward; moment params <- -(phase-2 backward)
                     (phase 2 differentiates -L_cond).
  * 'moment'       : moment params <- phase-2 backward; SDF params <- -(phase-3 backward).

The tower precision is ``set_precision('bf16' | 'fp32')`` (default bf16, or the
``DLAP_MODULE_PRECISION`` environment variable); fp32 is the reference's precision.
A repeated forward redraws the dropout masks: backpropagate a forward's outputs before the
next forward of the same model (the engine recomputes the masks of the last forward).
"""
from __future__ import annotations

import dataclasses
import os
import weakref
from collections import OrderedDict
from typing import Dict, List, Optional

import torch

from ..config import ModelSpec
from ..models import losses as L

_PHASE = {"unconditional": 1, "conditional": 3, "moment": 2}
_CACHE: "OrderedDict[tuple, _Slot]" = OrderedDict()
_CACHE_MAX = 4
SC = dict(loss_cond=0, loss_unc=1, loss_res=2, train_sharpe=3)


_PRECISION = {"value": os.environ.get("DLAP_MODULE_PRECISION", "bf16")}


def set_precision(precision: str) -> None:
    """Tower precision of the module-level GPU path: 'bf16' (default) or 'fp32' (reference)."""
    if precision not in ("bf16", "fp32"):
        raise ValueError(f"precision must be 'bf16' or 'fp32', not {precision!r}")
    _PRECISION["value"] = precision


class _Slot:
    def __init__(self, spec, precision):
        from ..engine.runner import GANEngine
        self.eng = GANEngine(spec, 1, max_epochs=8, precision=precision)
        self.spec = spec
        self.data_key = None
        self.param_key = None
        self.T = self.N = 0
        self.idx = None                 # flat indices of the valid (t, i): the engine's row order
        self.hidden_set = False
        self.step = 0
        # the dropout stream: seeded from torch's generator (torch.manual_seed reproduces it)
        self.eng.eng.set_seed(0, int(torch.randint(0, 2 ** 31 - 1, (1,)).item()))


class _ParamKey:
    """Identity of the uploaded parameter set: the parameter objects themselves (weak
    references) plus their storage addresses and autograd versions. Addresses alone are not
    enough: once a model is freed the caching allocator hands its storage to the next one, whose
    fresh parameters then carry the same addresses and version 0."""

    def __init__(self, params: List[torch.Tensor]):
        self.refs = [weakref.ref(p) for p in params]
        self.sig = tuple((p.data_ptr(), p._version) for p in params)

    def matches(self, params: List[torch.Tensor]) -> bool:
        return (len(params) == len(self.refs) and all(r() is p for r, p in zip(self.refs, params))
                and self.sig == tuple((p.data_ptr(), p._version) for p in params))


def invalidate_param_cache() -> None:
    """Make the next module-level GPU call re-upload the parameters and the panel.

    The engine keeps the last uploaded parameter vector and skips the upload while the very same
    parameter objects have the same storage and autograd versions; in-place edits through
    ``p.data`` (``p.data.copy_(...)``, ``p.data.mul_(...)``) do not bump the version counter, so
    call this after them (``load_state_dict`` and optimiser steps bump it and need nothing). The
    panel is cached the same way (the tensor objects plus storage address, shape, version and
    dtype: a different tensor at a recycled address is a new panel); call this too after writing
    new values into a panel tensor in place through ``.data``."""
    for s in _CACHE.values():
        s.param_key = None
        s.data_key = None


def _slot(spec) -> _Slot:
    prec = _PRECISION["value"]
    key = (repr(spec), prec)
    s = _CACHE.get(key)
    if s is None:
        s = _Slot(spec, prec)
        _CACHE[key] = s
        while len(_CACHE) > _CACHE_MAX:
            _CACHE.popitem(last=False)
    else:
        _CACHE.move_to_end(key)
    return s


def _tkey(t: Optional[torch.Tensor]):
    if t is None:
        return None
    return (t.data_ptr(), tuple(t.shape), t._version, str(t.dtype))


class _PanelKey:
    """Identity of the uploaded panel: weak references to its tensor objects plus their
    (address, shape, version, dtype). As for the parameters (``_ParamKey``), the address alone is
    not enough: a loop that calls ``x.cuda()`` on a new host batch every step gets the freed
    block back at the same address with version 0."""

    def __init__(self, tensors):
        self.refs = [None if t is None else weakref.ref(t) for t in tensors]
        self.sig = tuple(_tkey(t) for t in tensors)

    def matches(self, tensors) -> bool:
        if len(tensors) != len(self.refs):
            return False
        for r, t in zip(self.refs, tensors):
            if (r is None) != (t is None) or (r is not None and r() is not t):
                return False
        return self.sig == tuple(_tkey(t) for t in tensors)


def _ordered_params(model) -> List[torch.Tensor]:
    named = dict(model.named_parameters())
    return [named[k] for k, _ in model.spec.param_layout()]


def _flat_params(params: List[torch.Tensor], device) -> torch.Tensor:
    return torch.cat([p.detach().reshape(-1).to(device=device, dtype=torch.float32) for p in params])


def _bind(s: _Slot, device) -> int:
    """Order the engine's stream after torch's current stream; returns that stream's handle
    for the matching ``_release``."""
    torch.cuda.set_device(device)
    ts = torch.cuda.current_stream(device).cuda_stream
    s.eng.eng.join_from(ts)
    return ts


def _release(s: _Slot, ts: int):
    """Order torch's stream ``ts`` after everything queued on the engine so far."""
    s.eng.eng.join_to(ts)


def _prepare(model, spec: ModelSpec, params: List[torch.Tensor], flat_fn, macro, individual, returns, mask,
             training: bool, hidden=None) -> _Slot:
    # eval mode: an engine built without dropout, so the analytic backward of an eval forward
    # (rare, but legal in autograd) sees exactly the forward's activations; the residual term is
    # a torch function of the differentiable weights (the engine computes the moment losses)
    sp = spec if training else dataclasses.replace(spec, dropout=0.0)
    sp = dataclasses.replace(sp, residual_loss_factor=0.0)
    s = _slot(sp)
    dev = individual.device
    torch.cuda.set_device(dev)
    panel = (macro, individual, returns, mask)
    if s.data_key is None or not s.data_key.matches(panel):
        batch = {"individual_features": individual.detach(), "returns": returns.detach(),
                 "mask": mask.detach()}
        if macro is not None and spec.macro_dim > 0:
            batch["macro_features"] = macro.detach()
        s.eng.set_data(batch)
        s.data_key = _PanelKey(panel)
        s.T, s.N = int(mask.shape[0]), int(mask.shape[1])
        mflat = mask.detach().reshape(-1).bool()
        s.idx = mflat.nonzero().reshape(-1)              # (one sync per new panel)
        s.midx = (~mflat).nonzero().reshape(-1)          # masked entries (moments only)
    fresh = s.param_key is None or not s.param_key.matches(params)
    if fresh:
        s._flat = flat_fn(dev).contiguous()            # kept alive until the next call
    s.ts = _bind(s, dev)               # the engine waits for torch's queued work (panel, params)
    if fresh:
        s.eng.eng.set_params_dev(0, s._flat.data_ptr())
        s.param_key = _ParamKey(params)
    if hidden is not None:
        h0, c0 = (x.detach().reshape(-1).to(dev, torch.float32).contiguous() for x in hidden)
        s._hidden = (h0, c0)                                       # kept alive until copied
        s.eng.eng.set_hidden(0, 0, h0.data_ptr(), c0.data_ptr())
        s.hidden_set = True
    elif s.hidden_set:
        s.eng.eng.set_hidden(0, 0, 0, 0)
        s.hidden_set = False
    if training:
        # fresh dropout masks per call (the reference draws new Bernoulli masks every forward)
        s.step += 1
        s.eng.eng.set_drop_step(0, s.step)
    return s


def _copy(s: _Slot, name: str, n: int, dev) -> torch.Tensor:
    out = torch.empty(n, dtype=torch.float32, device=dev)
    s.eng.eng.join_from(s.ts)          # (out may reuse memory torch's stream still reads)
    got = s.eng.eng.copy_ws(0, 0, name, out.data_ptr())
    assert got == n, (name, got, n)
    return out


def _hidden_grad(s: _Slot, spec: ModelSpec, dev, ts):
    """dL/d(h0, c0) of the last LSTM backward, shaped like nn.LSTM's state [layers, 1, H]."""
    Lr, H = spec.rnn_layers, spec.rnn_hidden
    dh = torch.empty(Lr, 1, H, dtype=torch.float32, device=dev)
    dc = torch.empty(Lr, 1, H, dtype=torch.float32, device=dev)
    s.eng.eng.join_from(ts)
    s.eng.eng.copy_hidden_grad(0, dh.data_ptr(), dc.data_ptr())
    _release(s, ts)
    return dh, dc


class _EngineLoss(torch.autograd.Function):
    """The engine's fused moment loss (no residual term) as a function of the parameters and of
    an initial LSTM state (h0, c0) when one was passed (``nh`` = 2, else 0)."""

    @staticmethod
    def forward(ctx, loss_value, slot, spec, phase_id, to_params, nh, *inputs):
        ctx.slot, ctx.spec, ctx.phase_id, ctx.to_params, ctx.nh = slot, spec, phase_id, to_params, nh
        return loss_value.clone()

    @staticmethod
    def backward(ctx, g):
        s = ctx.slot
        eng = s.eng.eng
        dev = g.device
        ts = _bind(s, dev)
        P = sum(int(n) for n in ctx.spec.param_counts())
        P_sdf = ctx.spec.param_counts()[0]
        hg = [None, None]

        def grads(phase):
            out = torch.empty(P, dtype=torch.float32, device=dev)
            eng.join_from(ts)          # (out may reuse memory torch's stream still reads)
            eng.backward_only(phase, False)
            eng.copy_grads(0, out.data_ptr())
            _release(s, ts)
            if phase != 2 and ctx.nh:  # the SDF-side LSTM backward also gave dL/d(h0, c0)
                dh, dc = _hidden_grad(s, ctx.spec, dev, ts)
                sign = -1.0 if ctx.phase_id == 2 else 1.0
                hg[0], hg[1] = sign * dh * g, sign * dc * g
            return out

        flat = torch.zeros(P, dtype=torch.float32, device=dev)
        if ctx.phase_id == 1:
            flat[:P_sdf] = grads(1)[:P_sdf]
        elif ctx.phase_id == 3:
            flat[:P_sdf] = grads(3)[:P_sdf]
            flat[P_sdf:] = -grads(2)[P_sdf:]
        else:
            flat[P_sdf:] = grads(2)[P_sdf:]
            flat[:P_sdf] = -grads(3)[:P_sdf]
        return (None, None, None, None, None, None, *ctx.to_params(flat * g), *hg[:ctx.nh])


class _TowerW(torch.autograd.Function):
    """Raw SDF weights [T, N] (zero where masked) of the engine's forward as a function of the
    SDF parameters (and of (h0, c0) when passed): backward = the engine's SDF tower + LSTM
    backward from the incoming dL/dw (``Engine.xs_backward`` phase 1)."""

    @staticmethod
    def forward(ctx, w_raw, slot, spec, to_params, nh, *inputs):
        ctx.slot, ctx.spec, ctx.to_params, ctx.nh = slot, spec, to_params, nh
        return w_raw.clone()

    @staticmethod
    def backward(ctx, g):
        s = ctx.slot
        dev = g.device
        ts = _bind(s, dev)
        P = sum(int(n) for n in ctx.spec.param_counts())
        P_sdf = ctx.spec.param_counts()[0]
        dwc = g.reshape(-1).index_select(0, s.idx).float().contiguous()     # engine row order
        if dwc.numel() == 0:
            dwc = torch.zeros(1, device=dev)
        out = torch.empty(P, dtype=torch.float32, device=dev)
        s.eng.eng.join_from(ts)
        s.eng.eng.xs_backward(1, dwc.data_ptr(), 0, 0)
        s.eng.eng.copy_grads(0, out.data_ptr())
        _release(s, ts)
        s._keep = dwc
        flat = torch.zeros(P, dtype=torch.float32, device=dev)
        flat[:P_sdf] = out[:P_sdf]
        hg = list(_hidden_grad(s, ctx.spec, dev, ts)) if ctx.nh else []
        return (None, None, None, None, None, *ctx.to_params(flat), *hg)


class _TowerH(torch.autograd.Function):
    """Moments [K, T, N] of the engine's forward as a function of the moment parameters:
    backward = the engine's moment tower backward from dL/dh (``Engine.xs_backward`` phase 2)."""

    @staticmethod
    def forward(ctx, h, slot, spec, to_params, *params):
        ctx.slot, ctx.spec, ctx.to_params = slot, spec, to_params
        return h.clone()

    @staticmethod
    def backward(ctx, g):
        s = ctx.slot
        dev = g.device
        ts = _bind(s, dev)
        P = sum(int(n) for n in ctx.spec.param_counts())
        P_sdf = ctx.spec.param_counts()[0]
        dh = g.permute(1, 2, 0).float().contiguous()                       # engine layout [T][N][K]
        out = torch.empty(P, dtype=torch.float32, device=dev)
        s.eng.eng.join_from(ts)
        s.eng.eng.xs_backward(2, 0, 0, 0, dh.data_ptr())
        s.eng.eng.copy_grads(0, out.data_ptr())
        _release(s, ts)
        s._keep_h = dh
        flat = torch.zeros(P, dtype=torch.float32, device=dev)
        flat[P_sdf:] = out[P_sdf:]
        return (None, None, None, None, *ctx.to_params(flat))


def _split_flat(spec: ModelSpec, params: List[torch.Tensor]):
    sizes = [int(p.numel()) for p in params]

    def to_params(flat: torch.Tensor):
        return [c.reshape(p.shape).to(p.dtype) for c, p in zip(torch.split(flat, sizes), params)]
    return to_params


def _dense_raw(s: _Slot, dev) -> torch.Tensor:
    """The engine's raw SDF weights of the train split as a dense [T, N] tensor (0 where masked)."""
    R = int(s.idx.numel())
    wc = _copy(s, "w", max(R, 1), dev)
    # torch's stream reads wc below: it must wait for the engine's copy first (without this the
    # scatter raced the copy and could read the allocator's previous contents of wc)
    _release(s, s.ts)
    return torch.zeros(s.T * s.N, dtype=torch.float32, device=dev).index_copy(0, s.idx, wc[:R]).reshape(s.T, s.N)


def _masked_moments(model, s: _Slot, h: torch.Tensor, macro, individual) -> torch.Tensor:
    """The engine computes the moments of the valid (t, i) only (the losses never read the
    others); the module returns all of them, as the reference does. The masked entries' moments
    come from the moment network's own modules on just those rows' inputs [macro_t ; x_ti]
    (differentiable; a small GEMM chain over the masked rows)."""
    if s.midx.numel() == 0:
        return h
    T, N, K = s.T, s.N, h.shape[0]
    x = individual.reshape(T * N, -1).index_select(0, s.midx)
    if macro is not None and model.spec.macro_dim > 0:
        x = torch.cat([macro.index_select(0, torch.div(s.midx, N, rounding_mode="floor")), x], 1)
    net = model.moment_net
    hm = torch.tanh(net.output_proj(net.fc_layers(x)))                  # [n_masked, K]
    flat = h.permute(1, 2, 0).reshape(T * N, K).index_copy(0, s.midx, hm.to(h.dtype))
    return flat.reshape(T, N, K).permute(2, 0, 1)


def gan_forward(model, macro, individual, returns, mask, phase: str = "conditional", hidden=None) -> Dict:
    if phase not in _PHASE:
        raise ValueError(f"unknown phase {phase!r}")
    dev = individual.device
    spec = model.spec
    params = _ordered_params(model)
    if hidden is not None and (spec.rnn_layers == 0 or macro is None):
        hidden = None                                # (no LSTM: the reference ignores it too)
    s = _prepare(model, spec, params, lambda d: _flat_params(params, d), macro, individual, returns,
                 mask, bool(model.training), hidden)
    eng = s.eng.eng
    eng.forward_split(0, bool(model.training), True, False)
    T, N, K = s.T, s.N, spec.num_moments
    res_f = float(spec.residual_loss_factor)
    grad = torch.is_grad_enabled() and (any(q.requires_grad for q in params) or
                                        (hidden is not None and any(x.requires_grad for x in hidden)))
    sc = _copy(s, "scal", 8, dev)
    h = _copy(s, "h", T * N * K, dev).reshape(T, N, K).permute(2, 0, 1)
    w_raw = _dense_raw(s, dev) if (grad or res_f > 0) else None
    wn = _copy(s, "wn", T * N, dev).reshape(T, N) if w_raw is None else None
    p = _copy(s, "P", T, dev) if w_raw is None else None
    new_hidden = _new_hidden(s, spec, macro, dev)
    _release(s, s.ts)                 # torch's stream waits for the engine's results
    hin = list(hidden) if hidden is not None else []
    if w_raw is not None:
        to_p = _split_flat(spec, params)
        if grad:
            w_raw = _TowerW.apply(w_raw, s, spec, to_p, len(hin), *params, *hin)
            h = _TowerH.apply(h, s, spec, to_p, *params)
        wn = L.zero_mean_normalize(w_raw, mask) if spec.normalize_w else w_raw * mask.float()
        p = L.portfolio_returns(wn, returns, mask, spec.weighted_loss)
    h = _masked_moments(model, s, h, macro, individual)
    l_cond, l_unc = sc[SC["loss_cond"]], sc[SC["loss_unc"]]
    zero = torch.zeros((), device=dev)
    if phase == "unconditional":
        total, l_cond_out, l_unc_out = l_unc, zero, l_unc
    elif phase == "moment":
        total, l_cond_out, l_unc_out = -l_cond, l_cond, zero
    else:
        total, l_cond_out, l_unc_out = l_cond, l_cond, l_unc
    loss = total.clone()
    if grad:
        loss = _EngineLoss.apply(loss, s, spec, _PHASE[phase], _split_flat(spec, params), len(hin), *params, *hin)
    l_res = zero
    if res_f > 0:
        l_res = L.residual_loss(wn, returns, mask)
        loss = loss + res_f * l_res
    return {
        "weights": wn, "loss": loss, "loss_unconditional": l_unc_out, "loss_conditional": l_cond_out,
        "loss_residual": l_res, "sharpe": L.sharpe_monitor(p), "portfolio_returns": p,
        "hidden": new_hidden, "moments": h,
    }


_ZEROS: Dict[tuple, torch.Tensor] = {}


def _zeros_like_mask(mask):
    zk = _tkey(mask)
    zeros = _ZEROS.get(zk)
    if zeros is None:
        _ZEROS.clear()
        zeros = _ZEROS[zk] = torch.zeros(mask.shape, dtype=torch.float32, device=mask.device)
    return zeros


def _new_hidden(s: _Slot, spec: ModelSpec, macro, dev):
    """Final LSTM state (h_n, c_n) of the last forward, shaped like nn.LSTM's; None without an LSTM."""
    if spec.rnn_layers == 0 or macro is None:
        return None
    Lr, H = spec.rnn_layers, spec.rnn_hidden
    h_n = torch.empty(Lr, 1, H, device=dev)
    c_n = torch.empty(Lr, 1, H, device=dev)
    s.eng.eng.copy_hidden(0, h_n.data_ptr(), c_n.data_ptr())
    return h_n, c_n


def gan_weights(model, macro, individual, mask, normalized: bool = False, hidden=None):
    """``get_weights`` on the engine: (weights, new LSTM state). The weights are differentiable
    in the SDF parameters (and in ``hidden``) when grad mode is on."""
    # get_weights has no returns argument: a cached zero panel keeps the upload cache valid
    spec = model.spec
    params = _ordered_params(model)
    if hidden is not None and (spec.rnn_layers == 0 or macro is None):
        hidden = None
    s = _prepare(model, spec, params, lambda d: _flat_params(params, d), macro, individual,
                 _zeros_like_mask(mask), mask, bool(model.training), hidden)
    s.eng.eng.forward_split(0, bool(model.training), False, False)
    dev = individual.device
    grad = torch.is_grad_enabled() and (any(q.requires_grad for q in params) or
                                        (hidden is not None and any(x.requires_grad for x in hidden)))
    if grad:
        w_raw = _dense_raw(s, dev)
    else:
        w = _copy(s, "wn", s.T * s.N, dev).reshape(s.T, s.N)
    new_hidden = _new_hidden(s, spec, macro, dev)
    _release(s, s.ts)
    if grad:
        hin = list(hidden) if hidden is not None else []
        w_raw = _TowerW.apply(w_raw, s, spec, _split_flat(spec, params), len(hin), *params, *hin)
        w = L.zero_mean_normalize(w_raw, mask) if spec.normalize_w else w_raw * mask.float()
    if normalized:
        w = L.l1_normalize(w, mask)
    return w, new_hidden


# ---- SimpleSDF (`/root/reference/src/model.py:620-694`) on the engine ---------------------
# SimpleSDF is the engine's SDF tower without an LSTM (raw macro columns), unweighted
# unconditional loss, zero-mean weights, and no moment network. Its first Linear takes
# [macro ; x] (macro first) where the engine's SDF takes [x ; macro]: the flat vector permutes
# those columns, and a 1-output moment net with zero weights fills the engine's moment slot
# (never trained: phase-1 gradients only).
def simple_spec(model) -> ModelSpec:
    lin = [m for m in model.net if isinstance(m, torch.nn.Linear)]
    drop = [m for m in model.net if isinstance(m, torch.nn.Dropout)]
    M, F = model.macro_dim, model.individual_dim
    return ModelSpec(macro_dim=M, individual_dim=F, hidden=tuple(l.out_features for l in lin[:-1]),
                     rnn_layers=0, rnn_hidden=0, moment_hidden=(), num_moments=1,
                     dropout=float(drop[0].p) if drop else 0.0, normalize_w=True, weighted_loss=False,
                     residual_loss_factor=0.0)


def _simple_params(model):
    return [p for m in model.net if isinstance(m, torch.nn.Linear) for p in (m.weight, m.bias)]


def _simple_flat(model, spec: ModelSpec, dev) -> torch.Tensor:
    M = model.macro_dim
    lin = [m for m in model.net if isinstance(m, torch.nn.Linear)]
    parts = []
    for j, m in enumerate(lin):
        w = m.weight.detach().float()
        if j == 0 and M > 0:
            w = torch.cat([w[:, M:], w[:, :M]], dim=1)        # [macro ; x] -> [x ; macro]
        parts += [w.reshape(-1), m.bias.detach().float().reshape(-1)]
    n_mom = sum(int(torch.Size(s).numel()) for k, s in spec.param_layout() if k.startswith("moment_net"))
    parts.append(torch.zeros(n_mom, device=dev))
    return torch.cat([p.to(dev) for p in parts])


def _simple_to_params(model, spec: ModelSpec):
    M = model.macro_dim
    params = _simple_params(model)
    sizes = [int(p.numel()) for p in params]

    def to_params(flat: torch.Tensor):
        chunks = list(torch.split(flat[:sum(sizes)], sizes))
        out = []
        for k, (c, p) in enumerate(zip(chunks, params)):
            c = c.reshape(p.shape)
            if k == 0 and M > 0:                              # back to [macro ; x]
                F = p.shape[1] - M
                c = torch.cat([c[:, F:], c[:, :F]], dim=1)
            out.append(c.to(p.dtype))
        return out
    return to_params


def simple_forward(model, macro, individual, returns, mask) -> Dict:
    dev = individual.device
    spec = simple_spec(model)
    params = _simple_params(model)
    s = _prepare(model, spec, params, lambda d: _simple_flat(model, spec, d), macro, individual, returns,
                 mask, bool(model.training))
    s.eng.eng.forward_split(0, bool(model.training), False, False)
    T, N = s.T, s.N
    sc = _copy(s, "scal", 8, dev)
    w = _copy(s, "wn", T * N, dev).reshape(T, N)
    p = _copy(s, "P", T, dev)
    _release(s, s.ts)
    loss = sc[SC["loss_unc"]].clone()
    if torch.is_grad_enabled() and any(q.requires_grad for q in params):
        loss = _EngineLoss.apply(loss, s, s.spec, 1, _simple_to_params(model, spec), 0, *params)
    return {"weights": w, "loss": loss, "sharpe": L.sharpe_monitor(p), "portfolio_returns": p}
