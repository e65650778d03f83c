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
changed. ``loss`` is differentiable w.r.t. the module's parameters through ``_EngineLoss`` (the
engine's analytic backward); the other outputs are detached, as in every training / evaluation
path of the reference. ``hidden`` is the engine LSTM's final (h_n, c_n) of every layer.

Gradient scopes per phase (what ``loss.backward()`` produces, as in autograd):
  * 'unconditional': SDF params <- engine phase-1 backward; moment params get no gradient.
  * 'conditional'  : SDF params <- phase-3 backward; moment params <- -(phase-2 backward)
                     (phase 2 differentiates -L_cond).
  * 'moment'       : moment params <- phase-2 backward; SDF params <- -(phase-3 backward)
                     (only exact with residual_loss_factor == 0; with a residual term the SDF
                     side is unsupported and raises, the reference freezes it in that phase).
"""
from __future__ import annotations

import dataclasses
from collections import OrderedDict
from typing import Dict, List, Optional

import torch

from ..config import ModelSpec
from ..models import losses as L

_PHASE = {"unconditional": 1, "conditional": 3, "moment": 2}
_CACHE: "OrderedDict[tuple, _Slot]" = OrderedDict()
_CACHE_MAX = 4
SC = dict(loss_cond=0, loss_unc=1, loss_res=2, train_sharpe=3)


class _Slot:
    def __init__(self, spec):
        from ..engine.runner import GANEngine
        self.eng = GANEngine(spec, 1, max_epochs=8)
        self.spec = spec
        self.data_key = None
        self.param_key = None
        self.T = self.N = 0
        self.step = 0
        self.eng.eng.set_seed(0, 0x5EED)


def _slot(spec) -> _Slot:
    key = repr(spec)
    s = _CACHE.get(key)
    if s is None:
        s = _Slot(spec)
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
             training: bool) -> _Slot:
    # eval mode: an engine built without dropout, so the analytic backward of an eval forward
    # (rare, but legal in autograd) sees exactly the forward's activations
    sp = spec if training else dataclasses.replace(spec, dropout=0.0)
    s = _slot(sp)
    dev = individual.device
    torch.cuda.set_device(dev)
    key = (_tkey(macro), _tkey(individual), _tkey(returns), _tkey(mask))
    if key != s.data_key:
        batch = {"individual_features": individual.detach(), "returns": returns.detach(),
                 "mask": mask.detach()}
        if macro is not None and spec.macro_dim > 0:
            batch["macro_features"] = macro.detach()
        s.eng.set_data(batch)
        s.data_key = key
        s.T, s.N = int(mask.shape[0]), int(mask.shape[1])
    pkey = tuple((p.data_ptr(), p._version) for p in params)
    if pkey != s.param_key:
        s._flat = flat_fn(dev).contiguous()            # kept alive until the next call
    s.ts = _bind(s, dev)               # the engine waits for torch's queued work (panel, params)
    if pkey != s.param_key:
        s.eng.eng.set_params_dev(0, s._flat.data_ptr())
        s.param_key = pkey
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


class _EngineLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, loss_value, slot, spec, phase_id, res_factor, to_params, *params):
        ctx.slot, ctx.spec, ctx.phase_id, ctx.res, ctx.to_params = slot, spec, phase_id, res_factor, to_params
        return loss_value.clone()

    @staticmethod
    def backward(ctx, g):
        s = ctx.slot
        eng = s.eng.eng
        dev = g.device
        ts = _bind(s, dev)
        P = sum(int(n) for n in ctx.spec.param_counts())
        P_sdf = ctx.spec.param_counts()[0]

        def grads(phase):
            out = torch.empty(P, dtype=torch.float32, device=dev)
            eng.join_from(ts)          # (out may reuse memory torch's stream still reads)
            eng.backward_only(phase, False)
            eng.copy_grads(0, out.data_ptr())
            _release(s, ts)
            return out

        flat = torch.zeros(P, dtype=torch.float32, device=dev)
        if ctx.phase_id == 1:
            flat[:P_sdf] = grads(1)[:P_sdf]
        elif ctx.phase_id == 3:
            flat[:P_sdf] = grads(3)[:P_sdf]
            flat[P_sdf:] = -grads(2)[P_sdf:]
        else:
            flat[P_sdf:] = grads(2)[P_sdf:]
            if ctx.res > 0:
                raise NotImplementedError("SDF gradient of the 'moment' loss with a residual term")
            flat[:P_sdf] = -grads(3)[:P_sdf]
        return (None, None, None, None, None, None, *ctx.to_params(flat * g))


def _split_flat(spec: ModelSpec, params: List[torch.Tensor]):
    sizes = [int(p.numel()) for p in params]

    def to_params(flat: torch.Tensor):
        return [c.reshape(p.shape).to(p.dtype) for c, p in zip(torch.split(flat, sizes), params)]
    return to_params


def gan_forward(model, macro, individual, returns, mask, phase: str = "conditional") -> Dict:
    if phase not in _PHASE:
        raise ValueError(f"unknown phase {phase!r}")
    dev = individual.device
    params = _ordered_params(model)
    s = _prepare(model, model.spec, params, lambda d: _flat_params(params, d), macro, individual, returns,
                 mask, bool(model.training))
    eng = s.eng.eng
    eng.forward_split(0, bool(model.training), True, False)
    T, N, K = s.T, s.N, model.spec.num_moments
    sc = _copy(s, "scal", 8, dev)
    wn = _copy(s, "wn", T * N, dev).reshape(T, N)
    h = _copy(s, "h", T * N * K, dev).reshape(T, N, K).permute(2, 0, 1)
    p = _copy(s, "P", T, dev)
    hidden = None
    if model.spec.rnn_layers > 0 and macro is not None:
        Lr, H = model.spec.rnn_layers, model.spec.rnn_hidden
        h_n = torch.empty(Lr, 1, H, device=dev)
        c_n = torch.empty(Lr, 1, H, device=dev)
        eng.copy_hidden(0, h_n.data_ptr(), c_n.data_ptr())
        hidden = (h_n, c_n)
    _release(s, s.ts)                  # torch's stream waits for the engine's results
    l_cond, l_unc, l_res = sc[SC["loss_cond"]], sc[SC["loss_unc"]], sc[SC["loss_res"]]
    res_f = float(model.spec.residual_loss_factor)
    zero = torch.zeros((), device=dev)
    if phase == "unconditional":
        total, l_cond_out, l_unc_out = l_unc, zero, l_unc
    elif phase == "moment":
        total, l_cond_out, l_unc_out = -l_cond, l_cond, zero
    else:
        total, l_cond_out, l_unc_out = l_cond, l_cond, l_unc
    if res_f > 0:
        total = total + res_f * l_res
    loss = total.clone()
    if torch.is_grad_enabled() and any(q.requires_grad for q in params):
        loss = _EngineLoss.apply(loss, s, model.spec, _PHASE[phase], res_f, _split_flat(model.spec, params),
                                 *params)
    return {
        "weights": wn, "loss": loss, "loss_unconditional": l_unc_out, "loss_conditional": l_cond_out,
        "loss_residual": l_res if res_f > 0 else zero,
        "sharpe": L.sharpe_monitor(p), "portfolio_returns": p, "hidden": hidden, "moments": h,
    }


_ZEROS: Dict[tuple, torch.Tensor] = {}


def _zeros_like_mask(mask):
    zk = _tkey(mask)
    zeros = _ZEROS.get(zk)
    if zeros is None:
        _ZEROS.clear()
        zeros = _ZEROS[zk] = torch.zeros(mask.shape, dtype=torch.float32, device=mask.device)
    return zeros


def gan_weights(model, macro, individual, mask, normalized: bool = False) -> torch.Tensor:
    # get_weights has no returns argument: a cached zero panel keeps the upload cache valid
    params = _ordered_params(model)
    s = _prepare(model, model.spec, params, lambda d: _flat_params(params, d), macro, individual,
                 _zeros_like_mask(mask), mask, bool(model.training))
    s.eng.eng.forward_split(0, bool(model.training), False, False)
    w = _copy(s, "wn", s.T * s.N, individual.device).reshape(s.T, s.N)
    _release(s, s.ts)
    if normalized:
        w = L.l1_normalize(w, mask)
    return w


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
        loss = _EngineLoss.apply(loss, s, s.spec, 1, 0.0, _simple_to_params(model, spec), *params)
    return {"weights": w, "loss": loss, "sharpe": L.sharpe_monitor(p), "portfolio_returns": p}
