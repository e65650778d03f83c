"""Module-level GPU path: ``AssetPricingGAN.forward`` / ``get_weights`` on CUDA tensors run the
native HIP engine (fused MFMA towers, fused masked loss reductions, persistent LSTM), not eager
PyTorch ops.

Reference semantics: `/root/reference/src/model.py:485-594` (forward dict, get_weights).

The engine keeps its own copy of the panel (compacted valid rows, bf16 features) and of the
parameters; a call re-uploads the parameters (a few KB) and re-uploads the panel only when the
input tensors changed. ``loss`` is differentiable w.r.t. the module's parameters through
``_EngineLoss`` (the engine's analytic backward); the other outputs are detached, as they
are in every training/evaluation path of the reference.

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
from typing import Dict, Optional

import numpy as np
import torch

from ..models import losses as L

_PHASE = {"unconditional": 1, "conditional": 3, "moment": 2}
_CACHE: "OrderedDict[tuple, _Slot]" = OrderedDict()
_CACHE_MAX = 4


class _Slot:
    def __init__(self, spec):
        from ..engine.runner import GANEngine
        self.eng = GANEngine(spec, 1, max_epochs=8)
        self.data_key = None
        self.T = self.N = 0


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


def _prepare(model, macro, individual, returns, mask) -> _Slot:
    from ..engine.runner import flatten_state
    # eval mode: an engine built without dropout, so the analytic backward of a no-grad-free
    # eval forward (rare, but legal in autograd) sees exactly the forward's activations
    spec = model.spec if model.training else dataclasses.replace(model.spec, dropout=0.0)
    s = _slot(spec)
    key = (_tkey(macro), _tkey(individual), _tkey(returns), _tkey(mask))
    if key != s.data_key:
        batch = {"individual_features": individual.detach(), "returns": returns.detach(),
                 "mask": mask.detach()}
        if macro is not None and model.spec.macro_dim > 0:
            batch["macro_features"] = macro.detach()
        s.eng.set_data(batch)
        s.data_key = key
        s.T, s.N = int(mask.shape[0]), int(mask.shape[1])
    s.eng.eng.set_params(0, flatten_state(model, model.spec))
    if model.training:
        # fresh dropout masks per call (the reference draws new Bernoulli masks every forward)
        s.eng.eng.set_seed(0, int(torch.randint(0, 2 ** 31 - 1, (1,)).item()))
    return s


class _EngineLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, loss_value, slot, spec, phase_id, res_factor, *params):
        ctx.slot, ctx.spec, ctx.phase_id, ctx.res = slot, spec, phase_id, res_factor
        ctx.shapes = [p.shape for p in params]
        ctx.devices = [p.device for p in params]
        return loss_value.clone()

    @staticmethod
    def backward(ctx, g):
        eng = ctx.slot.eng.eng
        P_sdf = ctx.spec.param_counts()[0]

        def grads(phase):
            eng.backward_only(phase)
            return eng.get_grads(0)

        flat = np.zeros(sum(int(np.prod(s)) for s in ctx.shapes), np.float32)
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
        out, o = [], 0
        gs = float(g.item())
        for shp, dev in zip(ctx.shapes, ctx.devices):
            n = int(np.prod(shp))
            out.append(torch.from_numpy(flat[o:o + n].reshape(shp) * gs).to(dev))
            o += n
        return (None, None, None, None, None, *out)


def _ordered_params(model):
    named = dict(model.named_parameters())
    return [named[k] for k, _ in model.spec.param_layout()]


def gan_forward(model, macro, individual, returns, mask, phase: str = "conditional") -> Dict:
    if phase not in _PHASE:
        raise ValueError(f"unknown phase {phase!r}")
    dev = individual.device
    s = _prepare(model, macro, individual, returns, mask)
    eng = s.eng.eng
    eng.forward_split(0, bool(model.training), True)
    T, N, K = s.T, s.N, model.spec.num_moments
    sc = eng.read_ws(0, 0, "scal")
    wn = torch.from_numpy(eng.read_ws(0, 0, "wn").reshape(T, N)).to(dev)
    h = torch.from_numpy(eng.read_ws(0, 0, "h").reshape(T, N, K)).permute(2, 0, 1).contiguous().to(dev)
    p = torch.from_numpy(eng.read_ws(0, 0, "P")).to(dev)
    l_cond, l_unc, l_res = float(sc[0]), float(sc[1]), float(sc[2])
    res_f = float(model.spec.residual_loss_factor)
    if phase == "unconditional":
        total, l_cond_out, l_unc_out = l_unc, 0.0, l_unc
    elif phase == "moment":
        total, l_cond_out, l_unc_out = -l_cond, l_cond, 0.0
    else:
        total, l_cond_out, l_unc_out = l_cond, l_cond, l_unc
    if res_f > 0:
        total += res_f * l_res
    loss = torch.tensor(total, dtype=torch.float32, device=dev)
    params = _ordered_params(model)
    if torch.is_grad_enabled() and any(q.requires_grad for q in params):
        loss = _EngineLoss.apply(loss, s, model.spec, _PHASE[phase], res_f, *params)
    hidden = None
    lstm = getattr(model.sdf_net, "macro_lstm", None)
    if lstm is not None and macro is not None:
        with torch.no_grad():
            _, hidden = lstm(macro)
    return {
        "weights": wn, "loss": loss,
        "loss_unconditional": torch.tensor(l_unc_out, device=dev),
        "loss_conditional": torch.tensor(l_cond_out, device=dev),
        "loss_residual": torch.tensor(l_res if res_f > 0 else 0.0, device=dev),
        "sharpe": L.sharpe_monitor(p), "portfolio_returns": p, "hidden": hidden, "moments": h,
    }


_ZEROS: Dict[tuple, torch.Tensor] = {}


def gan_weights(model, macro, individual, mask, normalized: bool = False) -> torch.Tensor:
    # get_weights has no returns argument: a cached zero panel keeps the upload cache valid
    zk = _tkey(mask)
    zeros = _ZEROS.get(zk)
    if zeros is None:
        _ZEROS.clear()
        zeros = _ZEROS[zk] = torch.zeros(mask.shape, dtype=torch.float32, device=mask.device)
    s = _prepare(model, macro, individual, zeros, mask)
    s.eng.eng.forward_split(0, bool(model.training), False)
    w = torch.from_numpy(s.eng.eng.read_ws(0, 0, "wn").reshape(s.T, s.N)).to(individual.device)
    if normalized:
        w = L.l1_normalize(w, mask)
    return w
