"""SDF generator / moment discriminator modules with the reference's public API.

Parity contract: constructor arguments, submodule names and registration
order equal the reference (`/root/reference/src/model.py:21-694`), so ``state_dict`` keys,
shapes and the default-initialisation RNG stream are identical for a given torch seed.

Execution: on CPU the forward is the vectorised fp32 math of ``models.losses`` (the
semantic oracle).  On a GPU device the whole ``AssetPricingGAN.forward`` / ``get_weights``
runs through the native HIP engine (``ops.fused``): fused MFMA MLP, fused masked
E[h·w·R]² reductions and the persistent LSTM kernel — never eager PyTorch.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from ..config import ModelSpec
from . import losses as L


def _mlp(in_dim: int, widths: List[int], p: float) -> List[nn.Module]:
    mods: List[nn.Module] = []
    for w in widths:
        mods += [nn.Linear(in_dim, w), nn.ReLU(), nn.Dropout(p)]
        in_dim = w
    return mods


class MacroLSTM(nn.Module):
    """Macro-state encoder: one ``nn.LSTM`` over the whole [T, M] sequence (batch of 1).

    Every layer has width ``hidden_dims[-1]`` (reference quirk, `model.py:39-45`).
    """

    def __init__(self, input_dim: int, hidden_dims: List[int], dropout: float = 0.0):
        super().__init__()
        self.hidden_dims = list(hidden_dims)
        self.num_layers = len(self.hidden_dims)
        self.output_dim = self.hidden_dims[-1]
        self.lstm = nn.LSTM(input_size=input_dim, hidden_size=self.output_dim,
                            num_layers=self.num_layers, batch_first=True,
                            dropout=dropout if self.num_layers > 1 else 0)

    def forward(self, x: torch.Tensor, hidden=None):
        out, hidden = self.lstm(x[None], hidden)
        return out[0], hidden

    def init_hidden(self, device) -> Tuple[torch.Tensor, torch.Tensor]:
        h = torch.zeros(self.num_layers, 1, self.output_dim, device=device)
        return h, torch.zeros_like(h)


class MomentNetwork(nn.Module):
    """Discriminator h = tanh(FFN([macro ; x])) → [K, T, N].

    ``use_rnn`` / ``rnn_hidden_dims`` are accepted and ignored, as in the reference
    (`model.py:99-130`).
    """

    def __init__(self, input_dim: int, hidden_dims: List[int], num_moments: int,
                 use_rnn: bool = False, rnn_hidden_dims: List[int] = None, dropout: float = 0.05):
        super().__init__()
        self.use_rnn = use_rnn
        self.num_moments = num_moments
        layers = _mlp(input_dim, list(hidden_dims), dropout)
        self.fc_layers = nn.Sequential(*layers) if layers else nn.Identity()
        last = hidden_dims[-1] if len(hidden_dims) else input_dim
        self.output_proj = nn.Linear(last, num_moments)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        T, N, D = x.shape
        z = self.fc_layers(x.reshape(T * N, D))
        return torch.tanh(self.output_proj(z)).reshape(T, N, -1).permute(2, 0, 1)


class SDFNetwork(nn.Module):
    """Generator: per-stock portfolio weight from [x_i ; LSTM(macro)_t] (`model.py:164-281`)."""

    def __init__(self, macro_dim: int, individual_dim: int, hidden_dims: List[int],
                 use_rnn: bool = True, rnn_hidden_dims: List[int] = None,
                 dropout: float = 0.05, normalize_weights: bool = True):
        super().__init__()
        self.use_rnn = use_rnn
        self.normalize_weights = normalize_weights
        self.macro_dim = macro_dim
        if use_rnn and rnn_hidden_dims and macro_dim > 0:
            self.macro_lstm = MacroLSTM(macro_dim, rnn_hidden_dims, dropout)
            mdim = self.macro_lstm.output_dim
        else:
            self.macro_lstm = None
            mdim = macro_dim
        self.fc_layers = nn.Sequential(*_mlp(mdim + individual_dim, list(hidden_dims), dropout))
        self.output_proj = nn.Linear(hidden_dims[-1] if len(hidden_dims) else mdim + individual_dim, 1)

    def forward(self, macro_features, individual_features, mask, hidden=None):
        T, N, _ = individual_features.shape
        new_hidden = None
        state = macro_features
        if macro_features is not None and self.macro_lstm is not None:
            state, new_hidden = self.macro_lstm(macro_features, hidden)
        if state is not None:
            inp = torch.cat([individual_features, state[:, None, :].expand(T, N, state.shape[-1])], -1)
        else:
            inp = individual_features
        w = self.output_proj(self.fc_layers(inp.reshape(T * N, -1))).reshape(T, N)
        if self.normalize_weights:
            w = L.zero_mean_normalize(w, mask)
        else:
            w = w * mask.float()
        return w, new_hidden


class AssetPricingGAN(nn.Module):
    """The Chen–Pelger–Zhu GAN: ``sdf_net`` (generator) + ``moment_net`` (discriminator).

    ``forward(..., phase)`` semantics (`model.py:485-563`):
      * 'unconditional': loss = L_unc, loss_conditional = 0
      * 'moment':        loss = −L_cond (discriminator ascent), loss_unconditional = 0
      * 'conditional':   loss = L_cond, L_unc computed for logging
    plus ``residual_loss_factor · L_res``; returns the 9-key output dict.
    """

    def __init__(self, config: Dict):
        super().__init__()
        self.config = config
        spec = ModelSpec.from_config(config)
        self.spec = spec
        rnn = config.get("num_units_rnn", [4])
        rnn = [rnn] if isinstance(rnn, int) else list(rnn)
        rnn_m = config.get("num_units_rnn_moment", [32])
        rnn_m = [rnn_m] if isinstance(rnn_m, int) else list(rnn_m)
        use_rnn = config.get("use_rnn", True)
        self.sdf_net = SDFNetwork(
            macro_dim=spec.macro_dim, individual_dim=spec.individual_dim,
            hidden_dims=list(spec.hidden), use_rnn=use_rnn,
            rnn_hidden_dims=rnn if use_rnn else None, dropout=spec.dropout,
            normalize_weights=spec.normalize_w)
        use_rnn_m = config.get("use_rnn_moment", True)
        self.moment_net = MomentNetwork(
            input_dim=spec.moment_in, hidden_dims=list(spec.moment_hidden),
            num_moments=spec.num_moments, use_rnn=use_rnn_m,
            rnn_hidden_dims=rnn_m if use_rnn_m else None, dropout=spec.dropout)
        self.residual_loss_factor = spec.residual_loss_factor
        self.weighted_loss = spec.weighted_loss

    # -- losses (reference method names kept for API parity) ------------------------
    def compute_unconditional_loss(self, weights, returns, mask):
        return L.unconditional_loss(weights, returns, mask, self.weighted_loss)

    def compute_conditional_loss(self, weights, returns, mask, moments):
        return L.conditional_loss(weights, returns, mask, moments, self.weighted_loss)

    def compute_residual_loss(self, weights, returns, mask):
        return L.residual_loss(weights, returns, mask)

    def _moment_input(self, macro, individual):
        if macro is None:
            return individual
        T, N, _ = individual.shape
        return torch.cat([macro[:, None, :].expand(T, N, macro.shape[-1]), individual], -1)

    def forward(self, macro_features, individual_features, returns, mask, hidden=None,
                phase: str = "conditional") -> Dict[str, torch.Tensor]:
        if individual_features.is_cuda:
            from ..ops.fused import gan_forward
            return gan_forward(self, macro_features, individual_features, returns, mask, phase, hidden)
        weights, new_hidden = self.sdf_net(macro_features, individual_features, mask, hidden)
        moments = self.moment_net(self._moment_input(macro_features, individual_features))
        zero = torch.zeros((), device=weights.device)
        if phase == "unconditional":
            loss_unc, p = self.compute_unconditional_loss(weights, returns, mask)
            loss_cond, total = zero, loss_unc
        elif phase == "moment":
            loss_cond, p = self.compute_conditional_loss(weights, returns, mask, moments)
            loss_unc, total = zero, -loss_cond
        else:
            loss_cond, p = self.compute_conditional_loss(weights, returns, mask, moments)
            loss_unc, _ = self.compute_unconditional_loss(weights, returns, mask)
            total = loss_cond
        if self.residual_loss_factor > 0:
            loss_res = self.compute_residual_loss(weights, returns, mask)
            total = total + self.residual_loss_factor * loss_res
        else:
            loss_res = zero
        return {
            "weights": weights, "loss": total, "loss_unconditional": loss_unc,
            "loss_conditional": loss_cond, "loss_residual": loss_res,
            "sharpe": L.sharpe_monitor(p), "portfolio_returns": p,
            "hidden": new_hidden, "moments": moments,
        }

    def get_weights(self, macro_features, individual_features, mask, hidden=None,
                    normalized: bool = False):
        if individual_features.is_cuda:
            from ..ops.fused import gan_weights
            return gan_weights(self, macro_features, individual_features, mask, normalized, hidden)
        w, new_hidden = self.sdf_net(macro_features, individual_features, mask, hidden)
        if normalized:
            w = L.l1_normalize(w, mask)
        return w, new_hidden

    def get_sdf_factor(self, macro_features, individual_features, returns, mask, hidden=None,
                       normalized: bool = True) -> torch.Tensor:
        w, _ = self.get_weights(macro_features, individual_features, mask, hidden, normalized)
        return (w * returns * mask.float()).sum(dim=1)


class SimpleSDF(nn.Module):
    """Non-adversarial baseline: FFN on [macro ; x], zero-mean weights, unconditional loss
    (`model.py:620-694`). On CUDA tensors it runs the native engine's SDF tower (see
    ``ops.fused.simple_forward``)."""

    def __init__(self, macro_dim: int, individual_dim: int, hidden_dims: List[int] = (64, 64),
                 dropout: float = 0.05):
        super().__init__()
        hidden_dims = list(hidden_dims)
        self.macro_dim, self.individual_dim = int(macro_dim), int(individual_dim)
        mods = _mlp(macro_dim + individual_dim, hidden_dims, dropout)
        mods.append(nn.Linear(hidden_dims[-1] if hidden_dims else macro_dim + individual_dim, 1))
        self.net = nn.Sequential(*mods)

    def forward(self, macro_features, individual_features, returns, mask):
        # native engine (ops.fused.simple_forward); without hidden layers the model is one
        # Linear -- a library GEMV, no tower to fuse -- and the torch ops below run it
        if individual_features.is_cuda and any(isinstance(m, nn.ReLU) for m in self.net):
            from ..ops.fused import simple_forward
            return simple_forward(self, macro_features, individual_features, returns, mask)
        T, N, _ = individual_features.shape
        if macro_features is not None:
            x = torch.cat([macro_features[:, None, :].expand(T, N, macro_features.shape[-1]),
                           individual_features], -1)
        else:
            x = individual_features
        w = L.zero_mean_normalize(self.net(x.reshape(T * N, -1)).reshape(T, N), mask)
        p = (w * returns * mask.float()).sum(dim=1)
        e = L._moment_means(None, returns, mask, p + 1.0)
        return {"weights": w, "loss": (e ** 2).mean(), "sharpe": L.sharpe_monitor(p),
                "portfolio_returns": p}
