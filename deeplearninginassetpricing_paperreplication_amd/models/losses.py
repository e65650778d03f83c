"""Loss / metric math of the GAN, vectorised (no per-period or per-moment Python loops).

These are the *semantic* definitions (fp32, PyTorch autograd) that every fused HIP kernel
in ``csrc/`` is tested against.  Formulas follow the reference exactly:

* unconditional loss  `/root/reference/src/model.py:346-387`
* conditional loss    `/root/reference/src/model.py:389-433` (loop over K vectorised)
* residual loss       `/root/reference/src/model.py:435-483` (loop over T vectorised)
* L1 normalisation    `/root/reference/src/model.py:565-594` (loop over T vectorised)
"""
from __future__ import annotations

from typing import Tuple

import torch


def portfolio_returns(weights: torch.Tensor, returns: torch.Tensor, mask: torch.Tensor,
                      weighted: bool = True) -> torch.Tensor:
    """P_t = (N̄ / N_t) Σ_i w R m  (or the plain sum when ``weighted`` is False)."""
    m = mask.float()
    n_t = m.sum(dim=1).clamp(min=1)
    s = (weights * returns * m).sum(dim=1)
    if weighted:
        return s / n_t * n_t.mean()
    return s


def _moment_means(h: torch.Tensor, returns: torch.Tensor, mask: torch.Tensor,
                  sdf: torch.Tensor) -> torch.Tensor:
    """E[k, i] = Σ_t h[k,t,i] R m SDF_t / T_i  with T_i = max(Σ_t m, 1)."""
    m = mask.float()
    t_i = m.sum(dim=0).clamp(min=1)
    q = returns * m * sdf.unsqueeze(1)          # [T, N]
    if h is None:
        return (q.sum(dim=0) / t_i).unsqueeze(0)
    return (h * q.unsqueeze(0)).sum(dim=1) / t_i


def unconditional_loss(weights, returns, mask, weighted: bool = True
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    p = portfolio_returns(weights, returns, mask, weighted)
    e = _moment_means(None, returns, mask, p + 1.0)
    return (e ** 2).mean(), p


def conditional_loss(weights, returns, mask, moments, weighted: bool = True
                     ) -> Tuple[torch.Tensor, torch.Tensor]:
    p = portfolio_returns(weights, returns, mask, weighted)
    e = _moment_means(moments, returns, mask, p + 1.0)
    return (e ** 2).mean(dim=1).mean(), p


def residual_loss(weights: torch.Tensor, returns: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """Mean per-period projection residual over mean per-period R², both over valid stocks.

    Periods with <2 valid stocks are skipped; periods whose w·w ≤ 1e-8 contribute to the
    R² mean but not to the residual mean (the reference's two lists have different
    lengths, `model.py:468-475`).
    """
    m = mask.float()
    n = m.sum(dim=1)
    use = n >= 2
    ww = (weights * weights * m).sum(dim=1)
    rw = (returns * weights * m).sum(dim=1)
    has = use & (ww > 1e-8)
    beta = torch.where(has, rw / torch.where(has, ww, torch.ones_like(ww)), torch.zeros_like(ww))
    resid = ((returns - beta.unsqueeze(1) * weights) ** 2 * m).sum(dim=1) / n.clamp(min=1)
    rsq = (returns ** 2 * m).sum(dim=1) / n.clamp(min=1)
    # no host sync: with no usable period the masked numerators are 0 and the loss is exactly 0
    resid_mean = (resid * has.float()).sum() / has.float().sum().clamp(min=1)
    rsq_mean = (rsq * use.float()).sum() / use.float().sum().clamp(min=1)
    return resid_mean / rsq_mean.clamp(min=1e-8)


def zero_mean_normalize(w_raw: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """Per-period cross-sectional zero mean over valid stocks (`model.py:271-279`)."""
    m = mask.float()
    w = w_raw * m
    mu = (w * m).sum(dim=1, keepdim=True) / m.sum(dim=1, keepdim=True).clamp(min=1)
    return (w - mu) * m


def l1_normalize(weights: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """w_t / max(Σ_i |w_t| m_t, 1e-8) for every period (`model.py:586-590`)."""
    s = (weights.abs() * mask.float()).sum(dim=1, keepdim=True).clamp(min=1e-8)
    return weights / s


def sharpe_monitor(p: torch.Tensor) -> torch.Tensor:
    """mean / (unbiased std + 1e-8) — the in-forward monitor (`model.py:551`)."""
    return p.mean() / (p.std() + 1e-8)
