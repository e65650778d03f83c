"""Portfolio math shared by the ensemble evaluator, the plots and the distributed ensemble.

Vectorised (no per-period Python loops) versions of the reference's post-processing:
  * ensemble averaging of L1-normalised weights + per-period re-normalisation
    (`/root/reference/src/evaluate_ensemble.py:137-157`): rows whose masked abs-sum is
    <= 1e-8 are left as they are;
  * portfolio returns sum_i w R m;
  * paper-convention statistics of the SDF factor F = -w.R (numpy std, ddof=0)
    (`evaluate_ensemble.py:46-50,169-171`, `plots.py:404-426`).
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np

PAPER_TEST_SHARPE = 0.75


def renormalize(weights: np.ndarray, mask: np.ndarray) -> np.ndarray:
    """Per-period L1 re-normalisation over valid entries; near-zero rows untouched."""
    w = np.array(weights, copy=True)
    s = np.abs(w.astype(np.float64) * mask.astype(np.float64)).sum(axis=1, keepdims=True)
    ok = s > 1e-8
    q = np.divide(w, s, out=np.zeros(w.shape, np.float64), where=ok)
    return np.where(ok, q, w).astype(w.dtype)


def average_weights(weight_list: Sequence[np.ndarray], mask: np.ndarray) -> np.ndarray:
    """Mean over models of their normalised weights, then re-normalised per period."""
    return renormalize(np.mean(np.stack(list(weight_list)), axis=0), mask)


def portfolio_returns(weights: np.ndarray, returns: np.ndarray, mask: np.ndarray) -> np.ndarray:
    return (weights * returns * mask.astype(weights.dtype)).sum(axis=1)


def sharpe_ddof0(r: np.ndarray) -> float:
    """Monthly Sharpe with numpy's population std (0 below 1e-8), as in the ensemble tools."""
    r = np.asarray(r)
    sd = r.std()
    return 0.0 if sd < 1e-8 else float(r.mean() / sd)


def sdf_statistics(sdf_ret: np.ndarray) -> Dict[str, float]:
    """Table-2 style statistics of the SDF factor series (`plots.py:404-426`)."""
    r = np.asarray(sdf_ret, dtype=np.float64)
    mu, sd = r.mean(), r.std()
    z = (r - mu) / sd if sd > 0 else np.zeros_like(r)
    growth = np.cumprod(1.0 + r)
    peak = np.maximum.accumulate(growth)
    return {
        "mean": float(mu), "std": float(sd), "sharpe": float(mu / sd) if sd > 0 else float("nan"),
        "sharpe_annual": float(mu / sd * np.sqrt(12.0)) if sd > 0 else float("nan"),
        "min": float(r.min()), "max": float(r.max()),
        "skew": float((z ** 3).mean()), "kurtosis": float((z ** 4).mean() - 3.0),
        "cumulative_return": float(growth[-1] - 1.0),
        "max_drawdown": float(((growth - peak) / peak).min()),
    }


def ensemble_sharpes(weights_by_model: Sequence[Dict[str, np.ndarray]], batches: Dict[str, Dict]) -> Dict:
    """Individual (test) and ensemble (train/valid/test) paper-sign Sharpe ratios.

    ``weights_by_model[m][split]`` are the model's L1-normalised [T, N] weights; ``batches``
    holds numpy ``returns`` / ``mask`` per split.
    """
    out = {}
    for split, b in batches.items():
        R, m = b["returns"], b["mask"]
        avg = average_weights([w[split] for w in weights_by_model], m)
        out[f"{split}_sharpe"] = sharpe_ddof0(-portfolio_returns(avg, R, m))
    tb = batches["test"]
    out["individual_sharpes"] = [
        -sharpe_ddof0(portfolio_returns(w["test"], tb["returns"], tb["mask"])) for w in weights_by_model]
    return out


def ensemble_sharpes_device(wstack: Dict, batches: Dict[str, Dict]) -> Dict:
    """``ensemble_sharpes`` with the averaging, re-normalisation and portfolio returns in the
    native K11 kernel (``k_ensemble``) on the GPU. ``wstack[split]`` is a CUDA tensor [G, T, N]
    of the models' L1-normalised weights (e.g. straight out of an RCCL all-gather); ``batches``
    holds the splits' returns / mask (torch or numpy). Only the [T] and [G, T] portfolio series
    come back to the host."""
    import torch
    from ..ops.native import load
    nat = load(required=True)
    out = {}
    ind = None
    for split, b in batches.items():
        W = wstack[split].float()
        if not W.is_cuda:
            W = W.to(torch.device("cuda", torch.cuda.current_device()))
        W = W.contiguous()
        G, T, N = W.shape
        dev = W.device
        R = torch.as_tensor(b["returns"]).to(dev, torch.float32).contiguous()
        m = torch.as_tensor(b["mask"]).to(dev, torch.float32).contiguous()
        port = torch.empty(T, dtype=torch.float32, device=dev)
        pind = torch.empty(G, T, dtype=torch.float32, device=dev)
        nat.ensemble_portfolios(W.data_ptr(), G, T, N, R.data_ptr(), m.data_ptr(), port.data_ptr(), pind.data_ptr(),
                                torch.cuda.current_stream(dev).cuda_stream)
        pr = port.cpu().numpy().astype(np.float64)
        out[f"{split}_sharpe"] = sharpe_ddof0(-pr)
        if split == "test":
            ind = pind.cpu().numpy().astype(np.float64)
    if ind is not None:
        out["individual_sharpes"] = [-sharpe_ddof0(ind[g]) for g in range(ind.shape[0])]
    return out


# ------------------------------------------------------------------------------------------
# Paper metrics the reference does not implement (EV and XS-R² of Table I,
# turnover of Table A.VII, max 1-month loss of Table A.VI). The paper's loadings come from a
# separate beta network; here the loading direction of period t is the SDF weight vector itself
# (the cross-sectional projection the reference's residual loss uses, `model.py:435-483`),
# which makes the metrics computable from any checkpoint's weights.
# ------------------------------------------------------------------------------------------
def _projection_residuals(weights: np.ndarray, returns: np.ndarray, mask: np.ndarray) -> np.ndarray:
    m = mask.astype(np.float64)
    w = weights.astype(np.float64) * m
    r = returns.astype(np.float64) * m
    ww = (w * w).sum(axis=1, keepdims=True)
    rw = (r * w).sum(axis=1, keepdims=True)
    beta = np.divide(rw, ww, out=np.zeros_like(rw), where=ww > 1e-12)
    return (r - beta * w) * m


def explained_variation(weights: np.ndarray, returns: np.ndarray, mask: np.ndarray) -> float:
    """EV = 1 - sum_t mean_i eps^2 / sum_t mean_i R^2 over valid stocks (paper eq. for Table I)."""
    m = mask.astype(np.float64)
    n = np.maximum(m.sum(axis=1), 1.0)
    eps = _projection_residuals(weights, returns, mask)
    r = returns.astype(np.float64) * m
    den = ((r * r).sum(axis=1) / n).sum()
    return float(1.0 - ((eps * eps).sum(axis=1) / n).sum() / den) if den > 0 else float("nan")


def cross_sectional_r2(weights: np.ndarray, returns: np.ndarray, mask: np.ndarray) -> float:
    """XS-R² = 1 - mean_i (T_i/T) mean_t(eps_i)^2 / mean_i (T_i/T) mean_t(R_i)^2."""
    m = mask.astype(np.float64)
    T = m.shape[0]
    ti = m.sum(axis=0)
    ok = ti > 0
    eps = _projection_residuals(weights, returns, mask)
    r = returns.astype(np.float64) * m
    e_bar = np.divide(eps.sum(axis=0), ti, out=np.zeros_like(ti), where=ok)
    r_bar = np.divide(r.sum(axis=0), ti, out=np.zeros_like(ti), where=ok)
    num = ((ti / T) * e_bar ** 2)[ok].mean()
    den = ((ti / T) * r_bar ** 2)[ok].mean()
    return float(1.0 - num / den) if den > 0 else float("nan")


def turnover(weights: np.ndarray, returns: np.ndarray, mask: np.ndarray) -> float:
    """Mean over t of sum_i |w_{t+1,i} - w_{t,i} (1 + R_{t,i}) / (1 + sum_j w_{t,j} R_{t,j})|."""
    m = mask.astype(np.float64)
    w = weights.astype(np.float64) * m
    r = returns.astype(np.float64) * m
    if w.shape[0] < 2:
        return 0.0
    gross = 1.0 + (w * r).sum(axis=1, keepdims=True)
    drift = np.divide(w * (1.0 + r), gross, out=np.zeros_like(w), where=np.abs(gross) > 1e-12)
    return float(np.abs(w[1:] - drift[:-1]).sum(axis=1).mean())


def paper_metrics(weights: np.ndarray, returns: np.ndarray, mask: np.ndarray) -> Dict[str, float]:
    """Sharpe / EV / XS-R² / turnover / max 1-month loss (std units) of the SDF factor F = -w.R."""
    f = -portfolio_returns(weights, returns, mask).astype(np.float64)
    sd = f.std()
    return {
        "sharpe": sharpe_ddof0(f),
        "ev": explained_variation(weights, returns, mask),
        "xs_r2": cross_sectional_r2(weights, returns, mask),
        "turnover": turnover(weights, returns, mask),
        "max_1m_loss_std": float(-f.min() / sd) if sd > 0 else float("nan"),
    }
