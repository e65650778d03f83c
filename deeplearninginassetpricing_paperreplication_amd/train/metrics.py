"""Portfolio metrics (`/root/reference/src/train.py:29-42`, `src/plots.py:410-426`)."""
from __future__ import annotations

import numpy as np
import torch


def compute_sharpe(returns) -> float:
    """Monthly Sharpe, unbiased std; 0 when std < 1e-8 (not annualised)."""
    r = returns if isinstance(returns, torch.Tensor) else torch.as_tensor(returns)
    sd = r.std()
    if sd < 1e-8:
        return 0.0
    return (r.mean() / sd).item()


def compute_max_drawdown(returns: np.ndarray) -> float:
    cum = np.cumprod(1 + returns)
    peak = np.maximum.accumulate(cum)
    return ((cum - peak) / peak).min()


def sharpe_np(returns: np.ndarray) -> float:
    """Ensemble-script Sharpe: numpy std (ddof=0), 0 when std < 1e-8."""
    sd = returns.std()
    if sd < 1e-8:
        return 0.0
    return returns.mean() / sd


def summary_statistics(r: np.ndarray) -> dict:
    """The paper-style table of `plots.plot_summary_statistics` (SDF factor returns)."""
    mu, sd = r.mean(), r.std()
    sr = mu / sd
    cum = np.cumprod(1 + r)
    peak = np.maximum.accumulate(cum)
    return {
        "mean": mu, "std": sd, "sharpe": sr, "sharpe_annual": sr * np.sqrt(12),
        "min": r.min(), "max": r.max(),
        "skew": ((r - mu) ** 3).mean() / sd ** 3,
        "kurtosis": ((r - mu) ** 4).mean() / sd ** 4 - 3,
        "cumulative_return": np.prod(1 + r) - 1,
        "max_drawdown": ((cum - peak) / peak).min(),
    }
