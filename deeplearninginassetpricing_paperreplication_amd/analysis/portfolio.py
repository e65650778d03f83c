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
