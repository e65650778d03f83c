"""Non-finite detection (an addition: the reference has no NaN guard, a NaN loss propagates
silently into ``compute_sharpe``, `/root/reference/src/train.py:29-34`).

The GPU engine writes one history row per epoch on the device (train loss, gradient norm,
valid/test metrics). The host reads the rows only at print boundaries, where it already
synchronises, so the check costs nothing per epoch. Policies:

  * ``"warn"`` (default): report the first non-finite epoch of each model once, keep going —
    the reference behaviour plus a message;
  * ``"raise"``: raise ``NonFiniteError`` (single-model runs that should stop early);
  * ``"ignore"``: no check.

Batched runs (ensembles / sweep buckets) never raise for one member: the members are reported
through ``nonfinite_models`` so drivers can mark them failed without losing the others.
"""
from __future__ import annotations

import warnings
from typing import Dict, List, Optional, Sequence

import numpy as np

POLICIES = ("warn", "raise", "ignore")


class NonFiniteError(FloatingPointError):
    def __init__(self, model: int, epoch: int, field: str):
        super().__init__(f"model {model}: non-finite {field} at epoch {epoch + 1}")
        self.model, self.epoch, self.field = model, epoch, field


def first_nonfinite(rows: np.ndarray, cols: Dict[str, int], start: int = 0) -> Optional[tuple]:
    """(epoch, field) of the first row >= ``start`` with a non-finite train loss or gradient
    norm, or None. Rows of phase 2 have no gradient-norm of the SDF but are checked alike."""
    if rows.shape[0] <= start:
        return None
    sub = rows[start:]
    for name in ("train_loss", "grad_norm"):
        bad = ~np.isfinite(sub[:, cols[name]])
        if bad.any():
            return start + int(np.argmax(bad)), name
    return None


class NonFiniteMonitor:
    def __init__(self, n_models: int, cols: Dict[str, int], policy: str = "warn"):
        if policy not in POLICIES:
            raise ValueError(f"nan_policy must be one of {POLICIES}")
        self.policy, self.cols = policy, cols
        self.checked = [0] * n_models
        self.bad: Dict[int, tuple] = {}

    def check(self, g: int, rows: np.ndarray, raise_ok: bool = True):
        if self.policy == "ignore" or g in self.bad:
            self.checked[g] = rows.shape[0]
            return
        hit = first_nonfinite(rows, self.cols, self.checked[g])
        self.checked[g] = rows.shape[0]
        if hit is None:
            return
        self.bad[g] = hit
        if self.policy == "raise" and raise_ok:
            raise NonFiniteError(g, *hit)
        warnings.warn(f"model {g}: non-finite {hit[1]} first at epoch {hit[0] + 1}", RuntimeWarning)

    @property
    def nonfinite_models(self) -> List[int]:
        return sorted(self.bad)
