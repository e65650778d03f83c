"""Paper metrics added on top of the reference (EV, XS-R², turnover, max 1-month loss)."""
import numpy as np

from deeplearninginassetpricing_paperreplication_amd.analysis.portfolio import (
    cross_sectional_r2, explained_variation, paper_metrics, turnover)


def _panel(T=24, N=30, seed=0):
    rng = np.random.default_rng(seed)
    mask = rng.random((T, N)) > 0.3
    w = rng.standard_normal((T, N)) * mask
    return w, mask, rng


def test_returns_spanned_by_the_weights_are_fully_explained():
    w, mask, rng = _panel()
    R = (w * rng.standard_normal((w.shape[0], 1))) * mask          # R_t = f_t w_t
    assert abs(explained_variation(w, R, mask) - 1.0) < 1e-12
    assert abs(cross_sectional_r2(w, R, mask) - 1.0) < 1e-12


def test_orthogonal_returns_explain_nothing_and_metric_ranges():
    w, mask, rng = _panel(seed=1)
    R = rng.standard_normal(w.shape) * 0.1 * mask
    ev = explained_variation(w, R, mask)
    assert -1e-9 <= ev < 0.2                                       # projection R² is >= 0
    m = paper_metrics(w / np.abs(w).sum(1, keepdims=True), R, mask)
    assert set(m) == {"sharpe", "ev", "xs_r2", "turnover", "max_1m_loss_std"}
    assert m["turnover"] > 0 and m["max_1m_loss_std"] > 0


def test_buy_and_hold_has_zero_turnover():
    T, N = 10, 5
    mask = np.ones((T, N), bool)
    R = np.full((T, N), 0.01)
    w0 = np.full(N, 1.0 / N)
    w = np.stack([w0 * (1.01 ** t) / (1.01 ** t) for t in range(T)])  # drifts with equal returns
    assert turnover(w, R, mask) < 1e-12
