"""Oracle Sharpe yardsticks of the synthetic factor-model panel (an addition; the reference has no
such yardstick, and its 0.55-0.75 test Sharpe target refers to the real data,
`/root/reference/notebooks/demo_full.ipynb:867`).

The generator (`/root/reference/src/generate_synthetic_data.py:26-169`, ``data.synthetic``) draws
returns ``R_t = f_t b^T + e_t`` with K = 5 zero-mean AR(1) factors
``f_t = rho f_{t-1} + u_t`` (rho = 0.1, u_tk ~ N(0, sigma_k^2)), loadings ``b`` and independent
idiosyncratic noise. Every expected return is zero unconditionally, so the only priced
information is the one-month factor persistence (the macro series carry 0.3 f_{t-1} for the
first three factors). The conditional mean-variance optimal SDF portfolio therefore times the
factors: at t it holds ``a_tk = rho f_{t-1,k} / sigma_k^2`` units of factor k, earning
``x_t = sum_k a_tk f_tk``. Its population Sharpe ratio (monthly) is

    SR_k^2 = E[x_k]^2 / Var(x_k) = rho^2 / (1 - rho^2) / (1 + 2 rho^2 / (1 - rho^2)),
    SR*    = sqrt(K) SR_k  (independent factors)  = 0.2225 at rho = 0.1, K = 5,

independent of the factor volatilities. This is the *conditional mean-variance oracle*, not an
upper bound on the unconditional Sharpe: weights mu_t / sigma^2 maximise each month's conditional
Sharpe, while the unconditionally efficient managed portfolio holds mu_t / (sigma^2 + mu_t^2) and
reaches (Hansen-Richard / Ferson-Siegel bound, ``unconditional_bound``)

    SR_u^2 = E[S_t^2 / (1 + S_t^2)] / (1 - E[S_t^2 / (1 + S_t^2)]),   S_t^2 = q chi^2_K,

slightly above SR* (0.2226 vs 0.2225 at rho = 0.1, K = 5), so ``fraction_of_population`` may
exceed 1 without a bug. Finite test windows scatter around both (the standard error of a monthly
Sharpe over T periods is about 1 / sqrt(T): 0.058 on the 300-month test split).

``oracle_report`` also evaluates on the generated panel (paper sign: the SDF factor return):
  * ``true_signal``       a_tk from the true f_{t-1} and the true factor returns f_t;
  * ``tradable``          a realisable portfolio: the factor-mimicking portfolios of the valid
                          stocks (cross-sectional regression on the true loadings) priced with
                          last month's *estimated* factor returns -- past returns and the true
                          loadings only;
  * ``macro_signal``      the first three factors timed by a linear predictor of f_tk from the
                          observed macro series k fitted on the train split (information the
                          GAN's macro LSTM sees), mimicking portfolios as above.

What the GAN can reach: its SDF weights at t are a function of that month's characteristics
(noisy proxies of the static loadings) and the macro history; lagged returns, which reveal
f_{t-1}, are not inputs. Its attainable timing signal is the macro channel, where 0.3 f_{t-1}
(sd ~0.006) sits under persistent AR noise of sd ~0.3, so ``macro_signal`` is close to zero; any
static factor exposure has a population Sharpe of zero and a sampling standard error of
1/sqrt(T) (``test_se``). The ceilings bound every SDF; the SE sizes the noise of a realised test
Sharpe.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import numpy as np


def population_sharpe(rho: float = 0.1, K: int = 5) -> float:
    """Population monthly Sharpe of the conditional mean-variance factor-timing SDF."""
    q = rho * rho / (1.0 - rho * rho)            # = E[x_k] / Var-scale, see module docstring
    return math.sqrt(K) * math.sqrt(q / (1.0 + 2.0 * q))


def unconditional_bound(rho: float = 0.1, K: int = 5) -> float:
    """Population Sharpe of the unconditionally efficient managed portfolio (the maximum over all
    strategies using f_{t-1}): sqrt(E[s/(1+s)] / (1 - E[s/(1+s)])) with s = q chi^2_K the squared
    conditional Sharpe, integrated against the chi^2_K density."""
    from scipy import integrate, stats
    q = rho * rho / (1.0 - rho * rho)
    e = integrate.quad(lambda x: q * x / (1.0 + q * x) * stats.chi2.pdf(x, K), 0.0, np.inf)[0]
    return math.sqrt(e / (1.0 - e))


def _sharpe(x: np.ndarray) -> float:
    x = np.asarray(x, np.float64)
    sd = x.std()
    return float(x.mean() / sd) if sd > 1e-12 else 0.0


def _mimicking(ret: np.ndarray, mask: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Per-period factor-mimicking portfolio returns f_hat [T, K]: OLS of the valid stocks'
    returns on their loadings."""
    T, K = ret.shape[0], b.shape[1]
    out = np.zeros((T, K))
    for t in range(T):
        v = mask[t]
        if v.sum() <= K:
            continue
        B = b[v]
        out[t] = np.linalg.lstsq(B, ret[t, v], rcond=None)[0]
    return out


def oracle_report(ret, mask, macro, latent: Dict, cuts: Sequence[int]) -> Dict:
    """Oracle Sharpe ratios on a generated panel. ``ret``/``mask`` [T, N], ``macro`` [T, M]
    (raw, as generated), ``latent`` from ``generate_panel_fast(..., return_latent=True)``,
    ``cuts`` = (T_train, T_valid, T_test)."""
    f = np.asarray(latent["f"], np.float64)
    b = np.asarray(latent["b"], np.float64)
    vols = np.asarray(latent["vols"], np.float64)
    rho = float(latent["rho"])
    ret = np.asarray(ret, np.float64)
    mask = np.asarray(mask, bool)
    macro = np.asarray(macro, np.float64)
    T, K = f.shape
    a = np.zeros_like(f)
    a[1:] = rho * f[:-1] / vols ** 2
    x_true = (a * f).sum(1)
    fh = _mimicking(ret, mask, b)
    ah = np.zeros_like(fh)
    ah[1:] = rho * fh[:-1] / vols ** 2
    x_trad = (ah * fh).sum(1)
    # macro predictor of the first three factors, fitted on the train split: OLS of f_tk on the
    # macro series k that the generator feeds 0.3 f_{t-1,k} into, without an intercept (oracle
    # knowledge: which series matters, and that the factors have mean zero -- an intercept fits
    # the train window's sample mean; all M series overfit the 240 train months)
    t0 = int(cuts[0])
    k3 = min(3, K, macro.shape[1])
    am = np.zeros((T, K))
    for k in range(k3):
        m = macro[:, k]
        coef = float(m[:t0] @ f[:t0, k]) / max(float(m[:t0] @ m[:t0]), 1e-30)
        am[:, k] = coef * m / vols[k] ** 2
    x_mac = (am * fh).sum(1)
    bounds = np.cumsum([0] + list(cuts))
    out = {"population": population_sharpe(rho, K), "unconditional_bound": unconditional_bound(rho, K),
           "rho": rho, "K": K,
           "test_se": 1.0 / math.sqrt(max(int(cuts[2]), 1))}
    for name, x in (("true_signal", x_true), ("tradable", x_trad), ("macro_signal", x_mac)):
        out[name] = {sp: _sharpe(x[bounds[i]:bounds[i + 1]][1 if i == 0 else 0:])
                     for i, sp in enumerate(("train", "valid", "test"))}
    return out


def oracle_for_panel(T_split=(240, 60, 300), N=3000, F=46, M=178, seed: int = 0,
                     device: str = "cpu", ensemble_test_sharpe: Optional[float] = None) -> Dict:
    """Oracle report of the panel ``bench.make_panel`` / ``generate_panel_fast`` draws for
    ``seed``; with ``ensemble_test_sharpe``, also the fraction of the conditional-MV oracle it reaches (may exceed 1: the
    oracle is not an upper bound, see ``unconditional_bound``)."""
    from ..data.synthetic import generate_panel_fast
    ret, _, mask, mac, lat = generate_panel_fast(sum(T_split), N, F, M, seed=seed, device=device,
                                                 return_latent=True)
    lat = {k: (v.detach().cpu().numpy() if hasattr(v, "detach") else v) for k, v in lat.items()}
    rep = oracle_report(ret.cpu().numpy(), mask.cpu().numpy(), mac.cpu().numpy(), lat, T_split)
    rep["panel"] = {"T": list(T_split), "N": N, "F": F, "M": M, "seed": seed}
    if ensemble_test_sharpe is not None:
        rep["ensemble_test_sharpe"] = float(ensemble_test_sharpe)
        rep["fraction_of_population"] = float(ensemble_test_sharpe) / rep["population"]
        rep["fraction_of_unconditional_bound"] = float(ensemble_test_sharpe) / rep["unconditional_bound"]
        rep["fraction_of_true_signal_test"] = float(ensemble_test_sharpe) / rep["true_signal"]["test"]
    return rep
