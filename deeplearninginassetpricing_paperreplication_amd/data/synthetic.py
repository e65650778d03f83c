"""Synthetic factor-model panels in the reference ``.npz`` schema.

Two generators share one statistical design (`/root/reference/src/generate_synthetic_data.py`):
5 AR(1) latent factors, positive market loadings, characteristics that are noisy proxies of
the loadings (the first ``min(2K, F//2)``) or pure noise, each cross-sectionally winsorised at
p5/p95 and z-scored, heteroskedastic idiosyncratic returns, 8 persistent macro series of which
the first three lead the factors, and random entry / exit / gap missingness with the −99.99
sentinel.

* ``generate_all_splits`` / ``generate_dataset`` consume numpy's legacy RandomState stream in
  the reference's order, so a given seed reproduces the reference's files bit-for-bit (the
  shipped ``data/synthetic_data`` is 120/30/60 × 500 stocks, seed 42) — but the hot T×F
  percentile loop is one vectorised call instead of T·F Python iterations.
* ``generate_panel_fast`` draws the same model with torch (CPU or GPU, float32, chunked over
  time) for the BASELINE scaled panels (600×30000×512 is 9.2 G values); it returns arrays in
  memory instead of writing npz files.
"""
from __future__ import annotations

import argparse
import os
from pathlib import Path
from typing import Dict, Optional, Tuple

import numpy as np

FACTOR_VOL_SCALE = (1.0, 0.6, 0.5, 0.7, 0.4)
MACRO_PERSISTENCE = (0.95, 0.90, 0.98, 0.85, 0.80, 0.92, 0.75, 0.70)


# --------------------------------------------------------------------------------------
# Reference-stream generator (numpy legacy RandomState, float64 like the reference)
# --------------------------------------------------------------------------------------
def _factor_returns(T: int, K: int, monthly_vol: float = 0.02, rho: float = 0.1) -> np.ndarray:
    vols = monthly_vol * np.array(FACTOR_VOL_SCALE)[:K]
    innov = np.random.randn(T * K).reshape(T, K) * vols
    f = np.zeros((T, K))
    for t in range(T):
        f[t] = innov[t] if t == 0 else rho * f[t - 1] + innov[t]
    return f


def _loadings(N: int, K: int) -> np.ndarray:
    b = np.random.randn(N, K)
    b[:, 0] = np.abs(b[:, 0]) + 0.5
    return b


def _standardize_xs(ch: np.ndarray) -> np.ndarray:
    """Winsorise at p5/p95 and z-score every (t, f) cross-section. ch: [T, N, F] float64."""
    v = np.ascontiguousarray(ch.transpose(0, 2, 1))           # [T, F, N] rows contiguous
    lo, hi = np.percentile(v, [5, 95], axis=2)
    v = np.clip(v, lo[..., None], hi[..., None])
    v = (v - v.mean(axis=2, keepdims=True)) / (v.std(axis=2, keepdims=True) + 1e-8)
    return v.transpose(0, 2, 1)


def _characteristics(T: int, N: int, F: int, loadings: np.ndarray, noise: float = 0.5) -> np.ndarray:
    K = loadings.shape[1]
    npred = min(2 * K, F // 2)
    per_t = npred * (N + 1) + N * (F - npred)
    ch = np.zeros((T, N, F))
    for t in range(T):
        z = np.random.randn(per_t)
        o = 0
        for i in range(npred):
            ch[t, :, i] = loadings[:, i % K] + z[o:o + N] * noise + z[o + N] * 0.1
            o += N + 1
        ch[t, :, npred:] = z[o:].reshape(N, F - npred)
    return _standardize_xs(ch)


def _returns(f: np.ndarray, b: np.ndarray, idio_vol: float = 0.08) -> np.ndarray:
    vols = idio_vol * (0.5 + np.random.rand(b.shape[0]))
    return f @ b.T + np.random.randn(f.shape[0], b.shape[0]) * vols


def _macro(T: int, M: int, f: Optional[np.ndarray]) -> np.ndarray:
    rho = MACRO_PERSISTENCE[:M]
    z = np.random.randn(M * T).reshape(M, T) * 0.1
    m = np.zeros((T, M))
    for i in range(M):
        for t in range(T):
            m[t, i] = z[i, t] if t == 0 else rho[i] * m[t - 1, i] + z[i, t]
    if f is not None:
        for i in range(min(3, M, f.shape[1])):
            m[1:, i] += 0.3 * f[:-1, i]
    return m


def _missing(T: int, N: int, avg_cov: float = 0.7, min_hist: int = 12) -> np.ndarray:
    mask = np.zeros((T, N), dtype=bool)
    rs = np.random
    for i in range(N):
        start = rs.randint(0, max(0, T - min_hist) + 1)
        end = rs.randint(min(T, start + min_hist), T + 1)
        mask[start:end, i] = True
        if end - start > 24:
            for _ in range(rs.randint(0, 3)):
                g = rs.randint(start + 6, end - 6)
                mask[g:min(g + rs.randint(1, 4), end), i] = False
    for t in range(T):
        have = mask[t].sum()
        if have / N < avg_cov * 0.5:
            miss = np.where(~mask[t])[0]
            n_add = int(N * avg_cov * 0.5 - have)
            if n_add > 0 and len(miss) > 0:
                mask[t, rs.choice(miss, min(n_add, len(miss)), replace=False)] = True
    return mask


def _dates(T: int, start: int) -> np.ndarray:
    y, m = divmod(start, 100)
    k = (m - 1) + np.arange(T)
    return (y + k // 12) * 100 + (k % 12) + 1


def _char_npz(ret, ch, mask, F, start) -> Dict[str, np.ndarray]:
    T, N = ret.shape
    data = np.empty((T, N, F + 1), dtype=np.float32)
    data[:, :, 0] = ret
    data[:, :, 1:] = ch
    data[~mask] = -99.99
    return {"data": data, "date": _dates(T, start),
            "variable": np.array(["RET"] + [f"char_{i + 1}" for i in range(F)])}


def _macro_npz(m, start) -> Dict[str, np.ndarray]:
    return {"data": m.astype(np.float32), "date": _dates(m.shape[0], start)}


def _draw_all(T: int, N: int, F: int, M: int, K: int = 5):
    f = _factor_returns(T, K)
    b = _loadings(N, K)
    r = _returns(f, b)
    ch = _characteristics(T, N, F, b)
    mac = _macro(T, M, f)
    mask = _missing(T, N)
    return r, ch, mac, mask


# ---- public building blocks under the reference's names / signatures ---------------------
def generate_factor_returns(n_periods: int, n_factors: int = 5, monthly_vol: float = 0.02,
                            factor_autocorr: float = 0.1) -> np.ndarray:
    return _factor_returns(n_periods, n_factors, monthly_vol, factor_autocorr)


def generate_factor_loadings(n_stocks: int, n_factors: int = 5, loading_vol: float = 1.0) -> np.ndarray:
    b = np.random.randn(n_stocks, n_factors) * loading_vol
    b[:, 0] = np.abs(b[:, 0]) + 0.5
    return b


def generate_characteristics(n_periods: int, n_stocks: int, n_features: int,
                             factor_loadings: np.ndarray, noise_level: float = 0.5) -> np.ndarray:
    return _characteristics(n_periods, n_stocks, n_features, factor_loadings, noise_level)


def generate_returns(factor_returns: np.ndarray, factor_loadings: np.ndarray,
                     idio_vol: float = 0.08) -> np.ndarray:
    return _returns(factor_returns, factor_loadings, idio_vol)


def generate_macro_features(n_periods: int, n_macro: int = 8,
                            factor_returns: Optional[np.ndarray] = None) -> np.ndarray:
    return _macro(n_periods, n_macro, factor_returns)


def generate_missing_pattern(n_periods: int, n_stocks: int, avg_coverage: float = 0.7,
                             min_history: int = 12) -> np.ndarray:
    return _missing(n_periods, n_stocks, avg_coverage, min_history)


def apply_missing_values(data: np.ndarray, mask: np.ndarray, missing_value: float = -99.99) -> np.ndarray:
    """Sentinel at invalid (t, i) entries of a [T, N] or [T, N, F] array (copy)."""
    out = np.array(data, copy=True)
    out[~np.asarray(mask, dtype=bool)] = missing_value
    return out


def create_individual_npz(returns: np.ndarray, characteristics: np.ndarray, mask: np.ndarray,
                          n_features: int, start_date: int = 196703) -> Dict[str, np.ndarray]:
    return _char_npz(returns, characteristics, mask, n_features, start_date)


def create_macro_npz(macro_features: np.ndarray, start_date: int = 196703) -> Dict[str, np.ndarray]:
    return _macro_npz(macro_features, start_date)


def generate_dataset(n_periods: int, n_stocks: int, n_features: int = 46, n_macro: int = 8,
                     n_factors: int = 5, seed: Optional[int] = None, start_date: int = 196703):
    """One split as (individual npz dict, macro npz dict)."""
    if seed is not None:
        np.random.seed(seed)
    f = _factor_returns(n_periods, n_factors)
    b = _loadings(n_stocks, n_factors)
    r = _returns(f, b)
    ch = _characteristics(n_periods, n_stocks, n_features, b)
    mac = _macro(n_periods, n_macro, f)
    mask = _missing(n_periods, n_stocks)
    return _char_npz(r, ch, mask, n_features, start_date), _macro_npz(mac, start_date)


def split_start_dates(n_train: int, n_valid: int) -> Tuple[int, int, int]:
    """Split start dates with the reference's calendar quirk (`generate_synthetic_data.py:504-508`):
    valid starts at 197703 + (T_train//12)*100, test at 198003 + ((T_train+T_valid)//12)*100."""
    return 196703, 197703 + (n_train // 12) * 100, 198003 + ((n_train + n_valid) // 12) * 100


def generate_all_splits(output_dir: str, n_periods_train: int = 120, n_periods_valid: int = 30,
                        n_periods_test: int = 60, n_stocks: int = 1000, n_features: int = 46,
                        n_macro: int = 8, seed: int = 42, quiet: bool = False):
    """Write ``char/Char_{split}.npz`` and ``macro/macro_{split}.npz`` (compressed)."""
    out = Path(output_dir)
    (out / "char").mkdir(parents=True, exist_ok=True)
    (out / "macro").mkdir(parents=True, exist_ok=True)
    T = n_periods_train + n_periods_valid + n_periods_test
    np.random.seed(seed)
    r, ch, mac, mask = _draw_all(T, n_stocks, n_features, n_macro)
    bounds = [0, n_periods_train, n_periods_train + n_periods_valid, T]
    for k, (name, start) in enumerate(zip(("train", "valid", "test"),
                                          split_start_dates(n_periods_train, n_periods_valid))):
        a, z = bounds[k], bounds[k + 1]
        np.savez_compressed(out / "char" / f"Char_{name}.npz",
                            **_char_npz(r[a:z], ch[a:z], mask[a:z], n_features, start))
        np.savez_compressed(out / "macro" / f"macro_{name}.npz", **_macro_npz(mac[a:z], start))
        if not quiet:
            print(f"  wrote {name}: T={z - a} N={n_stocks} F={n_features} M={n_macro}")
    return out


# --------------------------------------------------------------------------------------
# Fast generator (torch, float32, CPU or GPU) for the scaled BASELINE panels
# --------------------------------------------------------------------------------------
def _row_quantiles(x, qs):
    """Per-row quantiles with torch.quantile's default linear interpolation, via one sort:
    torch.quantile refuses inputs above 2^24 elements (a 16-period chunk of a 30000 x 512
    panel is 2.5e8), and sorting once serves both percentiles."""
    import torch
    n = x.shape[1]
    srt = torch.sort(x, dim=1).values
    out = []
    for q in qs:
        pos = q * (n - 1)
        lo = int(pos)
        hi = min(lo + 1, n - 1)
        frac = pos - lo
        out.append(torch.lerp(srt[:, lo], srt[:, hi], torch.full((), frac, device=x.device, dtype=x.dtype)))
    return torch.stack(out)


def generate_panel_fast(T: int, N: int, F: int, M: int, seed: int = 0, device: str = "cpu",
                        n_factors: int = 5, chunk: int = 16, return_latent: bool = False):
    """Return (returns [T,N] f32, features [T,N,F] f32, mask [T,N] bool, macro [T,M] f32).

    Same model as the reference generator; invalid entries are already zero-filled (the
    loader's view of the data).  Runs in ``chunk``-period slices so a 600×30000×512 panel
    needs only one output copy; on a GPU it takes seconds.

    ``return_latent``: also return the generator's hidden truth as a 5th element, a dict with the
    factor returns ``f`` [T,K], the loadings ``b`` [N,K], the idiosyncratic vols ``idio`` [N],
    the factor innovation vols ``vols`` [K] and the AR(1) coefficient ``rho`` (for the oracle
    Sharpe ceiling, ``analysis.oracle``). The draws are identical with and without it.
    """
    import torch
    g = torch.Generator(device=device).manual_seed(seed)
    dev = torch.device(device)
    K = n_factors
    vols = 0.02 * torch.tensor(FACTOR_VOL_SCALE[:K], device=dev)
    innov = torch.randn(T, K, generator=g, device=dev) * vols
    f = torch.zeros(T, K, device=dev)
    for t in range(T):
        f[t] = innov[t] if t == 0 else 0.1 * f[t - 1] + innov[t]
    b = torch.randn(N, K, generator=g, device=dev)
    b[:, 0] = b[:, 0].abs() + 0.5
    idio = 0.08 * (0.5 + torch.rand(N, generator=g, device=dev))
    ret = f @ b.T + torch.randn(T, N, generator=g, device=dev) * idio

    feats = torch.empty(T, N, F, device=dev)
    npred = min(2 * K, F // 2)
    sel = torch.arange(npred, device=dev) % K
    for a in range(0, T, chunk):
        z = min(T, a + chunk)
        c = torch.randn(z - a, N, F, generator=g, device=dev)
        c[:, :, :npred] = (b[:, sel][None] + c[:, :, :npred] * 0.5
                           + torch.randn(z - a, 1, npred, generator=g, device=dev) * 0.1)
        q = _row_quantiles(c.transpose(1, 2).reshape(-1, N), (0.05, 0.95))  # [2, (z-a)*F]
        lo = q[0].reshape(z - a, 1, F)
        hi = q[1].reshape(z - a, 1, F)
        c = torch.minimum(torch.maximum(c, lo), hi)
        c = (c - c.mean(1, keepdim=True)) / (c.std(1, unbiased=False, keepdim=True) + 1e-8)
        feats[a:z] = c

    rho = torch.tensor((MACRO_PERSISTENCE * ((M + 7) // 8))[:M], device=dev)
    zm = torch.randn(T, M, generator=g, device=dev) * 0.1
    mac = torch.zeros(T, M, device=dev)
    for t in range(T):
        mac[t] = zm[t] if t == 0 else rho * mac[t - 1] + zm[t]
    k3 = min(3, M, K)
    mac[1:, :k3] += 0.3 * f[:-1, :k3]

    # entry/exit + gaps: vectorised draw of the same pattern family.
    max_start = max(0, T - 12)
    start = torch.randint(0, max_start + 1, (N,), generator=g, device=dev)
    lo_end = torch.clamp(start + 12, max=T)
    end = lo_end + (torch.rand(N, generator=g, device=dev) * (T + 1 - lo_end).float()).long()
    tt = torch.arange(T, device=dev)[:, None]
    mask = (tt >= start[None]) & (tt < end[None])
    for _ in range(2):
        has = (end - start) > 24
        gs = start + 6 + (torch.rand(N, generator=g, device=dev) * (end - start - 12).clamp(min=1).float()).long()
        gl = torch.randint(1, 4, (N,), generator=g, device=dev)
        take = has & (torch.rand(N, generator=g, device=dev) < 0.5)
        gap = (tt >= gs[None]) & (tt < (gs + gl)[None]) & take[None]
        mask &= ~gap
    cov = mask.float().mean(1)
    low = cov < 0.35
    if bool(low.any()):
        extra = torch.rand(T, N, generator=g, device=dev) < (0.35 - cov).clamp(min=0)[:, None] / (1 - cov).clamp(min=1e-6)[:, None]
        mask |= extra & low[:, None]
    ret = torch.where(mask, ret, torch.zeros((), device=dev))
    feats.mul_(mask[:, :, None])
    if return_latent:
        latent = {"f": f, "b": b, "idio": idio, "vols": vols, "rho": 0.1}
        return ret.float(), feats, mask, mac.float(), latent
    return ret.float(), feats, mask, mac.float()


def main(argv=None):
    p = argparse.ArgumentParser(description="Generate synthetic data for Deep Learning Asset Pricing")
    p.add_argument("--output_dir", type=str, default="./synthetic_data")
    p.add_argument("--n_periods_train", type=int, default=120)
    p.add_argument("--n_periods_valid", type=int, default=30)
    p.add_argument("--n_periods_test", type=int, default=60)
    p.add_argument("--n_stocks", type=int, default=1000)
    p.add_argument("--n_features", type=int, default=46)
    p.add_argument("--n_macro", type=int, default=8)
    p.add_argument("--seed", type=int, default=42)
    a = p.parse_args(argv)
    generate_all_splits(a.output_dir, a.n_periods_train, a.n_periods_valid, a.n_periods_test,
                        a.n_stocks, a.n_features, a.n_macro, a.seed)
    print(f"Synthetic data written to {os.path.abspath(a.output_dir)}")


if __name__ == "__main__":
    main()
