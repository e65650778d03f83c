"""Paper figures from trained checkpoints (`/root/reference/src/plots.py` behaviour).

Five outputs, same file names and CLI (``--data_dir --checkpoint_dirs ... --output_dir``):
  cumulative_sdf.png      ensemble-mean portfolio return, negated (paper SDF factor),
                          compounded, with train / valid / test shading (Figure 1)
  training_curves.png     history.npz loss (log) and paper-sign Sharpe, phase markers
  sharpe_comparison.png   individual / mean / ensemble test Sharpe vs the paper's 0.75
  monthly_returns.png     histogram + time series of the test SDF factor
  summary_statistics.png  Table-2 style statistics of the ensemble SDF factor (test)

The reference hard-codes the calendar (March 1967 start, test from 1992) and the phase
boundaries (256 / 320); those are the defaults here and can be overridden by keyword.
All numbers come from ``analysis.portfolio`` (vectorised, no per-period loops); model weights
come from ``analysis.ensemble`` (batched native engine when ``device='cuda'``).
"""
from __future__ import annotations

import argparse
import os
from datetime import datetime
from typing import Dict, List, Sequence

import matplotlib

matplotlib.use("Agg")
import matplotlib.dates as mdates  # noqa: E402
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402

from ..data.dataset import load_splits  # noqa: E402
from . import portfolio as pf  # noqa: E402
from .ensemble import SPLITS, get_weights_from_model, load_model, weights_batched_gpu  # noqa: E402

STYLE = {"figure.figsize": (10, 6), "font.size": 12, "axes.labelsize": 12, "axes.titlesize": 14,
         "legend.fontsize": 10, "lines.linewidth": 1.5}
plt.rcParams.update(STYLE)


def month_range(start_year: int = 1967, n: int = 600, start_month: int = 3) -> List[datetime]:
    """First-of-month dates, ``n`` consecutive months from (start_year, start_month)."""
    k0 = start_year * 12 + start_month - 1
    return [datetime((k0 + i) // 12, (k0 + i) % 12 + 1, 1) for i in range(n)]


get_date_range = month_range   # reference name


class _Panel:
    """Split batches + per-model normalised weights, computed once per figure set."""

    def __init__(self, checkpoint_dirs: Sequence[str], data_dir: str, device: str = "cpu"):
        ds = load_splits(data_dir)
        self.batches = {s: d.get_full_batch() for s, d in zip(SPLITS, ds)}
        self.np = {s: {"returns": b["returns"].numpy(), "mask": b["mask"].numpy()}
                   for s, b in self.batches.items()}
        models = [load_model(d, "cpu")[0] for d in checkpoint_dirs]
        if str(device).startswith("cuda"):
            wdev = weights_batched_gpu(models, self.batches)
            self.weights = [{s: wdev[s][i].cpu().numpy() for s in SPLITS} for i in range(len(models))]
        else:
            self.weights = [{s: get_weights_from_model(m, self.batches[s]) for s in SPLITS} for m in models]

    def model_returns(self, split: str) -> np.ndarray:
        b = self.np[split]
        return np.stack([pf.portfolio_returns(w[split], b["returns"], b["mask"]) for w in self.weights])

    def ensemble_factor(self, split: str) -> np.ndarray:
        b = self.np[split]
        avg = pf.average_weights([w[split] for w in self.weights], b["mask"])
        return -pf.portfolio_returns(avg, b["returns"], b["mask"])


def _save(fig, save_path):
    fig.tight_layout()
    if save_path:
        fig.savefig(save_path, dpi=150, bbox_inches="tight")
        print(f"Saved: {save_path}")


def plot_cumulative_sdf(checkpoint_dirs, data_dir, save_path=None, n_train=240, n_valid=60,
                        panel: _Panel = None, start_year=1967):
    panel = panel or _Panel(checkpoint_dirs, data_dir)
    mean_ret = np.concatenate([panel.model_returns(s).mean(axis=0) for s in SPLITS])
    growth = np.cumprod(1.0 - mean_ret)
    dates = month_range(start_year, len(growth))
    fig, ax = plt.subplots(figsize=(12, 6))
    ax.plot(dates, growth, "b-", linewidth=1.5, label="GAN SDF")
    cut1 = dates[min(n_train, len(dates)) - 1]
    cut2 = dates[min(n_train + n_valid, len(dates)) - 1]
    ax.axvline(cut1, color="gray", linestyle="--", alpha=0.7, label="Train/Valid")
    ax.axvline(cut2, color="gray", linestyle=":", alpha=0.7, label="Valid/Test")
    for (a, b, c, lab) in ((dates[0], cut1, "blue", "Training"), (cut1, cut2, "green", "Validation"),
                           (cut2, dates[-1], "red", "Test")):
        ax.axvspan(a, b, alpha=0.1, color=c, label=lab)
    ax.set(xlabel="Date", ylabel="Cumulative Return", title="Cumulative SDF Returns (Ensemble)")
    ax.legend(loc="upper left")
    ax.grid(True, alpha=0.3)
    ax.xaxis.set_major_locator(mdates.YearLocator(5))
    ax.xaxis.set_major_formatter(mdates.DateFormatter("%Y"))
    _save(fig, save_path)
    return fig, ax


def plot_training_curves(checkpoint_dir, save_path=None, phase_marks=(256, 320)):
    with np.load(os.path.join(checkpoint_dir, "history.npz"), allow_pickle=False) as h:
        hist = {k: h[k] for k in h.files}
    ep = np.arange(1, len(hist["train_loss"]) + 1)
    fig, (a1, a2) = plt.subplots(1, 2, figsize=(14, 5))
    a1.plot(ep, hist["train_loss"], "b-", label="Train", alpha=0.8)
    a1.plot(ep, hist["valid_loss"], "g-", label="Valid", alpha=0.8)
    a1.set(xlabel="Epoch", ylabel="Loss", title="Training Loss", yscale="log")
    for key, col, lab in (("train_sharpe", "b-", "Train"), ("valid_sharpe", "g-", "Valid"),
                          ("test_sharpe", "r-", "Test")):
        if key in hist:
            a2.plot(ep, -np.asarray(hist[key]), col, label=lab, alpha=0.8)
    a2.set(xlabel="Epoch", ylabel="Sharpe Ratio (Monthly)", title="Sharpe Ratio During Training")
    for a in (a1, a2):
        a.legend()
        a.grid(True, alpha=0.3)
        for x in phase_marks:
            a.axvline(x, color="gray", linestyle="--", alpha=0.5)
    _save(fig, save_path)
    return fig, (a1, a2)


def plot_sharpe_comparison(checkpoint_dirs, data_dir, save_path=None, panel: _Panel = None):
    panel = panel or _Panel(checkpoint_dirs, data_dir)
    ind = [pf.sharpe_ddof0(-r) for r in panel.model_returns("test")]
    ens = pf.sharpe_ddof0(panel.ensemble_factor("test"))
    vals = ind + [float(np.mean(ind)), ens]
    labels = [f"Model {i + 1}" for i in range(len(ind))] + ["Mean", "Ensemble"]
    fig, ax = plt.subplots(figsize=(12, 6))
    x = np.arange(len(vals))
    bars = ax.bar(x, vals, color=["steelblue"] * len(ind) + ["forestgreen", "darkred"], alpha=0.8,
                  edgecolor="black")
    ax.axhline(pf.PAPER_TEST_SHARPE, color="red", linestyle="--", linewidth=2,
               label=f"Paper ({pf.PAPER_TEST_SHARPE})")
    ax.set_xticks(x)
    ax.set_xticklabels(labels, rotation=45, ha="right")
    ax.set(ylabel="Test Sharpe Ratio (Monthly)", title="Individual vs Ensemble Sharpe Ratio")
    ax.legend()
    ax.grid(True, alpha=0.3, axis="y")
    for b, v in zip(bars, vals):
        ax.text(b.get_x() + b.get_width() / 2, b.get_height() + 0.01, f"{v:.3f}", ha="center",
                va="bottom", fontsize=9)
    _save(fig, save_path)
    return fig, ax


def plot_monthly_returns(checkpoint_dirs, data_dir, save_path=None, panel: _Panel = None,
                         test_start_year=1992):
    panel = panel or _Panel(checkpoint_dirs, data_dir)
    f = -panel.model_returns("test").mean(axis=0)
    fig, (a1, a2) = plt.subplots(1, 2, figsize=(14, 5))
    a1.hist(f, bins=30, density=True, alpha=0.7, color="steelblue", edgecolor="black")
    a1.axvline(f.mean(), color="red", linestyle="--", label=f"Mean: {f.mean():.4f}")
    a1.axvline(0, color="black", alpha=0.5)
    a1.set(xlabel="Monthly Return", ylabel="Density", title="Distribution of Monthly SDF Returns (Test)")
    a1.legend()
    dates = month_range(test_start_year, len(f))
    a2.plot(dates, f, "b-", alpha=0.7, linewidth=1)
    a2.axhline(0, color="black", alpha=0.5)
    a2.fill_between(dates, f, 0, where=f > 0, alpha=0.3, color="green")
    a2.fill_between(dates, f, 0, where=f < 0, alpha=0.3, color="red")
    a2.set(xlabel="Date", ylabel="Monthly Return", title="Monthly SDF Returns Over Time (Test)")
    a2.xaxis.set_major_locator(mdates.YearLocator(5))
    a2.xaxis.set_major_formatter(mdates.DateFormatter("%Y"))
    for a in (a1, a2):
        a.grid(True, alpha=0.3)
    _save(fig, save_path)
    return fig, (a1, a2)


def summary_rows(stats: Dict[str, float]) -> List[List[str]]:
    s = stats
    return [["Mean (Monthly)", f"{s['mean']:.4f}"], ["Std (Monthly)", f"{s['std']:.4f}"],
            ["Sharpe (Monthly)", f"{s['sharpe']:.4f}"], ["Sharpe (Annual)", f"{s['sharpe_annual']:.2f}"],
            ["Min", f"{s['min']:.4f}"], ["Max", f"{s['max']:.4f}"], ["Skewness", f"{s['skew']:.2f}"],
            ["Kurtosis", f"{s['kurtosis']:.2f}"], ["Cumulative Return", f"{s['cumulative_return']:.2%}"],
            ["Max Drawdown", f"{s['max_drawdown']:.2%}"], ["", ""],
            ["Paper Sharpe (Monthly)", f"{pf.PAPER_TEST_SHARPE}"],
            ["Our Sharpe / Paper", f"{s['sharpe'] / pf.PAPER_TEST_SHARPE:.1%}"]]


def plot_summary_statistics(checkpoint_dirs, data_dir, save_path=None, panel: _Panel = None):
    panel = panel or _Panel(checkpoint_dirs, data_dir)
    stats = pf.sdf_statistics(panel.ensemble_factor("test"))
    fig, ax = plt.subplots(figsize=(10, 6))
    ax.axis("off")
    tab = ax.table(cellText=summary_rows(stats), colLabels=["Metric", "Value"], loc="center",
                   cellLoc="center", colWidths=[0.4, 0.3])
    tab.auto_set_font_size(False)
    tab.set_fontsize(12)
    tab.scale(1.2, 1.8)
    for i in range(2):
        tab[(0, i)].set_facecolor("#4472C4")
        tab[(0, i)].set_text_props(color="white", fontweight="bold")
    ax.set_title("Summary Statistics - Test Period (1992-2016)", fontsize=14, fontweight="bold", pad=20)
    _save(fig, save_path)
    return fig, ax


def generate_all_plots(checkpoint_dirs, data_dir, output_dir="./plots", device: str = "cpu"):
    os.makedirs(output_dir, exist_ok=True)
    print("Generating plots...")
    print("=" * 50)
    panel = _Panel(checkpoint_dirs, data_dir, device)
    jobs = [
        ("Cumulative SDF Returns", "cumulative_sdf.png",
         lambda p: plot_cumulative_sdf(checkpoint_dirs, data_dir, p, panel=panel)),
        ("Training Curves", "training_curves.png", lambda p: plot_training_curves(checkpoint_dirs[0], p)),
        ("Sharpe Comparison", "sharpe_comparison.png",
         lambda p: plot_sharpe_comparison(checkpoint_dirs, data_dir, p, panel=panel)),
        ("Monthly Returns Distribution", "monthly_returns.png",
         lambda p: plot_monthly_returns(checkpoint_dirs, data_dir, p, panel=panel)),
        ("Summary Statistics", "summary_statistics.png",
         lambda p: plot_summary_statistics(checkpoint_dirs, data_dir, p, panel=panel)),
    ]
    for i, (title, fname, fn) in enumerate(jobs, 1):
        print(f"\n{i}. {title}...")
        fn(os.path.join(output_dir, fname))
    print("\n" + "=" * 50)
    print(f"All plots saved to: {output_dir}")
    plt.close("all")


def main(argv=None):
    p = argparse.ArgumentParser(description="Generate paper plots")
    p.add_argument("--data_dir", type=str, required=True, help="Path to data directory")
    p.add_argument("--checkpoint_dirs", type=str, nargs="+", required=True,
                   help="Paths to checkpoint directories")
    p.add_argument("--output_dir", type=str, default="./plots", help="Output directory for plots")
    p.add_argument("--device", type=str, default="cpu")
    a = p.parse_args(argv)
    generate_all_plots(a.checkpoint_dirs, a.data_dir, a.output_dir, a.device)


if __name__ == "__main__":
    main()
