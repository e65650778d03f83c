"""``python -m src.train`` command line (flags and defaults of `/root/reference/src/train.py:429-605`).

Additions (never changing reference defaults): ``--device``, ``--precision``,
``--selection_sign``, ``--resume`` (continue from ``save_dir/resume.pt``, which every run
writes at print boundaries and phase ends), ``--nan_policy``.
"""
from __future__ import annotations

import argparse
import json
import os
import random
from pathlib import Path

import numpy as np
import torch

from ..config import default_cli_config
from ..data.dataset import AssetPricingDataset, create_small_sample
from .trainer import save_history, train_3phase


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Train Asset Pricing GAN (Original Paper Setup)")
    p.add_argument("--config", type=str, help="Path to config JSON")
    p.add_argument("--data_dir", type=str, required=True, help="Path to data directory")
    p.add_argument("--save_dir", type=str, default="./checkpoints")
    p.add_argument("--epochs_unc", type=int, default=256)
    p.add_argument("--epochs_moment", type=int, default=64)
    p.add_argument("--epochs", type=int, default=1024)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--print_freq", type=int, default=128)
    p.add_argument("--ignore_epoch", type=int, default=64)
    p.add_argument("--save_best_freq", type=int, default=128)
    p.add_argument("--small_sample", action="store_true")
    p.add_argument("--n_periods", type=int, default=100)
    p.add_argument("--n_stocks", type=int, default=500)
    p.add_argument("--use_lstm", action="store_true", default=True)
    p.add_argument("--no_lstm", action="store_false", dest="use_lstm")
    p.add_argument("--hidden_dim", type=int, nargs="+", default=[64, 64])
    p.add_argument("--rnn_dim", type=int, nargs="+", default=[4])
    p.add_argument("--num_moments", type=int, default=8)
    p.add_argument("--dropout", type=float, default=0.05)
    p.add_argument("--hidden_dim_moment", type=int, nargs="+", default=[])
    p.add_argument("--rnn_dim_moment", type=int, nargs="+", default=[32])
    p.add_argument("--seed", type=int, default=42)
    # additions
    p.add_argument("--device", type=str, default=None, help="cpu | cuda[:k] (default: auto)")
    p.add_argument("--precision", type=str, default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--selection_sign", type=float, default=1.0,
                   help="+1: reference (un-negated Sharpe); -1: paper sign")
    p.add_argument("--resume", action="store_true",
                   help="continue an interrupted run from save_dir/resume.pt")
    p.add_argument("--nan_policy", type=str, default="warn", choices=["warn", "raise", "ignore"],
                   help="non-finite train loss / grad norm handling")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    random.seed(args.seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(args.seed)
    os.makedirs(args.save_dir, exist_ok=True)
    d = Path(args.data_dir)
    print("=" * 70 + "\nDeep Learning Asset Pricing - MI355X engine\n" + "=" * 70 + "\n\nLoading data...")
    tr = AssetPricingDataset(str(d / "char" / "Char_train.npz"), str(d / "macro" / "macro_train.npz"))
    mu, sd = tr.get_macro_stats()
    va = AssetPricingDataset(str(d / "char" / "Char_valid.npz"), str(d / "macro" / "macro_valid.npz"),
                             mean_macro=mu, std_macro=sd)
    te = AssetPricingDataset(str(d / "char" / "Char_test.npz"), str(d / "macro" / "macro_test.npz"),
                             mean_macro=mu, std_macro=sd)
    if args.small_sample:
        print(f"Using small sample: {args.n_periods} periods, {args.n_stocks} stocks")
        trd = create_small_sample(tr, args.n_periods, args.n_stocks)
        vad = create_small_sample(va, min(args.n_periods, va.T), args.n_stocks)
        ted = create_small_sample(te, min(args.n_periods, te.T), args.n_stocks)
    else:
        print("Using FULL dataset")
        trd, vad, ted = tr.get_full_batch(), va.get_full_batch(), te.get_full_batch()
    print("\nData shapes:")
    for name, b in (("Train", trd), ("Valid", vad), ("Test ", ted)):
        print(f"  {name}: {b['returns'].shape[0]} periods x {b['returns'].shape[1]} stocks")
    print(f"  Individual features: {tr.individual_feature_dim}\n  Macro features: {tr.macro_feature_dim}")

    if args.config:
        with open(args.config) as f:
            config = json.load(f)
    else:
        config = default_cli_config(tr.macro_feature_dim, tr.individual_feature_dim,
                                    args.hidden_dim, args.use_lstm, args.rnn_dim, args.num_moments,
                                    args.dropout, args.hidden_dim_moment, args.rnn_dim_moment)
    print("\nModel Configuration (matching paper):")
    print(f"  SDF hidden dims: {config['hidden_dim']}")
    print(f"  SDF LSTM: {config['use_rnn']} with units {config.get('num_units_rnn', [])}")
    print(f"  Moment hidden dims: {config['hidden_dim_moment']}")
    print(f"  Moment LSTM: {config.get('use_rnn_moment', False)} with units {config.get('num_units_rnn_moment', [])}")
    print(f"  Num moments: {config['num_condition_moment']}")
    print(f"  Dropout: {config['dropout']} (keep prob: {1 - config['dropout']:.2f})")
    print(f"\nTraining Configuration:\n  Phase 1 (unconditional): {args.epochs_unc} epochs\n"
          f"  Phase 2 (moment update): {args.epochs_moment} epochs\n  Phase 3 (conditional): {args.epochs} epochs\n"
          f"  Learning rate: {args.lr}\n  Random seed: {args.seed}")
    with open(os.path.join(args.save_dir, "config.json"), "w") as f:
        json.dump(config, f, indent=2)
    print("\n" + "=" * 70 + "\nStarting 3-Phase GAN Training\n" + "=" * 70)
    device = torch.device(args.device) if args.device else None
    model, history = train_3phase(config, trd, vad, ted, device=device,
                                  num_epochs_unc=args.epochs_unc, num_epochs_moment=args.epochs_moment,
                                  num_epochs=args.epochs, lr=args.lr, print_freq=args.print_freq,
                                  save_dir=args.save_dir, ignore_epoch=args.ignore_epoch,
                                  save_best_freq=args.save_best_freq, seed=args.seed,
                                  precision=args.precision, selection_sign=args.selection_sign,
                                  resume=args.resume, nan_policy=args.nan_policy)
    save_history(history, args.save_dir)
    print(f"\nCheckpoints saved to {args.save_dir}")
    return model, history


if __name__ == "__main__":
    main()
