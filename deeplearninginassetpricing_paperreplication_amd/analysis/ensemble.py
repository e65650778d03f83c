"""Ensemble evaluation: average the L1-normalised SDF weights of several trained models.

Behaviour of `/root/reference/src/evaluate_ensemble.py` (load each checkpoint's
``config.json`` + ``best_model_sharpe.pt``, weights per split, average, re-normalise, paper-sign
Sharpe with ddof=0; individual test Sharpe; comparison with the paper's 0.75), same CLI
(``--data_dir --checkpoint_dirs ...``) plus ``--device``.

On a GPU the weights of all checkpoints that share an architecture are produced by ONE batched
native-engine forward per split (models stacked along the engine's job axis) instead of one
PyTorch forward per model; they stay on the device, where the K11 kernel (``k_ensemble``)
averages, re-normalises and forms the portfolio series (one host transfer per split).
"""
from __future__ import annotations

import argparse
import json
import os
from typing import Dict, List, Sequence

import numpy as np
import torch

from ..data.dataset import load_splits
from ..models.gan import AssetPricingGAN
from .portfolio import (PAPER_TEST_SHARPE, average_weights, ensemble_sharpes, ensemble_sharpes_device,
                        paper_metrics)
from .portfolio import sharpe_ddof0 as compute_sharpe  # noqa: F401  (reference name)

SPLITS = ("train", "valid", "test")


def load_model(checkpoint_dir: str, device: str = "cpu", which: str = "best_model_sharpe.pt"):
    """``AssetPricingGAN`` from ``config.json`` + a state_dict file (safe tensor-only load)."""
    with open(os.path.join(checkpoint_dir, "config.json")) as fh:
        config = json.load(fh)
    model = AssetPricingGAN(config)
    sd = torch.load(os.path.join(checkpoint_dir, which), map_location="cpu", weights_only=True)
    model.load_state_dict(sd)
    model.to(device).eval()
    return model, config


def get_weights_from_model(model, data: Dict, device: str = "cpu") -> np.ndarray:
    macro = data.get("macro_features")
    with torch.no_grad():
        w, _ = model.get_weights(None if macro is None else macro.to(device),
                                 data["individual_features"].to(device), data["mask"].to(device),
                                 normalized=True)
    return w.detach().cpu().numpy()


def weights_batched_gpu(models: Sequence, batches: Dict[str, Dict]) -> Dict[str, torch.Tensor]:
    """L1-normalised weights of every model on every split as CUDA tensors [G, T, N] (model
    order), one batched engine forward per split for each group of models that share an
    architecture. Everything stays on the device: the engine's ``wn`` buffers are copied
    device-to-device into the stack (ordered after torch's stream with events, no host sync) and
    normalised there."""
    from ..engine.runner import GANEngine
    dev = torch.device("cuda", torch.cuda.current_device())
    ts = torch.cuda.current_stream(dev).cuda_stream
    out = {}
    for split in SPLITS:
        T, N = batches[split]["mask"].shape
        out[split] = torch.empty(len(models), T, N, dtype=torch.float32, device=dev)
    groups: Dict[object, List[int]] = {}
    for i, m in enumerate(models):
        groups.setdefault(m.spec, []).append(i)
    for spec, idx in groups.items():
        eng = GANEngine(spec, len(idx), max_epochs=4)
        eng.set_data(batches["train"], batches["valid"], batches["test"])
        for g, i in enumerate(idx):
            eng.set_model(g, models[i], 0)
        e = eng.eng
        e.join_from(ts)
        for s, split in enumerate(SPLITS):
            e.forward_split(s, False, False)
            for g, i in enumerate(idx):
                e.copy_ws(g, s, "wn", out[split][i].data_ptr())
        e.join_to(ts)
        e.sync()         # the engine (and its buffers) may be freed after this group
    for split in SPLITS:                 # per (model, period) L1 normalisation over the stocks
        m = batches[split]["mask"].to(dev).float()
        W = out[split]
        out[split] = W / (W.abs() * m[None]).sum(dim=2, keepdim=True).clamp(min=1e-8)
    return out


def evaluate_ensemble(checkpoint_dirs: Sequence[str], data_dir: str, device: str = "cpu",
                      verbose: bool = True, paper: bool = False) -> Dict:
    """Reference output and return value; ``paper=True`` (CLI ``--paper_metrics``) adds the
    paper's EV / XS-R² / turnover / max 1-month loss of the ensemble's SDF factor per split."""
    say = print if verbose else (lambda *a, **k: None)
    bar = "=" * 70
    say(bar); say(f"ENSEMBLE EVALUATION ({len(checkpoint_dirs)} models, averaged weights)"); say(bar); say()
    datasets = load_splits(data_dir)
    batches = {s: d.get_full_batch() for s, d in zip(SPLITS, datasets)}
    say("Loaded data:")
    for s in SPLITS:
        say(f"  {s.capitalize():6s} {batches[s]['returns'].shape[0]} periods")
    say()
    say(f"Loading {len(checkpoint_dirs)} models...")
    models = []
    for i, d in enumerate(checkpoint_dirs):
        say(f"  Model {i + 1}/{len(checkpoint_dirs)}: {os.path.basename(os.path.normpath(d))}")
        models.append(load_model(d, "cpu")[0])
    np_batches = {s: {"returns": batches[s]["returns"].numpy(), "mask": batches[s]["mask"].numpy()}
                  for s in SPLITS}
    if str(device).startswith("cuda"):
        # batched engine forward + K11 (k_ensemble) averaging on the device: the [T] ensemble
        # and [G, T] individual portfolio series are the only host transfers
        wdev = weights_batched_gpu(models, batches)
        res = ensemble_sharpes_device(wdev, np_batches)
        weights = None
        if paper:
            weights = [{s: wdev[s][i].cpu().numpy() for s in SPLITS} for i in range(len(models))]
    else:
        weights = [{s: get_weights_from_model(m, batches[s], "cpu") for s in SPLITS} for m in models]
        res = ensemble_sharpes(weights, np_batches)
    ind = res["individual_sharpes"]
    say(); say(bar); say("INDIVIDUAL MODEL RESULTS (for comparison)"); say(bar); say()
    for i, s in enumerate(ind):
        say(f"  Model {i + 1}: Test Sharpe = {s:.4f}")
    say(); say(f"  Mean of individual models: {np.mean(ind):.4f}")
    say(f"  Std of individual models:  {np.std(ind):.4f}")
    say(); say(bar); say("ENSEMBLE RESULTS (averaged weights)"); say(bar); say()
    for s in SPLITS:
        say(f"  {s.capitalize()} Sharpe: {res[s + '_sharpe']:.4f}")
    say(); say(bar); say("COMPARISON WITH PAPER"); say(bar); say()
    say(f"  Paper GAN Test Sharpe:     {PAPER_TEST_SHARPE}")
    say(f"  Our Ensemble Test Sharpe:  {res['test_sharpe']:.4f}")
    say(f"  Ratio (Our / Paper):       {res['test_sharpe'] / PAPER_TEST_SHARPE:.1%}")
    say()
    out = {"train_sharpe": res["train_sharpe"], "valid_sharpe": res["valid_sharpe"],
           "test_sharpe": res["test_sharpe"], "individual_sharpes": ind}
    if paper:
        out["paper_metrics"] = {}
        say(bar); say("PAPER METRICS OF THE ENSEMBLE SDF FACTOR (Table I / A.VI / A.VII)"); say(bar); say()
        for s in SPLITS:
            b = np_batches[s]
            avg = average_weights([w[s] for w in weights], b["mask"])
            pm = paper_metrics(avg, b["returns"], b["mask"])
            out["paper_metrics"][s] = pm
            say(f"  {s.capitalize():5s}  SR {pm['sharpe']:7.4f}  EV {pm['ev']:7.4f}  XS-R2 {pm['xs_r2']:7.4f}  "
                f"turnover {pm['turnover']:6.3f}  max 1m loss {pm['max_1m_loss_std']:5.2f} sd")
        say()
    return out


def main(argv=None):
    p = argparse.ArgumentParser(description="Evaluate an ensemble by averaging SDF weights")
    p.add_argument("--data_dir", type=str, required=True)
    p.add_argument("--checkpoint_dirs", type=str, nargs="+", required=True)
    p.add_argument("--device", type=str, default="cpu", help="cpu | cuda (batched native engine)")
    p.add_argument("--paper_metrics", action="store_true", help="also print EV / XS-R2 / turnover / max loss")
    a = p.parse_args(argv)
    return evaluate_ensemble(a.checkpoint_dirs, a.data_dir, a.device, paper=a.paper_metrics)


if __name__ == "__main__":
    main()
