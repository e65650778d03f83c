"""3-phase GAN training: ``train_epoch`` / ``evaluate`` / ``train_3phase`` (+ CLI in ``cli.py``).

Schedule semantics are those of `/root/reference/src/train.py:156-426`:

  phase 1  ``num_epochs_unc`` × (SDF step on L_unc, eval valid, eval test); best tracking
           strictly after ``ignore_epoch`` on valid L_unc (→ best_model_loss.pt) and valid
           Sharpe (→ best_model_sharpe.pt + in-memory best state)
  reload   the phase-1 best-Sharpe state (Adam moments are *not* rewound)
  phase 2  ``num_epochs_moment`` × moment step on −L_cond with the SDF frozen (dropout still
           active); best train L_cond → best_model_loss.pt (always fires at epoch 0)
  phase 3  ``num_epochs`` × (SDF step on L_cond, eval valid, eval test), fresh trackers
  finish   reload best-Sharpe state, final evals, final_model.pt

Two executors implement it:
  * CPU: PyTorch modules + ``torch.optim.Adam`` (BASELINE config 1, and the parity oracle);
  * GPU: the native HIP engine (``engine.GANEngine``): the whole panel resident in HBM, one
    hipGraph per epoch, device-side best tracking and history, no per-epoch host syncs.
Both write byte-compatible checkpoints (state_dict keys/shapes/dtype) and ``history.npz``.
"""
from __future__ import annotations

import os
import time
from typing import Dict, Optional

import numpy as np
import torch
import torch.optim as optim

from ..models.gan import AssetPricingGAN
from ..models import losses as L
from .metrics import compute_max_drawdown, compute_sharpe


def _to(data: Dict, device):
    macro = data.get("macro_features")
    return (None if macro is None else macro.to(device), data["individual_features"].to(device),
            data["returns"].to(device), data["mask"].to(device))


def _sharpe_dev(p: torch.Tensor) -> torch.Tensor:
    """``compute_sharpe`` on the device (0 when the unbiased std < 1e-8), no host sync."""
    sd = p.std()
    return torch.where(sd < 1e-8, torch.zeros_like(sd), p.mean() / sd)


def train_epoch(model, optimizer, data: dict, device, phase: str = "conditional",
                grad_clip: float = 1.0, scope: str = "all") -> dict:
    """One full-batch optimisation step (`/root/reference/src/train.py:45-103`).

    The six returned scalars are gathered on the device and read back with ONE host
    synchronisation (the reference calls ``.item()`` six times); values are identical."""
    model.train()
    macro, x, r, m = _to(data, device)
    optimizer.zero_grad()
    out = model(macro, x, r, m, phase=phase)
    loss = out["loss"]
    loss.backward()
    params = {"sdf": model.sdf_net.parameters, "moment": model.moment_net.parameters}.get(
        scope, model.parameters)()
    gn = torch.nn.utils.clip_grad_norm_(params, max_norm=grad_clip)
    optimizer.step()
    dev = loss.device
    z = torch.zeros((), device=dev)
    vals = torch.stack([loss.detach().reshape(()).float(),
                        out.get("loss_unconditional", z).detach().reshape(()).float().to(dev),
                        out.get("loss_conditional", z).detach().reshape(()).float().to(dev),
                        out.get("loss_residual", z).detach().reshape(()).float().to(dev),
                        _sharpe_dev(out["portfolio_returns"].detach().float()).to(dev),
                        torch.as_tensor(gn, device=dev).detach().reshape(()).float()])
    v = vals.tolist()                                              # the one host sync
    return {"loss": v[0], "loss_unc": v[1], "loss_cond": v[2], "loss_residual": v[3],
            "sharpe": v[4], "grad_norm": v[5]}


@torch.no_grad()
def evaluate(model, data: dict, device, normalized: bool = True) -> dict:
    """Eval-mode metrics with L1-normalised weights (`/root/reference/src/train.py:106-153`)."""
    model.eval()
    macro, x, r, m = _to(data, device)
    w, _ = model.get_weights(macro, x, m, normalized=normalized)
    pr = (w * r * m.float()).sum(dim=1)
    port = pr.cpu().numpy()
    out = model(macro, x, r, m, phase="conditional")
    return {
        "loss": out["loss"].item(),
        "loss_unc": out.get("loss_unconditional", torch.tensor(0)).item(),
        "loss_cond": out.get("loss_conditional", torch.tensor(0)).item(),
        "sharpe": compute_sharpe(pr.cpu()),
        "max_drawdown": compute_max_drawdown(port),
        "mean_return": port.mean(),
        "std_return": port.std(),
        "weights": w.cpu(),
    }


def _save(model, save_dir, name):
    if save_dir:
        torch.save(model.state_dict(), os.path.join(save_dir, name))


def _fmt_line(epoch, n, dt, tr, va, te, loss_key):
    s = (f"Epoch {epoch + 1:4d}/{n} ({dt:.1f}s) | Train: loss={tr['loss']:.4f} sharpe={tr['sharpe']:.2f} | "
         f"Valid: loss={va[loss_key]:.4f} sharpe={va['sharpe']:.2f}")
    if te is not None:
        s += f" | Test sharpe={te['sharpe']:.2f}"
    return s


def _print_header(title, n):
    print("\n" + "=" * 70 + f"\n{title}\nEpochs: {n}\n" + "=" * 70 + "\n")


def print_final(model_eval, train_data, valid_data, test_data):
    ft, fv = model_eval(train_data), model_eval(valid_data)
    print("\nBest Model Performance (normalized weights):")
    print(f"  Train - Sharpe: {ft['sharpe']:7.3f}, MaxDD: {ft['max_drawdown']:7.2%}")
    print(f"  Valid - Sharpe: {fv['sharpe']:7.3f}, MaxDD: {fv['max_drawdown']:7.2%}")
    if test_data is not None:
        fe = model_eval(test_data)
        print(f"  Test  - Sharpe: {fe['sharpe']:7.3f}, MaxDD: {fe['max_drawdown']:7.2%}")
    print("=" * 70)


def train_3phase(config: dict, train_data: dict, valid_data: dict, test_data: dict = None,
                 device: torch.device = None, num_epochs_unc: int = 256,
                 num_epochs_moment: int = 64, num_epochs: int = 1024, lr: float = 1e-3,
                 print_freq: int = 128, save_dir: str = None, ignore_epoch: int = 64,
                 save_best_freq: int = 128, *, seed: Optional[int] = None,
                 precision: str = "bf16", selection_sign: float = 1.0,
                 verbose: bool = True, resume: bool = False, resume_path: Optional[str] = None,
                 nan_policy: str = "warn", stop_after=None):
    """Train with the 3-phase schedule; returns ``(model, history)``.

    Extra keyword-only knobs (additions, defaults keep reference behaviour):
      seed            -- dropout stream seed of the GPU engine (defaults to torch's seed)
      precision       -- GPU GEMM input precision, 'bf16' (fp32 accumulate/master) or 'fp32'
      selection_sign  -- +1 selects the best epoch by the un-negated Sharpe (reference);
                         −1 by the paper-convention Sharpe of the SDF factor −w·R
      resume          -- continue from ``resume_path`` (default ``save_dir/resume.pt``), which
                         both executors write at every print boundary and phase end
      nan_policy      -- 'warn' | 'raise' | 'ignore' for non-finite train loss / grad norm
      stop_after      -- (phase, epochs): stop early after writing the resume record (tests)
    ``save_best_freq`` is accepted and unused, as in the reference. Returns None when
    ``stop_after`` stopped the run.
    """
    if device is None:
        device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    device = torch.device(device)
    if verbose:
        print(f"Training on device: {device}")
    if device.type == "cuda":
        from ..engine.runner import train_3phase_gpu
        return train_3phase_gpu(config, train_data, valid_data, test_data, device=device,
                                num_epochs_unc=num_epochs_unc, num_epochs_moment=num_epochs_moment,
                                num_epochs=num_epochs, lr=lr, print_freq=print_freq,
                                save_dir=save_dir, ignore_epoch=ignore_epoch, seed=seed,
                                precision=precision, selection_sign=selection_sign,
                                verbose=verbose, resume=resume, resume_path=resume_path,
                                nan_policy=nan_policy, stop_after=stop_after)
    return _train_3phase_cpu(config, train_data, valid_data, test_data, device, num_epochs_unc,
                             num_epochs_moment, num_epochs, lr, print_freq, save_dir,
                             ignore_epoch, selection_sign, verbose, resume, resume_path,
                             nan_policy, stop_after)


class _Stop(Exception):
    pass


def _train_3phase_cpu(config, train_data, valid_data, test_data, device, n_unc, n_mom, n_cond,
                      lr, print_freq, save_dir, ignore_epoch, sel, verbose, resume=False,
                      resume_path=None, nan_policy="warn", stop_after=None, *, model=None,
                      train_fn=None, eval_fn=None):
    """``model`` / ``train_fn`` / ``eval_fn`` substitute the module and the step / evaluation
    functions (the cross-sectionally sharded executor of ``parallel.xsection`` passes its own)."""
    from ..utils.guards import NonFiniteError, POLICIES
    import warnings
    if nan_policy not in POLICIES:
        raise ValueError(f"nan_policy must be one of {POLICIES}")
    say = print if verbose else (lambda *a, **k: None)
    train_epoch_ = train_fn or train_epoch
    evaluate_ = eval_fn or evaluate
    if model is None:
        model = AssetPricingGAN(config).to(device)
    n_sdf = sum(p.numel() for p in model.sdf_net.parameters())
    n_mom_p = sum(p.numel() for p in model.moment_net.parameters())
    say(f"Model has {n_sdf + n_mom_p:,} trainable parameters")
    say(f"  SDF network: {n_sdf:,}")
    say(f"  Moment network: {n_mom_p:,}")
    opt_sdf = optim.Adam(model.sdf_net.parameters(), lr=lr)
    opt_mom = optim.Adam(model.moment_net.parameters(), lr=lr)
    hist = {k: [] for k in ("train_loss", "train_sharpe", "valid_loss", "valid_sharpe",
                            "test_loss", "test_sharpe", "phase")}
    # schedule position + trackers (everything a resume record must carry)
    st = {"phase": 1, "done": 0, "best_loss": float("inf"), "best_sr": float("-inf"),
          "best_m": float("-inf"), "best_state": None, "elapsed": 0.0, "nonfinite": -1}
    schedule = [int(n_unc), int(n_mom), int(n_cond)]
    if resume_path is None and save_dir:
        resume_path = os.path.join(save_dir, "resume.pt")
    if resume and resume_path and os.path.isfile(resume_path):
        rec = torch.load(resume_path, map_location="cpu", weights_only=True)
        if rec.get("executor") != "cpu" or list(rec["schedule"]) != schedule:
            raise ValueError(f"{resume_path}: not a CPU resume record of schedule {schedule}")
        model.load_state_dict(rec["model"])
        opt_sdf.load_state_dict(rec["opt_sdf"])
        opt_mom.load_state_dict(rec["opt_mom"])
        hist = {k: list(v) for k, v in rec["hist"].items()}
        st.update(rec["state"])
        torch.set_rng_state(rec["rng"])
        say(f"Resumed from {resume_path}: phase {st['phase']}, {st['done']} epochs done")
    t0 = time.time() - st["elapsed"]

    def write_resume():
        if not resume_path:
            return
        st["elapsed"] = time.time() - t0
        rec = {"executor": "cpu", "schedule": schedule, "model": model.state_dict(),
               "opt_sdf": opt_sdf.state_dict(), "opt_mom": opt_mom.state_dict(),
               "hist": hist, "state": dict(st), "rng": torch.get_rng_state()}
        tmp = resume_path + ".tmp"
        torch.save(rec, tmp)
        os.replace(tmp, resume_path)

    def check_finite(e, tr):
        if nan_policy == "ignore" or st["nonfinite"] >= 0:
            return
        for field in ("loss", "grad_norm"):
            if not np.isfinite(tr[field]):
                st["nonfinite"] = len(hist["train_loss"]) - 1
                if nan_policy == "raise":
                    raise NonFiniteError(0, e, "train_loss" if field == "loss" else field)
                warnings.warn(f"non-finite {field} at epoch {e + 1}", RuntimeWarning)
                return

    def boundary(phase, e, n):
        """After epoch e of a phase: resume record at print boundaries / phase end."""
        st["phase"], st["done"] = phase, e + 1
        if (e + 1) % print_freq == 0 or e + 1 == n:
            write_resume()
        if stop_after is not None and tuple(stop_after) == (phase, e + 1):
            write_resume()
            raise _Stop()

    def run_sdf_phase(n, phase_id, phase, tag, loss_key):
        start = st["done"] if st["phase"] == phase_id else 0
        if start == 0:
            st["best_loss"], st["best_sr"] = float("inf"), float("-inf")
        for e in range(start, n):
            te0 = time.time()
            tr = train_epoch_(model, opt_sdf, train_data, device, phase=phase, scope="sdf")
            va = evaluate_(model, valid_data, device)
            te = evaluate_(model, test_data, device) if test_data is not None else None
            hist["train_loss"].append(tr["loss"]); hist["train_sharpe"].append(tr["sharpe"])
            hist["phase"].append(tag)
            hist["valid_loss"].append(va[loss_key]); hist["valid_sharpe"].append(va["sharpe"])
            if te is not None:
                hist["test_loss"].append(te[loss_key]); hist["test_sharpe"].append(te["sharpe"])
            check_finite(e, tr)
            if e > ignore_epoch:
                if va[loss_key] < st["best_loss"]:
                    st["best_loss"] = va[loss_key]
                    _save(model, save_dir, "best_model_loss.pt")
                if sel * va["sharpe"] > st["best_sr"]:
                    st["best_sr"] = sel * va["sharpe"]
                    st["best_state"] = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
                    _save(model, save_dir, "best_model_sharpe.pt")
            if (e + 1) % print_freq == 0 or e == 0:
                say(_fmt_line(e, n, time.time() - te0, tr, va, te, loss_key))
            boundary(phase_id, e, n)
        return st["best_sr"]

    try:
        if st["phase"] == 1:
            _print_header("PHASE 1: Training Unconditional Loss (E[w*R]^2)", n_unc) if verbose else None
            b1 = run_sdf_phase(n_unc, 1, "unconditional", "unc", "loss_unc")
            say("\nPhase 1 Complete!")
            say(f"Best validation Sharpe (phase 1): {sel * b1:.4f}")
            if st["best_state"] is not None:
                model.load_state_dict(st["best_state"])
                say("Loaded best model from Phase 1")
            st["phase"], st["done"], st["best_m"] = 2, 0, float("-inf")
            write_resume()

        if st["phase"] == 2:
            _print_header("PHASE 2: Updating Moment Conditions", n_mom) if verbose else None
            for p in model.sdf_net.parameters():
                p.requires_grad_(False)
            for e in range(st["done"], n_mom):
                te0 = time.time()
                tr = train_epoch_(model, opt_mom, train_data, device, phase="moment", scope="moment")
                if tr["loss_cond"] > st["best_m"]:
                    st["best_m"] = tr["loss_cond"]
                    _save(model, save_dir, "best_model_loss.pt")
                if (e + 1) % print_freq == 0 or e == 0:
                    say(f"Epoch {e + 1:4d}/{n_mom} ({time.time() - te0:.1f}s) | Conditional loss: {tr['loss_cond']:.6f}")
                boundary(2, e, n_mom)
            for p in model.sdf_net.parameters():
                p.requires_grad_(True)
            say("\nPhase 2 Complete!")
            st["phase"], st["done"] = 3, 0
            write_resume()

        # Phase 3: the moment net is never stepped again; freezing it skips dead gradient work.
        for p in model.moment_net.parameters():
            p.requires_grad_(False)
        _print_header("PHASE 3: Training Conditional Loss (E[h*w*R]^2)", n_cond) if verbose else None
        run_sdf_phase(n_cond, 3, "conditional", "cond", "loss_cond")
        for p in model.moment_net.parameters():
            p.requires_grad_(True)
    except _Stop:
        say(f"Stopped after {tuple(stop_after)}; resume record at {resume_path}")
        return None
    total = time.time() - t0
    if st["best_state"] is not None:
        model.load_state_dict(st["best_state"])
    say("\n" + "=" * 70 + "\nTraining Complete!")
    say(f"Total time: {total / 60:.1f} minutes")
    say(f"Total epochs: {n_unc + n_mom + n_cond} ({n_unc} + {n_mom} + {n_cond})\n" + "=" * 70)
    if verbose:
        print_final(lambda d: evaluate_(model, d, device), train_data, valid_data, test_data)
    _save(model, save_dir, "final_model.pt")
    return model, hist


def save_history(history: dict, save_dir: str):
    np.savez(os.path.join(save_dir, "history.npz"), **{k: np.array(v) for k, v in history.items()})
