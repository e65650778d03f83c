"""Resume checkpoints (an addition: the reference saves final/best state dicts only and cannot
resume, `/root/reference/src/train.py:262-272,320-323,373-382,399-424`).

``resume.pt`` sits next to the reference's five files in ``save_dir`` and holds everything the
GPU engine needs to continue a 3-phase run bit-for-bit where it stopped:

  * the schedule position: phase (1..3) and epochs completed in it, the epoch counts,
  * per model: parameters, Adam moments + step counters, the dropout stream (seed, step),
    the per-phase best trackers and snapshot flags, both best-model snapshots, the device
    history rows, the per-model learning rate,
  * a fingerprint of the architecture (``ModelSpec``) so a file is never applied to a
    different model, and a run fingerprint (learning rate, ``ignore_epoch``, selection sign and a
    cheap checksum of every split's shape / mask / returns) so it is never continued with other
    hyperparameters or data.

The file is written atomically (temp file + ``os.replace``) at every print boundary and phase
end, so a crash leaves either the previous or the new complete state. It contains only tensors,
numbers and strings and is read with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import torch

RESUME_FILE = "resume.pt"
FORMAT_VERSION = 1


def _t(a) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a)))


def capture_model(eng, g: int, seed: int, lr: Optional[float]) -> Dict:
    """Snapshot of model ``g`` of a native ``Engine`` (all tensors on the host)."""
    opt = eng.get_opt_state(g)
    trk = eng.get_tracker_state(g)
    return {
        "params": _t(eng.get_params(g)), "adam_m": _t(opt["m"]), "adam_v": _t(opt["v"]),
        "step_sdf": int(opt["step_sdf"]), "step_moment": int(opt["step_moment"]),
        "drop_step": int(opt["drop_step"]), "seed": int(seed),
        "lr": float(lr) if lr is not None else 0.0,
        "epoch": int(trk["epoch"]), "epoch_in_phase": int(trk["epoch_in_phase"]),
        "snap_loss_taken": int(trk["snap_loss_taken"]), "snap_sharpe_taken": int(trk["snap_sharpe_taken"]),
        "best_loss": float(trk["best_loss"]), "best_sharpe": float(trk["best_sharpe"]),
        "best_moment": float(trk["best_moment"]),
        "snap_loss": _t(trk["snap_loss"]), "snap_sharpe": _t(trk["snap_sharpe"]),
        "hist": _t(trk["hist"]),
    }


def restore_model(eng, g: int, st: Dict):
    eng.set_params(g, st["params"].numpy())
    eng.set_seed(g, int(st["seed"]) & 0xFFFFFFFF)
    if st.get("lr", 0.0) > 0:
        eng.set_lr(g, float(st["lr"]))
    eng.set_opt_state(g, st["adam_m"].numpy(), st["adam_v"].numpy(), int(st["step_sdf"]),
                      int(st["step_moment"]), int(st["drop_step"]))
    eng.set_tracker_state(g, int(st["epoch"]), int(st["epoch_in_phase"]), int(st["snap_loss_taken"]),
                          int(st["snap_sharpe_taken"]), float(st["best_loss"]), float(st["best_sharpe"]),
                          float(st["best_moment"]), st["snap_loss"].numpy(), st["snap_sharpe"].numpy(),
                          np.ascontiguousarray(st["hist"].numpy().reshape(-1)))


def spec_fingerprint(spec) -> str:
    return repr(spec)


def data_fingerprint(*batches) -> str:
    """Cheap identity of the training data: per split its [T, N] shape, the number of valid
    entries, and float64 sums of the mask pattern (weighted by position) and of the returns."""
    parts = []
    for b in batches:
        if b is None:
            parts.append("-")
            continue
        m = torch.as_tensor(b["mask"]).detach().to("cpu", torch.float64)
        r = torch.as_tensor(b["returns"]).detach().to("cpu", torch.float64) * m
        pos = torch.arange(m.numel(), dtype=torch.float64).reshape(m.shape)
        parts.append(f"{tuple(m.shape)}:{int(m.sum())}:{float((m * pos).sum()):.6e}:{float(r.sum()):.9e}")
    return "|".join(parts)


def run_fingerprint(lr: float, ignore_epoch: int, selection_sign: float, data: str) -> Dict:
    return {"lr": float(lr), "ignore_epoch": int(ignore_epoch), "selection_sign": float(selection_sign),
            "data": str(data)}


def save_resume(path: str, *, spec, phase: int, done: int, schedule, models: List[Dict],
                best_state: List[bool], elapsed: float, run: Optional[Dict] = None):
    rec = {
        "format": FORMAT_VERSION, "spec": spec_fingerprint(spec), "phase": int(phase),
        "done": int(done), "schedule": [int(x) for x in schedule], "models": models,
        "best_state": [bool(b) for b in best_state], "elapsed": float(elapsed),
        "run": dict(run) if run is not None else {},
    }
    tmp = path + ".tmp"
    torch.save(rec, tmp)
    os.replace(tmp, path)


def load_resume(path: str, spec=None, schedule=None, run: Optional[Dict] = None) -> Optional[Dict]:
    """The resume record at ``path`` (None if absent). Raises if it belongs to another
    architecture, schedule, or (``run``) learning rate / ignore_epoch / selection sign / data."""
    if not os.path.isfile(path):
        return None
    rec = torch.load(path, map_location="cpu", weights_only=True)
    if rec.get("format") != FORMAT_VERSION:
        raise ValueError(f"{path}: unsupported resume format {rec.get('format')}")
    if spec is not None and rec["spec"] != spec_fingerprint(spec):
        raise ValueError(f"{path}: saved for a different model architecture")
    if schedule is not None and list(rec["schedule"]) != [int(x) for x in schedule]:
        raise ValueError(f"{path}: saved for schedule {rec['schedule']}, not {list(schedule)}")
    if run is not None:
        saved = rec.get("run") or {}
        for k, v in run.items():
            if k not in saved:
                raise ValueError(f"{path}: record has no run fingerprint entry {k!r}")
            if saved[k] != v:
                raise ValueError(f"{path}: saved with {k}={saved[k]!r}, this run has {k}={v!r}")
    return rec
