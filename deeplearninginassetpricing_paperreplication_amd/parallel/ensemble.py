"""Seed-ensemble training over the GPUs of a node (BASELINE config 3).

The reference trains its 9-seed ensemble serially (`/root/reference/notebooks/demo_full.ipynb`,
~6 h on CPU) and then averages the L1-normalised weights
(`/root/reference/src/evaluate_ensemble.py:53-210`). Here:

  * seeds are sharded round-robin over ranks (one process per GPU; 9 over 8 -> rank 0 gets 2);
  * a rank trains ALL of its seeds at once: they are batched as jobs of one native engine
    (every kernel launch covers every member, the serial LSTM / loss kernels run the members
    in parallel workgroups), so an extra member costs far less than an extra run;
  * each member's best-Sharpe weights [T, N] per split are exchanged with ONE padded RCCL
    all-gather per split (``comm.all_gather_rows``), then every rank computes the ensemble
    metrics (identical on all ranks, no extra broadcast);
  * a member whose training raises is isolated: its weights are NaN, it is excluded from the
    average and reported in ``failed``.

Run:  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m \
          deeplearninginassetpricing_paperreplication_amd.parallel.ensemble --data_dir D
"""
from __future__ import annotations

import argparse
import json
import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..analysis.portfolio import ensemble_sharpes, ensemble_sharpes_device
from ..config import default_cli_config
from ..models.gan import AssetPricingGAN
from . import comm

PAPER_SEEDS = (42, 123, 456, 789, 1000, 2000, 3000, 4000, 5000)
SPLITS = ("train", "valid", "test")


def _init_models(config: Dict, seeds: Sequence[int]) -> List[AssetPricingGAN]:
    out = []
    for s in seeds:                       # same init as `python -m src.train --seed s`
        torch.manual_seed(s)
        np.random.seed(s % (2 ** 32))
        out.append(AssetPricingGAN(config))
    return out


def train_members(config: Dict, batches: Dict[str, Dict], seeds: Sequence[int], device: torch.device,
                  epochs=(256, 64, 1024), lr: float = 1e-3, ignore_epoch: int = 64,
                  print_freq: int = 128, save_root: Optional[str] = None, verbose: bool = False,
                  selection_sign: float = 1.0, fail_seeds: Sequence[int] = ()) -> List[Dict]:
    """Train ``seeds`` on this process. Returns one record per seed:
    ``{seed, ok, error, weights: {split: [T, N] float32}, history}``."""
    recs = [{"seed": int(s), "ok": False, "error": None, "weights": None, "history": None, "timing": None}
            for s in seeds]
    dirs = [None] * len(seeds)
    if save_root:
        for i, s in enumerate(seeds):
            dirs[i] = os.path.join(save_root, f"seed_{s}")
            os.makedirs(dirs[i], exist_ok=True)
            with open(os.path.join(dirs[i], "config.json"), "w") as fh:
                json.dump(config, fh, indent=2)
    n1, n2, n3 = epochs
    tr, va, te = batches["train"], batches["valid"], batches["test"]
    todo = [i for i, s in enumerate(seeds) if s not in set(fail_seeds)]
    for i, s in enumerate(seeds):
        if s in set(fail_seeds):
            recs[i]["error"] = "injected failure"
    if not todo:
        return recs
    if device.type == "cuda":
        from ..engine.runner import train_3phase_gpu
        from ..train.trainer import save_history
        try:
            models = _init_models(config, [seeds[i] for i in todo])
            res_m, res_h = train_3phase_gpu(
                config, tr, va, te, device=device, num_epochs_unc=n1, num_epochs_moment=n2,
                num_epochs=n3, lr=lr, print_freq=print_freq, ignore_epoch=ignore_epoch,
                selection_sign=selection_sign, verbose=verbose, models=models,
                seeds=[seeds[i] for i in todo], save_dirs=[dirs[i] for i in todo], final_weights_device=True)
            if len(todo) == 1:
                res_m, res_h = [res_m], [res_h]
            tm = dict(train_3phase_gpu.last_timers.total)
            tm["graph-capture"] = train_3phase_gpu.last_capture_s
            for i in todo:
                recs[i]["timing"] = tm
            for k, i in enumerate(todo):
                fe = res_m[k].engine_final_eval
                # (CUDA tensors: the members' weights never leave the GPU before the all-gather)
                recs[i].update(ok=True, history=res_h[k],
                               weights={sp: fe[j]["weights"] for j, sp in enumerate(SPLITS)})
                if dirs[i]:
                    save_history(res_h[k], dirs[i])
        except Exception as e:          # whole batch failed (e.g. OOM): isolate, do not hang peers
            for i in todo:
                recs[i]["error"] = f"{type(e).__name__}: {e}"
        return recs
    from ..train.trainer import evaluate, save_history, train_3phase
    for i in todo:
        s = seeds[i]
        try:
            torch.manual_seed(s)
            np.random.seed(s % (2 ** 32))
            model, hist = train_3phase(config, tr, va, te, device=torch.device("cpu"), num_epochs_unc=n1,
                                       num_epochs_moment=n2, num_epochs=n3, lr=lr, print_freq=print_freq,
                                       save_dir=dirs[i], ignore_epoch=ignore_epoch,
                                       selection_sign=selection_sign, verbose=verbose)
            w = {sp: evaluate(model, b, "cpu")["weights"].numpy() for sp, b in zip(SPLITS, (tr, va, te))}
            recs[i].update(ok=True, history=hist, weights=w)
            if dirs[i]:
                save_history(hist, dirs[i])
        except Exception as e:
            recs[i]["error"] = f"{type(e).__name__}: {e}"
    return recs


def run_ensemble(config: Dict, batches: Dict[str, Dict], seeds: Sequence[int] = PAPER_SEEDS,
                 dist: Optional[comm.Dist] = None, epochs=(256, 64, 1024), lr: float = 1e-3,
                 ignore_epoch: int = 64, print_freq: int = 128, save_root: Optional[str] = None,
                 verbose: bool = False, selection_sign: float = 1.0, fail_seeds: Sequence[int] = ()) -> Dict:
    """Train the ensemble across the process group and evaluate the averaged weights."""
    d = dist or comm.Dist()
    mine = comm.shard(len(seeds), d.rank, d.world)
    t0 = time.time()
    recs = train_members(config, batches, [seeds[i] for i in mine], d.device, epochs, lr, ignore_epoch,
                         print_freq, save_root, verbose, selection_sign, fail_seeds)
    t_train = time.time() - t0
    # per-rank breakdown of the non-epoch costs (BREAKDOWN order), seconds
    tm = next((r["timing"] for r in recs if r.get("timing")), None) or {}
    epochs_s = sum(v for k, v in tm.items() if k.endswith("-epochs"))
    parts = {"engine_build": tm.get("engine-build", 0.0), "panel_compaction": tm.get("panel-compaction", 0.0),
             "set_params": tm.get("set-params", 0.0), "graph_capture": tm.get("graph-capture", 0.0),
             "epochs": max(0.0, epochs_s - tm.get("graph-capture", 0.0)), "final_eval": tm.get("final-eval", 0.0)}
    t1 = time.time()
    ok_local = np.array([r["ok"] for r in recs], dtype=np.float32).reshape(-1, 1)
    ok = comm.all_gather_rows(d, ok_local, len(seeds), mine)[:, 0] > 0.5
    weights: List[Dict[str, np.ndarray]] = [dict() for _ in seeds]
    on_gpu = d.device.type == "cuda"
    wdev = {}
    for sp in SPLITS:
        T, N = batches[sp]["mask"].shape
        if on_gpu:
            # RCCL all-gather into the rank's GPU, the ensemble math stays there (K11 kernel): the
            # members' weights go to the device once, nothing comes back to the host
            loc_t = torch.full((len(recs), T, N), float("nan"), dtype=torch.float32, device=d.device)
            for k, r in enumerate(recs):
                if r["ok"]:
                    loc_t[k].copy_(torch.as_tensor(r["weights"][sp]), non_blocking=True)
            allt = comm.all_gather_rows_tensor(d, loc_t, len(seeds), mine)
            wdev[sp] = allt.to(d.device)    # (a gloo rehearsal gathers on the host)
            continue
        loc = np.full((len(recs), T, N), np.nan, np.float32)
        for k, r in enumerate(recs):
            if r["ok"]:
                loc[k] = r["weights"][sp]
        allw = comm.all_gather_rows(d, loc, len(seeds), mine)   # one collective per split
        for i in range(len(seeds)):
            weights[i][sp] = allw[i]
    if on_gpu:
        torch.cuda.synchronize(d.device)
    parts["all_gather"] = time.time() - t1
    walls = comm.all_gather_rows(d, np.array([[t_train]], np.float64), d.world, [d.rank])[:, 0]
    good = [i for i in range(len(seeds)) if ok[i]]
    np_b = {sp: {"returns": _host(batches[sp]["returns"]), "mask": _host(batches[sp]["mask"])} for sp in SPLITS}
    out = {"seeds": [int(s) for s in seeds], "ok": ok.tolist(),
           "failed": [int(seeds[i]) for i in range(len(seeds)) if not ok[i]],
           "world_size": d.world, "train_wall_s_per_rank": walls.tolist(),
           "train_wall_s": float(walls.max())}
    if good:
        if on_gpu:       # K11 on the device, on the all-gathered tensors
            res = ensemble_sharpes_device({sp: wdev[sp][good] for sp in SPLITS}, np_b)
        else:
            res = ensemble_sharpes([weights[i] for i in good], np_b)
        out.update({k: res[k] for k in ("train_sharpe", "valid_sharpe", "test_sharpe")})
        ind = np.full(len(seeds), np.nan)
        ind[good] = res["individual_sharpes"]
        out["individual_sharpes"] = ind.tolist()
    parts["ensemble_metrics"] = time.time() - t1 - parts["all_gather"]
    parts["train_total"] = t_train
    keys = list(parts)
    rows = comm.all_gather_rows(d, np.array([[parts[k] for k in keys]], np.float64), d.world, [d.rank])
    out["breakdown_s_per_rank"] = [{k: round(float(v), 4) for k, v in zip(keys, row)} for row in rows]
    out["errors"] = {int(r["seed"]): r["error"] for r in recs if r["error"]}
    return out


def _host(a) -> np.ndarray:
    return a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)


def load_batches(args, d: Optional[comm.Dist] = None) -> Dict[str, Dict]:
    """The three splits for a driver run. With a process group, only rank 0 reads the .npz
    files / generates the panel and RCCL broadcasts it (peers receive it straight into their
    GPU's memory, where the engine compacts it without a host round trip)."""
    if d is None or not d.active:
        return _load_batches(args)
    b = _load_batches(args) if d.rank == 0 else None
    return comm.broadcast_batches(d, b)


def _load_batches(args) -> Dict[str, Dict]:
    if args.synthetic:
        from ..data.synthetic import generate_panel_fast
        T1, T2, T3, N, F, M = args.synthetic
        ret, feats, mask, mac = generate_panel_fast(T1 + T2 + T3, N, F, M, seed=args.data_seed)
        mu = mac[:T1].mean(0, keepdim=True)
        sd = mac[:T1].std(0, unbiased=False, keepdim=True) + 1e-8
        mac = (mac - mu) / sd
        cuts = {"train": (0, T1), "valid": (T1, T1 + T2), "test": (T1 + T2, T1 + T2 + T3)}
        return {k: {"returns": ret[a:b], "individual_features": feats[a:b], "mask": mask[a:b],
                    "macro_features": mac[a:b]} for k, (a, b) in cuts.items()}
    from ..data.dataset import load_splits
    return {k: ds.get_full_batch() for k, ds in zip(SPLITS, load_splits(args.data_dir))}


def main(argv=None):
    p = argparse.ArgumentParser(description="Seed-ensemble training over the GPUs of one node")
    p.add_argument("--data_dir", type=str, default=None)
    p.add_argument("--synthetic", type=int, nargs=6, metavar=("T_TRAIN", "T_VALID", "T_TEST", "N", "F", "M"),
                   default=None, help="train on a generated panel instead of --data_dir")
    p.add_argument("--data_seed", type=int, default=0)
    p.add_argument("--seeds", type=int, nargs="+", default=list(PAPER_SEEDS))
    p.add_argument("--epochs_unc", type=int, default=256)
    p.add_argument("--epochs_moment", type=int, default=64)
    p.add_argument("--epochs", type=int, default=1024)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--ignore_epoch", type=int, default=64)
    p.add_argument("--print_freq", type=int, default=128)
    p.add_argument("--save_root", type=str, default=None)
    p.add_argument("--selection_sign", type=float, default=1.0)
    p.add_argument("--cpu", action="store_true", help="gloo + CPU trainer (no GPU)")
    p.add_argument("--verbose", action="store_true")
    a = p.parse_args(argv)
    if not a.synthetic and not a.data_dir:
        p.error("--data_dir or --synthetic is required")
    d = comm.init(use_gpu=not a.cpu and torch.cuda.is_available())
    batches = load_batches(a, d)
    cfg = default_cli_config(batches["train"]["macro_features"].shape[-1] if "macro_features" in batches["train"] else 0,
                             batches["train"]["individual_features"].shape[-1])
    res = run_ensemble(cfg, batches, a.seeds, d, (a.epochs_unc, a.epochs_moment, a.epochs), a.lr,
                       a.ignore_epoch, a.print_freq, a.save_root, a.verbose, a.selection_sign)
    if d.is_main:
        print(json.dumps(res))
    comm.shutdown(d)
    return res


if __name__ == "__main__":
    main()
