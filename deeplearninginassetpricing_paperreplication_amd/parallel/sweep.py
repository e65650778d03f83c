"""Hyperparameter sweep over the paper's 384-configuration grid, sharded over the GPUs of a node
(BASELINE config 4).

Grid (paper Table A.VIII):
    HL  {2,3,4}        SDF hidden layers of 64 units        -> hidden_dim = [64] * HL
    SMV {4,8}          macro LSTM states                    -> num_units_rnn = [SMV]
    CSMV {16,32}       conditional-network macro states     -> num_units_rnn_moment = [CSMV]
                       (accepted and ignored by the model, exactly as in the reference)
    CHL {0,1}          conditional hidden layers            -> hidden_dim_moment = [] | [CHU]
    CHU {4,8,16,32}    conditional units (moment count)     -> num_condition_moment = CHU
    LR  {1e-3,5e-4,2e-4,1e-4}
3 * 2 * 2 * 2 * 4 * 4 = 384 configurations. The paper does not list the number of moments as a
separate axis; its CHU (conditional hidden units) sets the moment count here (with CHL = 0 the
conditional network has no hidden units, so CHU can only be its output width; with CHL = 1 it is
both the hidden width and the output width). ``--chu hidden`` instead keeps 8 moments and uses
CHU only for the hidden layer. Which mapping the paper's code used is parity-unpinned.

``--grid baseline`` is BASELINE.json config 4's literal axes instead (hidden_dim x lr x dropout x
num_moments, with SMV doubling it to 384): HL {2,3,4} x LR {4 values} x dropout {0, 0.05, 0.1,
0.2} x moments {4, 8, 16, 32} x SMV {4, 8}, no conditional hidden layer.

Execution: configurations that build the same network form a *bucket* (LR, dropout and the
no-op CSMV vary inside it); a bucket is trained as ONE batched native-engine run, one member per
config (per-member learning rates and dropout rates, ``Engine.set_lr`` / ``Engine.set_dropout``),
so the paper grid's 384 configs are 48 engine runs and the baseline grid's 24 runs of 16. Buckets are assigned to ranks longest-processing-time first (``comm.assign_lpt``) by
``bucket_cost``: the measured per-epoch time of that architecture's 8-member engine on the
600 x 3000 panel (``sweep_costs.json``, written by ``tools/sweep_costs.py`` on an MI355X) or,
for architectures it does not list, an analytic estimate. A bucket that raises marks its
configs failed (metrics NaN) without stopping the sweep; the per-config metric table is
exchanged with one all-gather and every rank ranks the configs identically (best = highest
validation Sharpe of the paper-sign SDF factor by default). Per-rank wall-clocks are reported.
"""
from __future__ import annotations

import argparse
import dataclasses
import itertools
import json
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..config import ModelSpec, default_cli_config
from . import comm
from .ensemble import SPLITS, _init_models, load_batches

GRID = {"HL": (2, 3, 4), "SMV": (4, 8), "CSMV": (16, 32), "CHL": (0, 1), "CHU": (4, 8, 16, 32),
        "LR": (1e-3, 5e-4, 2e-4, 1e-4)}
BASELINE_GRID = {"HL": (2, 3, 4), "SMV": (4, 8), "DROPOUT": (0.0, 0.05, 0.1, 0.2), "K": (4, 8, 16, 32),
                 "LR": (1e-3, 5e-4, 2e-4, 1e-4)}
COSTS_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sweep_costs.json")
METRICS = ("ok", "valid_sharpe", "test_sharpe", "train_sharpe", "valid_loss", "test_loss", "wall_s")


def paper_grid(M: int, F: int, grid: Dict = GRID, dropout: float = 0.05,
               chu: str = "both") -> List[Tuple[Dict, float, Dict]]:
    """[(model config, lr, grid point)] in a fixed order (384 entries for the paper grid).
    ``chu``: "both" -- CHU is the moment count and the conditional hidden width; "hidden" --
    8 moments, CHU only the conditional hidden width."""
    keys = list(grid)
    out = []
    for vals in itertools.product(*(grid[k] for k in keys)):
        pt = dict(zip(keys, vals))
        k = pt["CHU"] if chu == "both" else 8
        cfg = default_cli_config(M, F, hidden_dim=[64] * pt["HL"], rnn_dim=[pt["SMV"]],
                                 num_moments=k, dropout=dropout,
                                 hidden_dim_moment=[pt["CHU"]] * pt["CHL"], rnn_dim_moment=[pt["CSMV"]])
        out.append((cfg, float(pt["LR"]), pt))
    return out


def baseline_grid(M: int, F: int, grid: Dict = BASELINE_GRID) -> List[Tuple[Dict, float, Dict]]:
    """BASELINE.json config 4's axes (hidden_dim x lr x dropout x num_moments, x SMV): 384."""
    keys = list(grid)
    out = []
    for vals in itertools.product(*(grid[k] for k in keys)):
        pt = dict(zip(keys, vals))
        cfg = default_cli_config(M, F, hidden_dim=[64] * pt["HL"], rnn_dim=[pt["SMV"]],
                                 num_moments=pt["K"], dropout=pt["DROPOUT"])
        out.append((cfg, float(pt["LR"]), pt))
    return out


def arch_key(spec: ModelSpec) -> str:
    """Cost-table key of an architecture: SDF depth, LSTM width, moment hidden widths, moments."""
    return f"HL{len(spec.hidden)}-H{spec.rnn_hidden}-CH{'x'.join(map(str, spec.moment_hidden)) or 0}-K{spec.num_moments}"


def _load_costs() -> Dict[str, float]:
    try:
        with open(COSTS_FILE) as fh:
            return {k: float(v) for k, v in json.load(fh)["ms_per_epoch"].items()}
    except (OSError, ValueError, KeyError):
        return {}


def bucket_cost(spec: ModelSpec, members: int = 8, table: Optional[Dict[str, float]] = None) -> float:
    """Relative cost of training one bucket (``members`` configs batched in one engine).

    The measured per-epoch time of the architecture (``sweep_costs.json``) when listed, else an
    analytic per-epoch estimate in the same unit (ms at 600 x 3000 x 46, 8 members): a fixed
    serial part (LSTM recurrence, loss passes, launches), plus tower work that grows with the
    SDF depth (the HL >= 3 backward kernels run with spilled registers) and with the padded
    moment-tower width and depth."""
    table = _load_costs() if table is None else table
    key = arch_key(spec)
    if key in table:
        return table[key] * members / 8.0
    hl = len(spec.hidden)
    wm = max([spec.num_moments] + list(spec.moment_hidden))
    wmb = 1 if wm <= 16 else (2 if wm <= 32 else 4)
    sdf = 0.45 * hl * (1.6 if hl >= 3 else 1.0)
    mom = 0.12 * wmb * (1 + len(spec.moment_hidden))
    serial = 0.5 + (0.1 if spec.rnn_hidden > 4 else 0.0)
    return (serial + (sdf + mom) * members / 8.0)


def buckets(entries: Sequence[Tuple[Dict, float, Dict]]) -> List[List[int]]:
    """Group config indices that build the same network (one batched engine run each).

    The key is the ``ModelSpec`` the config produces without its dropout rate, so configs that
    differ only in lr, in dropout (a per-member rate of the batched engine) or in keys the model
    ignores -- CSMV (``num_units_rnn_moment``) is such a no-op in the reference
    (`/root/reference/src/model.py:309-311`) -- share a bucket: the paper grid's 384 configs
    are 48 architectures x 8 members, the baseline grid's 24 x 16.

    With hidden moment layers the engine's structural switch "the train split's moments can be
    cached in phase 3" depends on whether ANY batched member drops out (their keep masks change
    the moments), so there the key also carries ``dropout > 0``: a p = 0 member then trains in a
    bucket of p = 0 members, exactly as it would alone."""
    groups: Dict[object, List[int]] = {}
    for i, (cfg, _, _) in enumerate(entries):
        spec = ModelSpec.from_config(cfg)
        key = (dataclasses.replace(spec, dropout=0.0), len(spec.moment_hidden) > 0 and spec.dropout > 0)
        groups.setdefault(key, []).append(i)
    return list(groups.values())


def _sharpe_unbiased(p: np.ndarray) -> float:
    sd = float(np.std(p, ddof=1)) if len(p) > 1 else 0.0
    return 0.0 if sd < 1e-8 else float(np.mean(p) / sd)


def run_bucket(entries, idx: List[int], batches: Dict[str, Dict], device: torch.device, epochs, ignore_epoch,
               seed: int, selection_sign: float, models=None) -> np.ndarray:
    """Train one architecture bucket; returns [len(idx), len(METRICS)]. ``models``: the members'
    initial modules (built by the caller when buckets run concurrently)."""
    out = np.full((len(idx), len(METRICS)), np.nan)
    out[:, 0] = 0.0
    cfg = entries[idx[0]][0]
    lrs = [entries[i][1] for i in idx]
    drops = [float(entries[i][0].get("dropout", 0.05)) for i in idx]
    t0 = time.time()
    n1, n2, n3 = epochs
    tr, va, te = (batches[s] for s in SPLITS)
    if device.type == "cuda":
        from ..engine.runner import train_3phase_gpu
        if models is None:
            models = _init_models(cfg, [seed] * len(idx))
        ms, hs = train_3phase_gpu(cfg, tr, va, te, device=device, num_epochs_unc=n1, num_epochs_moment=n2,
                                  num_epochs=n3, lr=lrs[0], print_freq=10 ** 9, ignore_epoch=ignore_epoch,
                                  selection_sign=selection_sign, verbose=False, models=models,
                                  seeds=[seed + 17 * k for k in range(len(idx))], lrs=lrs, dropouts=drops,
                                  final_weights_device=True)      # (metrics only: no [T, N] host copies)
        if len(idx) == 1:
            ms = [ms]
        tm = dict(train_3phase_gpu.last_timers.total)
        tm["graph-capture"] = train_3phase_gpu.last_capture_s
        run_bucket.last_timing = tm
        finals = [m.engine_final_eval for m in ms]
        for k, fe in enumerate(finals):
            out[k, 1:6] = [fe[1]["sharpe"], fe[2]["sharpe"], fe[0]["sharpe"], fe[1]["loss"], fe[2]["loss"]]
    else:
        from ..train.trainer import evaluate, train_3phase
        for k, lr in enumerate(lrs):
            torch.manual_seed(seed)
            model, _ = train_3phase(entries[idx[k]][0], tr, va, te, device=torch.device("cpu"), num_epochs_unc=n1,
                                    num_epochs_moment=n2, num_epochs=n3, lr=lr, print_freq=10 ** 9,
                                    ignore_epoch=ignore_epoch, selection_sign=selection_sign, verbose=False)
            ev = [evaluate(model, b, "cpu") for b in (tr, va, te)]
            out[k, 1:6] = [ev[1]["sharpe"], ev[2]["sharpe"], ev[0]["sharpe"], ev[1]["loss"], ev[2]["loss"]]
    out[:, 0] = 1.0
    out[:, 6] = time.time() - t0
    return out


def plan(entries, world: int, balance: str = "lpt", dist: Optional[comm.Dist] = None
         ) -> Tuple[List[List[int]], List[List[int]], List[float]]:
    """(buckets, per-rank bucket lists, per-bucket cost). ``balance``: "lpt" (cost-aware,
    default) or "round_robin".

    With an active process group the ranks plan from RANK 0's cost vector (one all-gather of
    the [n_buckets] costs): every rank reads ``sweep_costs.json`` from its own filesystem, and
    LPT is only consistent when all ranks see the same costs -- a stale or missing table on one
    node would otherwise give ranks different ``owners`` and misplace rows in the result
    all-gather without an error."""
    bks = buckets(entries)
    table = _load_costs()
    costs = [bucket_cost(ModelSpec.from_config(entries[b[0]][0]), len(b), table) for b in bks]
    if dist is not None and dist.active:
        allc = comm.all_gather_rows(dist, np.asarray([costs], np.float64), dist.world, [dist.rank])
        if not np.array_equal(allc[0], allc[dist.rank]):
            print(f"[sweep rank {dist.rank}] bucket costs differ from rank 0's "
                  f"(sweep_costs.json out of sync?); planning with rank 0's", flush=True)
        costs = [float(c) for c in allc[0]]
    if balance == "lpt":
        owners = comm.assign_lpt(costs, world)
    else:
        owners = [comm.shard(len(bks), r, world) for r in range(world)]
    return bks, owners, costs


def run_sweep(batches: Dict[str, Dict], entries, dist: Optional[comm.Dist] = None, epochs=(256, 64, 1024),
              ignore_epoch: int = 64, seed: int = 42, selection_sign: float = 1.0,
              rank_sign: float = -1.0, fail_buckets: Sequence[int] = (), verbose: bool = False,
              concurrency: Optional[int] = None, balance: str = "lpt") -> Dict:
    d = dist or comm.Dist()
    bks, owners, costs = plan(entries, d.world, balance, d)
    mine = owners[d.rank]
    local = {}
    errors = {}
    t_start = time.time()
    if concurrency is None:
        # Buckets of one rank can train concurrently (one engine per thread, graphs replayed
        # from several host threads). On the paper grid one 8-member bucket already fills the
        # GPU: 2 and 3 concurrent buckets measured 247.8 s and 246.7 s vs 251 s serial, so 1.
        concurrency = int(os.environ.get("DLAP_SWEEP_CONCURRENCY", "1")) if d.device.type == "cuda" else 1
    # initial modules built up front in bucket order (torch's global RNG is not per thread)
    inits = {b: (_init_models(entries[bks[b][0]][0], [seed] * len(bks[b])) if d.device.type == "cuda" else None)
             for b in mine}
    done = [0]
    timing: Dict[str, float] = {}

    def one(b):
        try:
            if d.device.type == "cuda":
                # HIP's current device is per host thread: a pool thread starts on device 0
                torch.cuda.set_device(d.device)
            if b in set(fail_buckets):
                raise RuntimeError("injected failure")
            res = run_bucket(entries, bks[b], batches, d.device, epochs, ignore_epoch, seed, selection_sign,
                             models=inits[b])
            tm = getattr(run_bucket, "last_timing", None) or {}
            for k, v in tm.items():            # this rank's time per stage, summed over its buckets
                timing[k] = timing.get(k, 0.0) + v
            done[0] += 1
            if verbose:
                print(f"[sweep rank {d.rank}] bucket {done[0]}/{len(mine)} ({len(bks[b])} configs) "
                      f"done, {time.time() - t_start:.1f} s", flush=True)
            return b, res, None
        except Exception as e:  # isolate: this bucket's configs report NaN
            z = np.full((len(bks[b]), len(METRICS)), np.nan)
            z[:, 0] = 0.0
            return b, z, f"{type(e).__name__}: {e}"

    if concurrency > 1 and len(mine) > 1:
        # several architecture engines share the GPU: each engine's epoch graphs are latency-
        # bound, so independent buckets fill each other's idle CUs (the engine releases the GIL)
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=concurrency) as pool:
            results = list(pool.map(one, mine))
    else:
        results = [one(b) for b in mine]
    for b, res, err in results:
        local[b] = res
        if err:
            errors[b] = err
    # one all-gather of a fixed-size table per rank: rows = configs in bucket order
    width = max(len(x) for x in bks)
    tab = np.full((len(mine), width, len(METRICS)), np.nan)
    for k, b in enumerate(mine):
        tab[k, :len(bks[b])] = local[b]
    allb = comm.all_gather_rows(d, tab, len(bks), mine, owners)
    table = np.full((len(entries), len(METRICS)), np.nan)
    for b, ids in enumerate(bks):
        table[ids] = allb[b, :len(ids)]
    ok = table[:, 0] > 0.5
    score = np.where(ok, rank_sign * table[:, 1], -np.inf)
    best = int(np.argmax(score)) if ok.any() else -1
    walls = comm.all_gather_rows(d, np.array([[time.time() - t_start]]), d.world, [d.rank])[:, 0]
    loads = [float(sum(costs[b] for b in o)) for o in owners]
    return {"n_configs": len(entries), "n_buckets": len(bks), "n_ok": int(ok.sum()),
            "world_size": d.world, "wall_s": float(walls.max()),
            "wall_s_per_rank": [float(w) for w in walls], "balance": balance,
            "predicted_load_per_rank": loads,
            "predicted_imbalance": (max(loads) / min(loads)) if min(loads) > 0 else float("inf"),
            "failed": [int(i) for i in np.where(~ok)[0]], "best_index": best,
            "best_point": entries[best][2] if best >= 0 else None,
            "best_valid_sharpe": float(table[best, 1]) if best >= 0 else None,
            "best_test_sharpe": float(table[best, 2]) if best >= 0 else None,
            "table": table, "metrics": METRICS, "errors_local": errors,
            "stage_s_local": {k: round(v, 3) for k, v in timing.items()}}


def main(argv=None):
    p = argparse.ArgumentParser(description="384-config hyperparameter sweep over the GPUs of one node")
    p.add_argument("--data_dir", type=str, default=None)
    p.add_argument("--synthetic", type=int, nargs=6, default=None,
                   metavar=("T_TRAIN", "T_VALID", "T_TEST", "N", "F", "M"))
    p.add_argument("--data_seed", type=int, default=0)
    p.add_argument("--epochs_unc", type=int, default=256)
    p.add_argument("--epochs_moment", type=int, default=64)
    p.add_argument("--epochs", type=int, default=1024)
    p.add_argument("--ignore_epoch", type=int, default=64)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--limit", type=int, default=None, help="only the first K grid points")
    p.add_argument("--out", type=str, default=None, help="write the metric table (.npz) here")
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--grid", choices=["paper", "baseline"], default="paper",
                   help="paper: Table A.VIII axes; baseline: BASELINE.json config 4 axes")
    p.add_argument("--chu", choices=["both", "hidden"], default="both",
                   help="paper grid: CHU sets the moment count and hidden width (both) or the hidden width only")
    p.add_argument("--balance", choices=["lpt", "round_robin"], default="lpt")
    a = p.parse_args(argv)
    if not a.synthetic and not a.data_dir:
        p.error("--data_dir or --synthetic is required")
    d = comm.init(use_gpu=not a.cpu and torch.cuda.is_available())
    batches = load_batches(a, d)
    M = batches["train"]["macro_features"].shape[-1] if "macro_features" in batches["train"] else 0
    F = batches["train"]["individual_features"].shape[-1]
    entries = paper_grid(M, F, chu=a.chu) if a.grid == "paper" else baseline_grid(M, F)
    if a.limit:
        entries = entries[:a.limit]
    res = run_sweep(batches, entries, d, (a.epochs_unc, a.epochs_moment, a.epochs), a.ignore_epoch, a.seed,
                    verbose=True, balance=a.balance)
    if d.is_main:
        if a.out:
            np.savez(a.out, table=res["table"], metrics=np.array(METRICS))
        print(json.dumps({k: v for k, v in res.items() if k not in ("table",)}, default=str))
    comm.shutdown(d)
    return res


if __name__ == "__main__":
    main()
