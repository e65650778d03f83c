"""Record the CPU side of the bf16 parity test: the reference-semantics CPU trainer (fp32,
torch dropout) on the shipped synthetic panel (120/30/60 x 500 x 46, M = 8, regenerated
bit-exactly), the 9 paper seeds, the full 256/64/1024 schedule. Per seed: paper-sign individual
test Sharpe of the selected model and the phase-1 / phase-3 best epochs; plus the ensemble.

    python tools/cpu_parity_record.py [--procs 4] [--out tests/fixtures/cpu_parity_record.json]
    python tools/cpu_parity_record.py --dropout 0 --out tests/fixtures/cpu_parity_record_p0.json

``--dropout 0`` makes the run deterministic (no dropout RNG on either executor), so the GPU test
can compare seed by seed: selected epochs and test Sharpe isolate the bf16 effect.
"""
import argparse
import json
import os
import sys
import tempfile
import time
from multiprocessing import get_context

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _generate(d):
    from deeplearninginassetpricing_paperreplication_amd.data import synthetic as syn
    syn.generate_all_splits(d, 120, 30, 60, n_stocks=500, n_features=46, n_macro=8, seed=42, quiet=True)


def _panel(d):
    from deeplearninginassetpricing_paperreplication_amd.data.dataset import load_splits
    return [ds.get_full_batch() for ds in load_splits(d)]


def _one(args):
    seed, threads, d, dropout = args
    import numpy as np
    import torch
    torch.set_num_threads(threads)
    from deeplearninginassetpricing_paperreplication_amd.analysis.parity import SCHEDULE, best_epochs
    from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
    from deeplearninginassetpricing_paperreplication_amd.train.trainer import evaluate, train_3phase
    tr, va, te = _panel(d)
    cfg = default_cli_config(8, 46)
    if dropout is not None:
        cfg["dropout"] = float(dropout)
    torch.manual_seed(seed)
    np.random.seed(seed)
    t0 = time.time()
    model, hist = train_3phase(cfg, tr, va, te, device=torch.device("cpu"), num_epochs_unc=SCHEDULE[0],
                               num_epochs_moment=SCHEDULE[1], num_epochs=SCHEDULE[2], print_freq=10 ** 9,
                               verbose=False)
    w = {sp: evaluate(model, b, "cpu")["weights"].numpy() for sp, b in zip(("train", "valid", "test"), (tr, va, te))}
    be = list(best_epochs(hist, SCHEDULE[0]))
    vs = hist["valid_sharpe"]
    vbest = [float(vs[be[0]]) if be[0] >= 0 else None,
             float(vs[SCHEDULE[0] + be[1]]) if be[1] >= 0 else None]
    return seed, w, be, time.time() - t0, vbest


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--dropout", type=float, default=None, help="override the config's dropout (0: deterministic)")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "fixtures", "cpu_parity_record.json"))
    a = ap.parse_args()
    import numpy as np
    from deeplearninginassetpricing_paperreplication_amd.analysis.parity import SEEDS, SCHEDULE, summarize
    from deeplearninginassetpricing_paperreplication_amd.analysis.portfolio import ensemble_sharpes
    threads = max(1, (os.cpu_count() or 8) // a.procs)
    with tempfile.TemporaryDirectory() as d:
        _generate(d)
        t0 = time.time()
        with get_context("spawn").Pool(a.procs) as pool:
            res = sorted(pool.map(_one, [(s, threads, d, a.dropout) for s in SEEDS]), key=lambda r: SEEDS.index(r[0]))
        wall = time.time() - t0
        tr, va, te = _panel(d)
    nb = {sp: {"returns": b["returns"].numpy(), "mask": b["mask"].numpy()}
          for sp, b in zip(("train", "valid", "test"), (tr, va, te))}
    ens = ensemble_sharpes([r[1] for r in res], nb)
    rec = {"panel": "shipped synthetic 120/30/60 x 500 x 46, M=8 (generate_all_splits seed 42)",
           "schedule": list(SCHEDULE), "seeds": list(SEEDS),
           "executor": "CPU trainer (reference semantics, fp32, torch dropout)",
           "dropout": a.dropout if a.dropout is not None else 0.05,
           "valid_sharpes_at_best": [r[4] for r in res],
           "wall_s": wall, "seconds_per_seed": [r[3] for r in res],
           "individual_test_sharpes": [float(x) for x in ens["individual_sharpes"]],
           "best_epochs": [r[2] for r in res],
           "ensemble": {k: float(ens[k]) for k in ("train_sharpe", "valid_sharpe", "test_sharpe")}}
    rec["summary"] = summarize(rec["individual_test_sharpes"], rec["best_epochs"])
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec["summary"]))


if __name__ == "__main__":
    main()
