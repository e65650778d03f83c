"""bf16 statistical parity on the current tree: the 9 paper seeds
on the shipped synthetic panel (120/30/60 x 500 x 46, M = 8, regenerated bit-exactly), full
256/64/1024 schedule, batched on one MI355X, against the CPU trainer's record
(``tests/fixtures/cpu_parity_record.json``, ``tools/cpu_parity_record.py``: fp32, torch dropout).
The dropout streams differ, so the check is statistical: the mean paper-sign individual test
Sharpe and the mean phase-1 / phase-3 best-epoch indices (the reference's selection rule,
`/root/reference/src/train.py:268,378`) agree within 3 standard errors of the difference."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "cpu_parity_record.json")
# dropout 0: both executors are deterministic, so the comparison is per seed
FIXTURE_P0 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "cpu_parity_record_p0.json")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_summary(name, rec):
    """GPU-side records land in gpurun_out/ (merged back from the GPU box; committed copies live in
    profiles/)."""
    out = os.environ.get("DLAP_PARITY_OUT", os.path.join(ROOT, "gpurun_out"))
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, name), "w") as fh:
        json.dump(rec, fh, indent=1)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    native.load(required=True)


def _train_gpu(tmp_path, dropout=None, precision="bf16"):
    from deeplearninginassetpricing_paperreplication_amd.analysis import parity
    from deeplearninginassetpricing_paperreplication_amd.analysis.portfolio import ensemble_sharpes
    from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
    from deeplearninginassetpricing_paperreplication_amd.data import synthetic as syn
    from deeplearninginassetpricing_paperreplication_amd.data.dataset import load_splits
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import train_3phase_gpu
    from deeplearninginassetpricing_paperreplication_amd.parallel.ensemble import _init_models
    d = tmp_path / precision
    d.mkdir(exist_ok=True)
    syn.generate_all_splits(str(d), 120, 30, 60, n_stocks=500, n_features=46, n_macro=8, seed=42, quiet=True)
    tr, va, te = (ds.get_full_batch() for ds in load_splits(str(d)))
    cfg = default_cli_config(8, 46) if dropout is None else default_cli_config(8, 46, dropout=dropout)
    seeds = list(parity.SEEDS)
    n1, n2, n3 = parity.SCHEDULE
    models, hists = train_3phase_gpu(cfg, tr, va, te, num_epochs_unc=n1, num_epochs_moment=n2, num_epochs=n3,
                                     print_freq=10 ** 9, ignore_epoch=parity.IGNORE_EPOCH, verbose=False,
                                     models=_init_models(cfg, seeds), seeds=seeds, precision=precision)
    w = [{sp: m.engine_final_eval[k]["weights"].numpy() for k, sp in enumerate(("train", "valid", "test"))}
         for m in models]
    nb = {sp: {"returns": b["returns"].numpy(), "mask": b["mask"].numpy()}
          for sp, b in zip(("train", "valid", "test"), (tr, va, te))}
    ens = ensemble_sharpes(w, nb)
    best = [parity.best_epochs(h, n1) for h in hists]
    vbest = [[float(h["valid_sharpe"][b[0]]) if b[0] >= 0 else None,
              float(h["valid_sharpe"][n1 + b[1]]) if b[1] >= 0 else None] for h, b in zip(hists, best)]
    return seeds, ens, best, vbest


def _per_seed(seeds, ens, best, vbest, cpu):
    rows = []
    for k, s in enumerate(seeds):
        rows.append({"seed": s, "best": list(best[k]), "cpu_best": list(cpu["best_epochs"][k]),
                     "test_sharpe": float(ens["individual_sharpes"][k]),
                     "cpu_test_sharpe": float(cpu["individual_test_sharpes"][k]),
                     "best_valid_sharpe": vbest[k], "cpu_best_valid_sharpe": cpu["valid_sharpes_at_best"][k]})
    return rows


def test_bf16_engine_matches_deterministic_cpu_record_per_seed(tmp_path):
    """Dropout 0 (no RNG on either side): the bf16 engine against the fp32 CPU trainer seed by
    seed, with the fp32 engine (`--precision fp32`, the reference's arithmetic) as the control.

    Over 1344 epochs the trajectories are chaotic: any rounding difference -- fp32 GPU reduction
    orders as much as bf16 GEMM operands -- moves the argmax of the noisy validation-Sharpe curve
    (the reference's selection rule, `/root/reference/src/train.py:268,378`), so the selected
    epoch is not a stable observable (the fp32 control shows the same drift). What the selection
    produces is: per seed the selected model's test Sharpe and the best validation Sharpe of each
    phase must match the CPU record within 0.02, and the 9-seed ensemble's test Sharpe within
    0.005 (`/root/reference/src/evaluate_ensemble.py:137-166`)."""
    from deeplearninginassetpricing_paperreplication_amd.analysis import parity
    with open(FIXTURE_P0) as fh:
        cpu = json.load(fh)
    assert cpu["dropout"] == 0.0
    rec = {"panel": cpu["panel"], "dropout": 0.0, "schedule": cpu["schedule"],
           "cpu_ensemble_test_sharpe": cpu["ensemble"]["test_sharpe"]}
    for prec in ("bf16", "fp32"):
        seeds, ens, best, vbest = _train_gpu(tmp_path, dropout=0.0, precision=prec)
        assert cpu["seeds"] == seeds and cpu["schedule"] == list(parity.SCHEDULE)
        rows = _per_seed(seeds, ens, best, vbest, cpu)
        rec[prec] = {"per_seed": rows, "ensemble_test_sharpe": float(ens["test_sharpe"]),
                     "phase1_same_epoch": sum(r["best"][0] == r["cpu_best"][0] for r in rows),
                     "phase3_same_epoch": sum(r["best"][1] == r["cpu_best"][1] for r in rows),
                     "max_abs_dtest_sharpe": max(abs(r["test_sharpe"] - r["cpu_test_sharpe"]) for r in rows),
                     "max_abs_dbest_valid_sharpe": max(abs(a - b) for r in rows
                                                        for a, b in zip(r["best_valid_sharpe"], r["cpu_best_valid_sharpe"])
                                                        if a is not None and b is not None)}
    _write_summary("r5_parity_p0_gpu.json", rec)
    print("\n" + json.dumps({p: {k: v for k, v in rec[p].items() if k != "per_seed"} for p in ("bf16", "fp32")}))
    for prec in ("bf16", "fp32"):
        r = rec[prec]
        assert r["max_abs_dtest_sharpe"] < 0.02, (prec, r)
        assert r["max_abs_dbest_valid_sharpe"] < 0.02, (prec, r)
        assert abs(r["ensemble_test_sharpe"] - cpu["ensemble"]["test_sharpe"]) < 0.005, (prec, r)


def test_bf16_engine_matches_cpu_record_statistically(tmp_path):
    from deeplearninginassetpricing_paperreplication_amd.analysis import parity
    with open(FIXTURE) as fh:
        cpu = json.load(fh)
    seeds, ens, best, _ = _train_gpu(tmp_path)
    gpu = parity.summarize(ens["individual_sharpes"], best)
    corr = float(np.corrcoef(ens["individual_sharpes"], cpu["individual_test_sharpes"])[0, 1])
    print(f"\nGPU {json.dumps(gpu)}\nCPU {json.dumps(cpu['summary'])}\nper-seed test-Sharpe correlation {corr:.3f}, "
          f"ensemble test Sharpe GPU {ens['test_sharpe']:.4f} CPU {cpu['ensemble']['test_sharpe']:.4f}")
    _write_summary("r5_parity_dropout_gpu.json", {"gpu": gpu, "cpu": cpu["summary"], "per_seed_correlation": corr,
                                                  "gpu_individual_test_sharpes": [float(x) for x in ens["individual_sharpes"]],
                                                  "gpu_best_epochs": [list(b) for b in best],
                                                  "ensemble_test_sharpe": {"gpu": float(ens["test_sharpe"]),
                                                                           "cpu": cpu["ensemble"]["test_sharpe"]}})
    assert cpu["seeds"] == seeds and cpu["schedule"] == list(parity.SCHEDULE)
    for key in ("test_sharpe", "best_p1", "best_p3"):
        assert parity.within_se(gpu, cpu["summary"], key), (key, gpu, cpu["summary"])
