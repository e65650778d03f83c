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


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    native.load(required=True)


def test_bf16_engine_matches_cpu_record_statistically(tmp_path):
    from deeplearninginassetpricing_paperreplication_amd.analysis import parity
    from deeplearninginassetpricing_paperreplication_amd.analysis.portfolio import ensemble_sharpes
    from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
    from deeplearninginassetpricing_paperreplication_amd.data import synthetic as syn
    from deeplearninginassetpricing_paperreplication_amd.data.dataset import load_splits
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import train_3phase_gpu
    from deeplearninginassetpricing_paperreplication_amd.parallel.ensemble import _init_models
    with open(FIXTURE) as fh:
        cpu = json.load(fh)
    syn.generate_all_splits(str(tmp_path), 120, 30, 60, n_stocks=500, n_features=46, n_macro=8, seed=42, quiet=True)
    tr, va, te = (ds.get_full_batch() for ds in load_splits(str(tmp_path)))
    cfg = default_cli_config(8, 46)
    seeds = list(parity.SEEDS)
    n1, n2, n3 = parity.SCHEDULE
    models, hists = train_3phase_gpu(cfg, tr, va, te, num_epochs_unc=n1, num_epochs_moment=n2, num_epochs=n3,
                                     print_freq=10 ** 9, ignore_epoch=parity.IGNORE_EPOCH, verbose=False,
                                     models=_init_models(cfg, seeds), seeds=seeds)
    w = [{sp: m.engine_final_eval[k]["weights"].numpy() for k, sp in enumerate(("train", "valid", "test"))}
         for m in models]
    nb = {sp: {"returns": b["returns"].numpy(), "mask": b["mask"].numpy()}
          for sp, b in zip(("train", "valid", "test"), (tr, va, te))}
    ens = ensemble_sharpes(w, nb)
    best = [parity.best_epochs(h, n1) for h in hists]
    gpu = parity.summarize(ens["individual_sharpes"], best)
    corr = float(np.corrcoef(ens["individual_sharpes"], cpu["individual_test_sharpes"])[0, 1])
    print(f"\nGPU {json.dumps(gpu)}\nCPU {json.dumps(cpu['summary'])}\nper-seed test-Sharpe correlation {corr:.3f}, "
          f"ensemble test Sharpe GPU {ens['test_sharpe']:.4f} CPU {cpu['ensemble']['test_sharpe']:.4f}")
    assert cpu["seeds"] == seeds and cpu["schedule"] == list(parity.SCHEDULE)
    for key in ("test_sharpe", "best_p1", "best_p3"):
        assert parity.within_se(gpu, cpu["summary"], key), (key, gpu, cpu["summary"])
