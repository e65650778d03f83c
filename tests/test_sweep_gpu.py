"""The hyperparameter sweep (BASELINE config 4, `parallel/sweep.py`) on a real MI355X: a 3-bucket
slice of the paper grid -- SDF depth 2 / 3 / 4 and both LSTM widths -- through ``run_sweep`` with a
short schedule. Every bucket trains as ONE batched engine run (a member per learning rate), so each
member's metrics must equal the same configuration trained alone, bit for bit (the engine's batch
invariance: the tower partitions depend on the panel only). Reference motivation:
`/root/reference/README.md:205-207`."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EPOCHS = (3, 2, 3)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    native.load(required=True)


def test_sweep_slice_members_equal_solo_runs():
    sys.path.insert(0, ROOT)
    from bench import make_panel
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import train_3phase_gpu
    from deeplearninginassetpricing_paperreplication_amd.parallel import comm, sweep
    tr, va, te = make_panel(seed=5, device="cuda", keep_on_device=True)
    batches = {"train": tr, "valid": va, "test": te}
    grid = sweep.paper_grid(178, 46)
    bks = sweep.buckets(grid)
    pick = []
    for hl, smv in ((2, 4), (3, 8), (4, 4)):      # one bucket per depth, both LSTM widths
        b = next(b for b in bks if grid[b[0]][2]["HL"] == hl and grid[b[0]][2]["SMV"] == smv)
        pick.append(b[:4])                          # 4 learning rates of the bucket
    entries = [grid[i] for b in pick for i in b]
    d = comm.Dist(device=torch.device("cuda", 0))
    res = sweep.run_sweep(batches, entries, d, epochs=EPOCHS, ignore_epoch=0, seed=42)
    assert res["n_buckets"] == 3 and res["n_ok"] == len(entries), res["errors_local"]
    table = res["table"]
    assert np.isfinite(table[:, 1:6]).all()
    # member k of each bucket alone: its seed (seed + 17 k), lr, dropout and the shared init
    for b in sweep.buckets(entries):
        k = len(b) - 1                              # the last member (highest batch position)
        cfg, lr, _ = entries[b[k]]
        model = sweep._init_models(cfg, [42])[0]
        m, _ = train_3phase_gpu(cfg, tr, va, te, device="cuda", num_epochs_unc=EPOCHS[0],
                                num_epochs_moment=EPOCHS[1], num_epochs=EPOCHS[2], lr=lr, print_freq=10 ** 9,
                                ignore_epoch=0, verbose=False, models=[model], seeds=[42 + 17 * k],
                                lrs=[lr], dropouts=[float(cfg.get("dropout", 0.05))])
        fe = m.engine_final_eval
        solo = [fe[1]["sharpe"], fe[2]["sharpe"], fe[0]["sharpe"], fe[1]["loss"], fe[2]["loss"]]
        np.testing.assert_array_equal(np.asarray(solo), table[b[k], 1:6])
