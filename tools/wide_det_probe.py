"""Determinism probe of the wide layer-0 path: two identical wide engines, 4 / 2 / 4 epochs;
prints which history columns differ (and by how much) and whether the parameters are equal."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from test_engine_gpu import _batch, _engine  # noqa: E402

from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.engine.runner import HIST  # noqa: E402

cfg = default_cli_config(8, 46)
data = _batch()
runs = []
for _ in range(3):
    eng, _ = _engine(cfg, data=data)
    for ph, n in ((1, 4), (2, 2), (3, 4)):
        eng.eng.begin_phase(ph)
        eng.run(ph, n, 1e-3, 1, 1.0, True)
    eng.eng.sync()
    runs.append((np.nan_to_num(eng.history_rows(0)), eng.params(0)))
names = {v: k for k, v in HIST.items()}
for k in (1, 2):
    h0, p0 = runs[0]
    h1, p1 = runs[k]
    print(f"run0 vs run{k}: params equal {np.array_equal(p0, p1)}")
    d = np.argwhere(h0 != h1)
    for c in sorted(set(d[:, 1])):
        rows = d[d[:, 1] == c][:, 0]
        print(f"   {names.get(c, c)}: epochs {rows.tolist()} max|d| {np.abs(h0[:, c] - h1[:, c]).max():.3e}")
