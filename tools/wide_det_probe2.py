"""Bitwise repeatability of the wide-path training step on a panel with many tiles per wave
(T=48, N=20000): the same model's phase-3 backward (streamed forward -> one-pass backward ->
k_wgrad0) on two engines, gradients compared bit for bit; and a 3-epoch run's history twice."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN  # noqa: E402

ret, feats, mask, mac = generate_panel_fast(48, 20000, 46, 8, seed=3)
mac = (mac - mac.mean(0)) / (mac.std(0, unbiased=False) + 1e-8)
b = {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}
cfg = default_cli_config(8, 46, dropout=0.05)
out = []
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    eng = GANEngine(AssetPricingGAN(cfg).spec, 1, max_epochs=8)
    assert int(eng.desc["tbwd"]) == 1
    eng.set_data(b, b, b)
    torch.manual_seed(100)
    eng.set_model(0, AssetPricingGAN(cfg), 11)
    eng.eng.backward_only(3)
    g = eng.eng.get_grads(0).copy()
    eng.eng.begin_phase(3)
    eng.run(3, 3, 1e-3, 0, 1.0, True)
    eng.eng.sync()
    out.append((g, np.nan_to_num(eng.history_rows(0)), eng.params(0)))
from deeplearninginassetpricing_paperreplication_amd.engine.runner import HIST  # noqa: E402
names = {v: k for k, v in HIST.items()}
d = np.argwhere(out[0][1] != out[1][1])
print("differing history entries (epoch, column):", sorted({int(r) for r, c in d}), sorted({names.get(int(c), int(c)) for r, c in d})[:4],
      "max|d|", float(np.abs(out[0][1] - out[1][1]).max()))
print("rows", int(mask.sum()), "grads bitwise equal", np.array_equal(out[0][0], out[1][0]),
      "history equal", np.array_equal(out[0][1], out[1][1]), "params equal", np.array_equal(out[0][2], out[1][2]))

for i in range(2, len(out)):
    print(f"engine 1 vs engine {i + 1}: history equal", np.array_equal(out[1][1], out[i][1]),
          "| engine 0 vs engine", i + 1, np.array_equal(out[0][1], out[i][1]))
